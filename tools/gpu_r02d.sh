# r02d: full bench line (PMC traffic + VALU passes, CPU baseline, e2e) and a rocprofv3 kernel trace of the same bench
set -o pipefail
mkdir -p gpurun_out/r02d
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > gpurun_out/r02d/bench.json 2> gpurun_out/r02d/bench.err || { tail -20 gpurun_out/r02d/bench.err; exit 1; }
cat gpurun_out/r02d/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02d/prof -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --pmc-traffic 0 --e2e 0 > gpurun_out/r02d/bench_under_rocprof.json 2> gpurun_out/r02d/rocprof.err || { tail -20 gpurun_out/r02d/rocprof.err; exit 1; }
find gpurun_out/r02d/prof -name "*kernel_stats.csv" | head -1 | xargs cat | head -8
