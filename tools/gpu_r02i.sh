# r02i: full bench line (OpenSSL CPU leg added) + rocprofv3 kernel trace of the same bench
set -o pipefail
D=gpurun_out/r02i
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
cat $D/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --pmc-traffic 0 --e2e 0 > $D/bench_under_rocprof.json 2> $D/rocprof.err || { tail -20 $D/rocprof.err; exit 1; }
find $D/prof -name "*kernel_stats.csv" | head -1 | xargs cat | head -4
