# r02ae: round-2 final build (lattice ping-pong): GPU parity, smoke, full bench line, rocprofv3 kernel trace
set -o pipefail
D=gpurun_out/r02ae
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -30 $D/gpu_tests.txt; exit 1; }
tail -2 $D/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || { tail -20 $D/smoke.txt; exit 1; }
timeout -k 10 600 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
cat $D/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --pmc-traffic 0 --e2e 0 > $D/bench_under_rocprof.json 2> $D/rocprof.err || { tail -20 $D/rocprof.err; exit 1; }
find $D/prof -name "*kernel_stats.csv" | head -1 | xargs cat | head -4
