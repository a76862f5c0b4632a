# r03j: overlapped launches (two scratch sets, two launch streams): GPU suite, bench (full line), bench with one scratch
# set (serial launches) for the A/B, rocprofv3 kernel trace of the bench
set -o pipefail
D=gpurun_out/r03j
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -40 $D/gpu_tests.txt; exit 1; }
tail -3 $D/gpu_tests.txt
timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
cat $D/bench.json
for r in 1 2; do
AT2V_SCRATCH_SETS=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --pmc-traffic 0 --cpu-sample 0 --e2e 0 > $D/bench_serial_$r.json 2>> $D/bench.err || exit 1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --pmc-traffic 0 --cpu-sample 0 --e2e 0 > $D/bench_overlap_$r.json 2>> $D/bench.err || exit 1
done
grep -ho '"value": [0-9.e+]*' $D/bench_serial_*.json $D/bench_overlap_*.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 bench.py --steps 20 --warmup 3 --pmc-traffic 0 --cpu-sample 0 --e2e 0 > $D/bench_under_rocprof.json 2>> $D/bench.err || exit 1
find $D/prof -name '*kernel_stats.csv' -exec cp {} $D/kernel_stats.csv \;
head -5 $D/kernel_stats.csv
