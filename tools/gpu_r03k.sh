# r03k: per-sender combs (at2v_comb.h) + overlapped launches: GPU suite, bench (full line), 64-sender benches (tables vs
# combs), rocprofv3 kernel trace of the default bench
set -o pipefail
D=gpurun_out/r03k
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1
rc=$?
tail -5 $D/gpu_tests.txt
grep -E "FAILED|ERROR" $D/gpu_tests.txt | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
cat $D/bench.json
for m in 0 1; do
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --senders 64 --sender-cache 1024 --sender-comb $m --pmc-traffic 0 --cpu-sample 0 --e2e 0 > $D/bench_s64_comb$m.json 2>> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
done
grep -ho '"value": [0-9.e+]*' $D/bench_s64_comb*.json
AT2V_SCRATCH_SETS=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --pmc-traffic 0 --cpu-sample 0 --e2e 0 > $D/bench_serial.json 2>> $D/bench.err || exit 1
grep -ho '"value": [0-9.e+]*' $D/bench_serial.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 bench.py --steps 20 --warmup 3 --pmc-traffic 0 --cpu-sample 0 --e2e 0 > $D/bench_under_rocprof.json 2>> $D/bench.err || exit 1
find $D/prof -name '*kernel_stats.csv' -exec cp {} $D/kernel_stats.csv \;
head -4 $D/kernel_stats.csv
exit $rc
