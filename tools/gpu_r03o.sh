# r03o: two records per lane in the comb throughput kernel (shared inversion): GPU suite; full bench line with the
# AT2-traffic leg; world-1 torchrun bench (RCCL gathers of overlapped steps); rocprofv3 kernel trace with one scratch set
set -o pipefail
D=gpurun_out/r03o
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1
rc=$?
tail -3 $D/gpu_tests.txt
grep -E "FAILED|ERROR" $D/gpu_tests.txt | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python3 -c "
import json; r=json.load(open('$D/bench.json'))
print('value', r['value'], 'kernel_ms', r['kernel_ms'], 'alone', r['launch_ms_alone'], 'clk', r['effective_clock_ghz'], 'frac', r['roofline']['frac'], 'traffic/verify', r['roofline']['traffic_detail']['bytes_per_verify'] if r['roofline'].get('traffic_detail') else None)
print('at2_traffic', r.get('at2_traffic'))
print('e2e', r.get('e2e_verifies_per_s'), 'cpu', r['cpu_baseline']['value'], r['cpu_baseline'].get('openssl',{}).get('value'))
"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 3 --pmc-traffic 0 --cpu-sample 0 > $D/bench_torchrun_n1.json 2> $D/torchrun.err || { tail -20 $D/torchrun.err; exit 1; }
python3 -c "
import json; r=json.load(open('$D/bench_torchrun_n1.json')); print('torchrun n1', r['value'], r['verdict_match'], r['config']['parallelism'])"
AT2V_SCRATCH_SETS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 20 --warmup 3 --pmc-traffic 0 --cpu-sample 0 --e2e 0 --traffic-leg 0 > $D/bench_serial_under_rocprof.json 2> $D/rocprof.err || { tail -20 $D/rocprof.err; exit 1; }
find $D/prof -name '*kernel_stats.csv' -exec cp {} $D/kernel_stats_serial.csv \;
head -3 $D/kernel_stats_serial.csv | cut -c1-200
grep -o '"launch_ms_alone": [0-9.]*' $D/bench_serial_under_rocprof.json
