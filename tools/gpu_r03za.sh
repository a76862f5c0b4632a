# r03za: the 10-bit comb build: GPU suite, full bench line, rocprofv3 kernel trace with one scratch set, small-batch
# latency with combs
set -o pipefail
D=gpurun_out/r03za
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1
rc=$?
tail -3 $D/gpu_tests.txt
grep -E "FAILED|ERROR" $D/gpu_tests.txt | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
cp gpurun_out/config5_comb.json gpurun_out/config5_eager.json $D/ 2>/dev/null
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || { tail -20 $D/smoke.txt; exit 1; }
tail -2 $D/smoke.txt
timeout -k 10 400 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python3 -c "
import json; r=json.load(open('$D/bench.json'))
print('value', r['value'], 'kernel_ms', r['kernel_ms'], 'alone', r['launch_ms_alone'], 'clk', r['effective_clock_ghz'], 'frac', r['roofline']['frac'], 'valu/verify', r['roofline']['valu_measured']['valu_lane_ops_per_verify'], 'traffic/verify', r['roofline']['traffic_detail']['bytes_per_verify'])
print('at2_traffic', r['at2_traffic']['value'], r['at2_traffic']['verdicts_ok'], 'e2e', r.get('e2e_verifies_per_s'), 'cpu', r['cpu_baseline']['value'])
"
AT2V_SCRATCH_SETS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 20 --warmup 3 --pmc-traffic 0 --cpu-sample 0 --e2e 0 --traffic-leg 0 > $D/bench_serial_under_rocprof.json 2> $D/rocprof.err || { tail -20 $D/rocprof.err; exit 1; }
find $D/prof -name '*kernel_stats.csv' -exec cp {} $D/kernel_stats_serial.csv \;
python3 -c "
import csv
for r in csv.DictReader(open('$D/kernel_stats_serial.csv')):
    if 'verify' in r['Name']: print(r['Name'][:30], r['Calls'], float(r['AverageNs'])/1e6)
"
grep -o '"launch_ms_alone": [0-9.]*' $D/bench_serial_under_rocprof.json
timeout -k 10 300 python3 tools/latency_probe.py --reps 100 --comb 1 > $D/latency_comb1.json 2> $D/latency.err || { tail -20 $D/latency.err; exit 1; }
python3 -c "
import json
r=json.load(open('$D/latency_comb1.json'))
print({B:{k:round(v['p50_us']) for k,v in x.items()} for B,x in r['sizes'].items()})
r=json.load(open('$D/config5_comb.json')); print('config5 comb queue p50', [p['queue_p50_us'] for p in r['per_node']], 'e2e p50', r['p50_us'])
"
