# r03m: low-latency comb kernel (four-wave split): GPU suite, latency probe with combs, config 5 with combs
set -o pipefail
D=gpurun_out/r03m
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1
rc=$?
tail -4 $D/gpu_tests.txt
grep -E "FAILED|ERROR" $D/gpu_tests.txt | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/latency_probe.py --reps 100 --comb 1 > $D/latency_comb1.json 2> $D/latency.err || { tail -20 $D/latency.err; exit 1; }
python3 -c "
import json
r=json.load(open('$D/latency_comb1.json'))
print({B:{k:round(v['p50_us']) for k,v in x.items()} for B,x in r['sizes'].items()})
"
python3 -c "
import json
r=json.load(open('gpurun_out/config5_comb.json')); print('config5 comb queue p50', [p['queue_p50_us'] for p in r['per_node']], 'e2e p50', r['p50_us'])
"
exit $rc
