# r03p: trimmed small-batch comb launches: GPU suite, latency probe with combs, rocprofv3 trace of the probe
set -o pipefail
D=gpurun_out/r03p
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1
rc=$?
tail -3 $D/gpu_tests.txt
grep -E "FAILED|ERROR" $D/gpu_tests.txt | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/latency_probe.py --reps 100 --comb 1 > $D/latency_comb1.json 2> $D/latency.err || { tail -20 $D/latency.err; exit 1; }
python3 -c "
import json
r=json.load(open('$D/latency_comb1.json'))
print({B:{k:round(v['p50_us']) for k,v in x.items()} for B,x in r['sizes'].items()})
r=json.load(open('gpurun_out/config5_comb.json')); print('config5 comb queue p50', [p['queue_p50_us'] for p in r['per_node']], 'e2e p50', r['p50_us'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $D/prof -o run -- python3 tools/latency_probe.py --reps 30 --comb 1 --sizes 20 > $D/latency_under_rocprof.json 2> $D/rocprof.err || { tail -20 $D/rocprof.err; exit 1; }
find $D/prof -name '*kernel_stats.csv' -exec cp {} $D/latency_kernel_stats.csv \;
cut -c1-160 $D/latency_kernel_stats.csv | head -12
