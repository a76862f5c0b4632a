# r03zg: round-3 final build (comb builds: a block per new key, 8 lanes per position, for up to 256 new keys per launch,
# else a wave per key): GPU suite, smoke, full bench line, first-launch latency of new keys
set -o pipefail
D=gpurun_out/r03zg
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -30 $D/gpu_tests.txt; exit 1; }
tail -2 $D/gpu_tests.txt
cp gpurun_out/config5_comb.json $D/ 2>/dev/null
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || { tail -20 $D/smoke.txt; exit 1; }
tail -1 $D/smoke.txt
timeout -k 10 400 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python3 -c "
import json; r=json.load(open('$D/bench.json'))
print('value', r['value'], 'kernel_ms', r['kernel_ms'], 'clk', r['effective_clock_ghz'], 'frac', r['roofline']['frac'])
t=r['at2_traffic']; print('at2_traffic', t['value'], t['verdicts_ok'], 'comb frac', t['roofline']['frac'], 'cpu', r['cpu_baseline']['value'])
r=json.load(open('$D/config5_comb.json')); print('config5 comb queue p50', [p['queue_p50_us'] for p in r['per_node']], 'e2e p50', r['p50_us'])
"
timeout -k 10 300 python3 tools/latency_probe.py --reps 100 --comb 1 > $D/latency_comb1.json 2> $D/latency.err || { tail -20 $D/latency.err; exit 1; }
python3 -c "
import json
r=json.load(open('$D/latency_comb1.json'))
for B,x in r['sizes'].items(): print(B, {k:(round(v['p50_us']) if isinstance(v,dict) else round(v)) for k,v in x.items()})
"
