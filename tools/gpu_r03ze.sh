# r03ze: small-batch latency with combs, including the first launch of new keys (comb builds), 10-bit combs
set -o pipefail
D=gpurun_out/r03ze
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/latency_probe.py --reps 100 --comb 1 > $D/latency_comb1.json 2> $D/latency.err || { tail -20 $D/latency.err; exit 1; }
python3 -c "
import json
r=json.load(open('$D/latency_comb1.json'))
for B,x in r['sizes'].items(): print(B, {k:(round(v['p50_us']) if isinstance(v,dict) else round(v)) for k,v in x.items()})
"
