# r03zg: comb builds: a block per new key, 8 lanes per position, for up to 256 new keys per launch, else a wave per key: cache/comb GPU tests, config 5 with
# combs, first-launch latency of new keys
set -o pipefail
D=gpurun_out/r03zg
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cache.py tests/test_gpu_boundary.py -v --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -30 $D/gpu_tests.txt; exit 1; }
tail -2 $D/gpu_tests.txt
timeout -k 10 300 python3 tools/latency_probe.py --reps 100 --comb 1 > $D/latency_comb1.json 2> $D/latency.err || { tail -20 $D/latency.err; exit 1; }
python3 -c "
import json
r=json.load(open('$D/latency_comb1.json'))
for B,x in r['sizes'].items(): print(B, {k:(round(v['p50_us']) if isinstance(v,dict) else round(v)) for k,v in x.items()})
"
