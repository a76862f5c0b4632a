# config 5 with combs and a stream of first-seen senders: queue latency per node at several fresh-sender fractions
# usage (on the GPU box): bash tools/fresh_sweep.sh <tag> [fractions...]
set -o pipefail
D=gpurun_out/${1:-fresh}; shift
mkdir -p $D
for f in ${@:-0.0 0.002 0.005 0.02}; do
  timeout -k 10 200 python3 tools/mininode.py --nodes 4 --rate 20000 --seconds 2 --batch 1024 --delay-us 1000 --eager 1 --comb 1 --fresh-frac $f > $D/mininode_fresh_$f.json 2> $D/mininode_fresh_$f.err || { tail -20 $D/mininode_fresh_$f.err; exit 1; }
  python3 -c "
import json; r=json.loads([l for l in open('$D/mininode_fresh_$f.json') if l.startswith('{')][-1])
print('fresh $f', r['fresh_senders'], 'p50', [p['queue_p50_us'] for p in r['per_node']], 'p99', [p['queue_p99_us'] for p in r['per_node']], 'ok', r['ledgers_identical'], r['all_real_applied'])"
done
