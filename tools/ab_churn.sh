#!/bin/bash
# A/B of libat2v builds on the bench's AT2-traffic and sender-churn legs (run ON the GPU box from the repo root):
#   bash tools/ab_churn.sh <tag> <variant_a> <variant_b> [rounds]
# Each round runs bench.py once per variant (at2-node_amd/at2v/variants/libat2v_<v>.so copied over the package's
# library for that run; the box's copy of the tree is scratch), alternating, and prints the legs' rates.
set -o pipefail
TAG=$1; A=$2; B=$3; ROUNDS=${4:-2}
D=gpurun_out/$TAG
mkdir -p $D
L=at2-node_amd/at2v/libat2v.so
cp $L $D/.orig.so
for r in $(seq 1 $ROUNDS); do
  for v in $A $B; do
    cp at2-node_amd/at2v/variants/libat2v_$v.so $L
    echo "[ab_churn] round $r variant $v"
    timeout -k 10 240 python3 bench.py --steps 10 --cpu-sample 0 --pmc-traffic 0 --e2e 0 > $D/churn_${v}_$r.txt 2>&1 \
      || { echo "[ab_churn] $v FAILED rc=$?"; tail -20 $D/churn_${v}_$r.txt; cp $D/.orig.so $L; exit 1; }
    grep "^{" $D/churn_${v}_$r.txt | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
legs = {'plain': d['value'], 'at2': d['at2_traffic']['value']}
legs.update({k: v['value'] for k, v in d['sender_churn'].items() if k != 'method'})
print('$v', ' '.join(f'{k} {x / 1e6:.1f}' for k, x in legs.items()))"
  done
done
cp $D/.orig.so $L
