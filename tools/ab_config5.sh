#!/bin/bash
# A/B of libat2v builds on config 5 (4 nodes, 20k tx/s, combs, eager queue) with 2% first-seen senders and without
# (run ON the GPU box from the repo root):  bash tools/ab_config5.sh <tag> <variant_a> <variant_b> [rounds]
# Each run copies at2-node_amd/at2v/variants/libat2v_<v>.so over the package's library (the box's tree is scratch) and
# prints each node's queue p50 / p99.
set -o pipefail
TAG=$1; A=$2; B=$3; ROUNDS=${4:-2}
D=gpurun_out/$TAG
mkdir -p $D
L=at2-node_amd/at2v/libat2v.so
cp $L $D/.orig.so
for r in $(seq 1 $ROUNDS); do
  for v in $A $B; do
    for fresh in 0 0.02; do
      cp at2-node_amd/at2v/variants/libat2v_$v.so $L
      out=$D/c5_${v}_f${fresh}_$r.txt
      timeout -k 10 240 python3 tools/mininode.py --nodes 4 --rate 20000 --seconds 2 --batch 1024 --delay-us 1000 \
        --eager 1 --comb 1 --fresh-frac $fresh > $out 2>&1 \
        || { echo "[ab_config5] $v FAILED rc=$?"; tail -20 $out; cp $D/.orig.so $L; exit 1; }
      grep "^{" $out | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('$v fresh $fresh', [(round(n['queue_p50_us']), round(n['queue_p99_us'])) for n in d['per_node']],
      'wall_s %.2f' % d['wall_s'])"
    done
  done
done
cp $D/.orig.so $L
