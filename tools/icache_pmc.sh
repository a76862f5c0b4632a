#!/bin/bash
# Instruction-cache behaviour of the comb kernel (AT2 traffic, verify_kernel_comb_part) against the ladder kernel
# (distinct keys, verify_kernel): one rocprofv3 --pmc pass per workload with the SQC instruction-cache hit/miss
# counters and the SQ's instruction-fetch count next to the wave cycles.
#   bash tools/icache_pmc.sh <tag>      (on the GPU box, from the repo root)
set -o pipefail
TAG=${1:-ic}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
AT2="bench.py --steps 2 --warmup 2 --cpu-sample 0 --pmc-traffic 0 --e2e 0 --traffic-leg 0 --churn-legs 0 --senders 64 --sender-cache 1024 --sender-comb 1"
DIST="bench.py --steps 2 --warmup 0 --cpu-sample 0 --pmc-traffic 0 --e2e 0 --traffic-leg 0 --churn-legs 0"
CTRS="SQ_WAVE_CYCLES SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES"
timeout -s KILL 150 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $OUT/at2 -o run -- python3 $AT2 > $OUT/at2.log 2>&1 || exit 11
timeout -s KILL 150 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $OUT/dist -o run -- python3 $DIST > $OUT/dist.log 2>&1 || exit 12
for p in at2:verify_kernel_comb dist:verify_kernel\(; do
f=$(find $OUT/${p%%:*} -name "*counter_collection.csv" | head -1)
python3 - "$f" "${p#*:}" <<'PY'
import csv, sys, collections
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r.get("Kernel_Name", ""):
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
last = sorted(per)[-2:]  # the two timed steps
acc = collections.defaultdict(float)
for d in last:
    for k, v in per[d].items():
        acc[k] += v
h, m = acc.get("SQC_ICACHE_HITS", 0.0), acc.get("SQC_ICACHE_MISSES", 0.0)
print(sys.argv[2], dict(acc), "icache miss rate %.4f" % (m / max(1.0, h + m)),
      "misses per 1k wave-cycles %.3f" % (1000 * m / max(1.0, acc.get("SQ_WAVE_CYCLES", 1.0))))
PY
done
