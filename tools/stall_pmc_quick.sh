#!/bin/bash
# Wave-cycle split of the verify kernel (one rocprofv3 --pmc pass over a short bench run, no e2e leg):
# SQ_WAVE_CYCLES = SQ_ACTIVE_INST_ANY + SQ_WAIT_INST_ANY (issue stall) + SQ_WAIT_ANY (s_waitcnt / barrier), MI355X guide.
set -o pipefail
TAG=${1:-quick}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --churn-legs 0 --steps 2 --warmup 0 --cpu-sample 0 --pmc-traffic 0 --e2e 0 > $OUT/run.log 2>&1 || exit 11
f=$(find $OUT -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "verify_kernel" in r.get("Kernel_Name", ""):
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
w = acc["SQ_WAVE_CYCLES"]
print({k: round(v / w, 4) for k, v in acc.items()})
PY
