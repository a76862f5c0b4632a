#!/bin/bash
# Wave-cycle split of the AT2-traffic comb kernel (verify_kernel_comb, 64 repeating senders with combs), two rocprofv3
# --pmc passes over the two steady-state steps of a short bench run (the two warm-up launches claim and build the keys):
#   pass 1: SQ_WAVE_CYCLES = SQ_ACTIVE_INST_ANY + SQ_WAIT_INST_ANY (issue stall) + SQ_WAIT_ANY (s_waitcnt / barrier)
#   pass 2: LDS and VMEM instruction counts and the LDS issue stall (SQ_WAIT_INST_LDS)
set -o pipefail
TAG=${1:-at2}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="bench.py --steps 2 --warmup 2 --cpu-sample 0 --pmc-traffic 0 --e2e 0 --traffic-leg 0 --senders 64 --sender-cache 1024 --sender-comb 1"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $OUT/p1 -o run -- python3 $ARGS > $OUT/run1.log 2>&1 || exit 11
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $OUT/p2 -o run -- python3 $ARGS > $OUT/run2.log 2>&1 || exit 12
for p in p1 p2; do
f=$(find $OUT/$p -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "verify_kernel_comb" in r.get("Kernel_Name", ""):
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
last = sorted(per)[-2:]  # the two timed steps
acc = collections.defaultdict(float)
for d in last:
    for k, v in per[d].items():
        acc[k] += v
w = acc["SQ_WAVE_CYCLES"]
print({k: (round(v / w, 4) if k != "SQ_WAVE_CYCLES" else v) for k, v in acc.items()})
PY
done
