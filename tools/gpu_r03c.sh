# r03c: profiles of the round-3 build: rocprofv3 kernel trace + stats of the bench, the wave-cycle split (one PMC pass),
# and the stall / instruction-mix passes the verdict asked for (LDS issue stalls, SMEM, VMEM cycles, scratch)
set -o pipefail
D=gpurun_out/r03c
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --pmc-traffic 0 --e2e 0 > $D/bench_under_rocprof.json 2> $D/rocprof.err || { tail -20 $D/rocprof.err; exit 1; }
find $D/prof -name "*kernel_stats.csv" | head -1 | xargs cat | head -6
B="python3 bench.py --steps 2 --warmup 0 --cpu-sample 0 --pmc-traffic 0 --e2e 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD --kernel-trace --output-format csv -d $D/pmc_a -o run -- $B > $D/pmc_a.log 2>&1 || { tail -5 $D/pmc_a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $D/pmc_b -o run -- $B > $D/pmc_b.log 2>&1 || { tail -5 $D/pmc_b.log; exit 1; }
python3 - $D <<'PY'
import csv, sys, glob, collections
d = sys.argv[1]
for sub in ("pmc_a", "pmc_b"):
    acc = collections.defaultdict(float); disp = set()
    for f in glob.glob(f"{d}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "verify_kernel" in r.get("Kernel_Name", ""):
                acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
    n = max(1, len(disp))
    print(sub, {k: v / n for k, v in acc.items()})
    if "SQ_WAVE_CYCLES" in acc:
        w = acc["SQ_WAVE_CYCLES"]
        print(sub, "shares of wave cycles", {k: round(v / w, 4) for k, v in acc.items() if k.startswith("SQ_WAIT") or k.startswith("SQ_ACTIVE")})
PY
