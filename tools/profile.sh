#!/bin/bash
# Profile the verify kernel on the GPU box (run from the repo root). Writes under gpurun_out/prof_$TAG.
# Kernel trace + stats in one pass; PMC counters in separate passes (never combined with sys/runtime trace).
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 --pmc-traffic 0 --churn-legs 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || exit 11
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-trace --output-format csv -d $OUT/pmc1 -o run -- $B > $OUT/pmc1.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pmc2 -o run -- $B > $OUT/pmc2.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc3 -o run -- $B > $OUT/pmc3.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc4 -o run -- $B > $OUT/pmc4.log 2>&1 || exit 15
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $OUT/pmc5 -o run -- $B > $OUT/pmc5.log 2>&1 || true
echo done
