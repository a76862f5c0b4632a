#!/bin/bash
# Stall-reason / instruction-cache PMC passes over a short bench run (one rocprofv3 pass per counter set).
set -o pipefail
TAG=${1:-stall}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 0 --cpu-sample 0 --pmc-traffic 0 --churn-legs 0"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --kernel-trace --output-format csv -d $OUT/a -o run -- $B > $OUT/a.log 2>&1 || exit 11
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_IFETCH SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU --kernel-trace --output-format csv -d $OUT/b -o run -- $B > $OUT/b.log 2>&1 || exit 12
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC --kernel-trace --output-format csv -d $OUT/c -o run -- $B > $OUT/c.log 2>&1 || exit 13
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/d -o run -- $B > $OUT/d.log 2>&1 || exit 14
echo done
