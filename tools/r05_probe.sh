#!/bin/bash
# r05_probe.sh — round-5 GPU probes (run ON the box from the repo root, under gpurun):
#   bash tools/r05_probe.sh <tag> <stage> [<stage> ...]
#   partprof   rocprofv3 kernel trace of AT2 traffic (64 senders, combs) as the main bench leg, partitioned launches
#   distprof   rocprofv3 kernel trace of the headline + the distinct-key churn leg (verify_kernel vs the partitioned
#              launch's classify and miss kernels on the same kind of records)
#   partab     the same traffic, wall-clock rate with AT2V_CACHE_PARTITION=0 / 1 alternating (2 rounds)
#   pollute2   config 5 (2% first-seen) beside TWO polluter processes, node processes with HIP's default 4 hardware
#              queues vs GPU_MAX_HW_QUEUES=2 (2 rounds)
#   stallat2   tools/stall_pmc_at2.sh (wave-cycle split of the comb kernel on AT2 traffic)
#   pollute    config 5 with 2% first-seen senders, without / with a polluter process (RCCL + 6 streams), for the queue
#              stream settings default / AT2V_QUEUE_STREAMS=1 / AT2V_QUEUE_STREAMS=1 + AT2V_QUEUE_PRIORITY=1
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
run() {  # run <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "[probe] $name ($t s): $*"
  timeout -k 10 "$t" "$@" > "$D/$name.txt" 2>&1 || { echo "[probe] $name FAILED rc=$?"; tail -30 "$D/$name.txt"; exit 1; }
  tail -2 "$D/$name.txt" | cut -c1-400
}
AT2="--senders 64 --sender-cache 1024 --sender-comb 1 --steps 10 --cpu-sample 0 --e2e 0 --pmc-traffic 0 --traffic-leg 0 --churn-legs 0"
DIST="--steps 10 --cpu-sample 0 --e2e 0 --pmc-traffic 0 --traffic-leg 0 --churn-legs distinct"
for st in "$@"; do
  case "$st" in
    partprof) run partprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py $AT2
              find $D/prof -name '*kernel_stats.csv' -exec cp {} $D/partprof_kernel_stats.csv \; ;;
    distprof) run distprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/dprof -o run -- python3 bench.py $DIST
              find $D/dprof -name '*kernel_stats.csv' -exec cp {} $D/distprof_kernel_stats.csv \; ;;
    partab) for r in 1 2; do for v in 0 1; do
              AT2V_CACHE_PARTITION=$v run partab_p${v}_$r 200 python3 bench.py $AT2
            done; done ;;
    pollute) for p in 0 1; do
               for mode in default s1 s1p; do
                 case $mode in default) E="";; s1) E="AT2V_QUEUE_STREAMS=1";; s1p) E="AT2V_QUEUE_STREAMS=1 AT2V_QUEUE_PRIORITY=1";; esac
                 run c5_pol${p}_$mode 240 env $E python3 tools/mininode.py --nodes 4 --rate 20000 --seconds 2 --batch 1024 \
                   --delay-us 1000 --eager 1 --comb 1 --fresh-frac 0.02 --polluter $p
               done
             done ;;
    pollute2) for r in 1 2; do for mode in default hwq2; do
                case $mode in default) E="";; hwq2) E="--node-hw-queues 2";; esac
                run c5_pol2_${mode}_$r 240 python3 tools/mininode.py --nodes 4 --rate 20000 --seconds 2 --batch 1024 \
                  --delay-us 1000 --eager 1 --comb 1 --fresh-frac 0.02 --polluter 2 $E
              done; done ;;
    stallat2) run stallat2 400 bash tools/stall_pmc_at2.sh $TAG ;;
    *) echo "[probe] unknown stage $st"; exit 2 ;;
  esac
done
echo "[probe] done: $D"
