#!/bin/bash
# gpu_run.sh — the GPU-box recipe (runs ON the box, from the repo root, under gpurun):
#   tools/gpu.sh 900 'bash tools/gpu_run.sh <tag> <stage> [<stage> ...]'
# Stages run in the order given; each has its own time limit, and the first failing stage ends the run (no GPU step
# after a failure). Outputs go to gpurun_out/<tag>/ (copy what is to be kept into profiles/<tag>/).
#   suite         pytest -m gpu (the whole parity / boundary / cache suite)
#   tests=<expr>  pytest -m gpu -k <expr>
#   files=<a,b>   pytest -m gpu on those test files
#   probe=<expr>  pytest -m gpu -k <expr>, output gpu_probe<N>.txt; test failures (exit 1) do not end the run, any other
#                 failure (time limit, crash) does
#   smoke         __graft_entry__.smoke()
#   bench         python bench.py (the default driver line: config 2 + at2_traffic + roofline + cpu_baseline)
#   benchat2      python bench.py on AT2 traffic as the main leg (64 senders, combs) with the PMC passes
#   bench1        python bench.py with the PMC passes and CPU baseline off (a quick rate check)
#   torchrun1     the world-1 torchrun rehearsal of the N > 1 bench path (RCCL gather inside the timed loop)
#   torchrun3     the same with config 3's per-rank load (2M records per rank: 16M over 8 GPUs)
#   rocprof       rocprofv3 --kernel-trace --stats of a bench run with one scratch set (per-kernel averages)
#   latency       tools/latency_probe.py --comb 1 (small-batch and first-seen-sender latency)
#   latab         latency probe and config 5 (combs) with the queue's verdict copy (AT2V_QUEUE_DIRECT=0) and with direct
#                 verdict writes (=1), alternating
#   spinab        the same A/B for the completer's event polling (AT2V_QUEUE_SPIN_US=0 vs 2000)
#   zcab          the same A/B for kernels reading small batches from pinned host memory (AT2V_QUEUE_ZEROCOPY=0 vs 1024)
#   lhab          the same A/B for launches from the producer / completer thread (AT2V_QUEUE_LAUNCH_HERE=0 vs 1)
#   latprof       rocprofv3 --kernel-trace of a short latency probe (per-launch kernel durations)
#   fresh         tools/fresh_sweep.sh: config 5 with a stream of first-seen senders (queue p50/p99 per node)
#   stall/stallat2 wave-cycle split (issue / issue-stall / s_waitcnt) of verify_kernel / verify_kernel_comb
#   icache        tools/icache_pmc.sh: instruction-cache hits / misses of the comb and ladder kernels
#   abchurn=<a,b> tools/ab_churn.sh: the bench's AT2-traffic and churn legs with variant a / b, alternating, 2 rounds
#   ab5=<a,b>     tools/ab_config5.sh: config 5 (0% and 2% first-seen senders) with variant a / b, alternating
#   pmc           tools/profile.sh: rocprofv3 kernel trace + the PMC passes (one counter group per pass)
#   ab=<a,b,...>  tools/ab_bench.py over at2-node_amd/at2v/variants/libat2v_<a>.so ... (distinct keys)
#   abcomb=<...>  the same on 64-sender traffic with combs (abwide=: with the wide comb of B, AT2V_CTX_BCOMB_WIDE)
#   cprobe=<...>  the same with --probe: per-wait cycle table of builds made with -DAT2V_COMB_PROBE (cprobex=: without
#                 the verdict check, for timing-only experiment builds)
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
# the library's A/B and test hooks (AT2V_SCRATCH_SETS, AT2V_QUEUE_*, ...) act only with this gate (csrc/at2v_env.h); the
# driver's own bench and test runs do not set it (the suite's conftest does)
export AT2V_TEST_HOOKS=1
run() {  # run <name> <seconds> <cmd...>: stdout+stderr to $D/<name>.txt, tail on failure
  local name=$1 t=$2; shift 2
  echo "[gpu_run] $name ($t s): $*"
  timeout -k 10 "$t" "$@" > "$D/$name.txt" 2>&1 || { echo "[gpu_run] $name FAILED rc=$?"; tail -40 "$D/$name.txt"; exit 1; }
  tail -3 "$D/$name.txt"
}
NPROBE=0
for st in "$@"; do
  case "$st" in
    suite) run gpu_tests 1100 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread
           cp gpurun_out/config5_*.json $D/ 2>/dev/null ;;
    files=*) run gpu_tests_f 900 python -u -m pytest $(echo "${st#files=}" | tr ',' ' ') -m gpu -v -x --timeout 300 \
               --timeout-method thread
             cp gpurun_out/config5_*.json $D/ 2>/dev/null ;;
    tests=*) run gpu_tests_k 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "${st#tests=}"
             cp gpurun_out/config5_*.json $D/ 2>/dev/null ;;
    probe=*) NPROBE=$((NPROBE + 1))
             echo "[gpu_run] probe$NPROBE: ${st#probe=}"
             timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
               -k "${st#probe=}" > $D/gpu_probe$NPROBE.txt 2>&1
             rc=$?
             tail -3 $D/gpu_probe$NPROBE.txt
             mkdir -p $D/probe$NPROBE && cp gpurun_out/config5_*.json $D/probe$NPROBE/ 2>/dev/null
             [ $rc -le 1 ] || { echo "[gpu_run] probe$NPROBE FAILED rc=$rc"; exit 1; } ;;
    smoke) run smoke 180 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 500 python3 bench.py
           grep '^{' $D/bench.txt > $D/bench.json ;;
    benchat2) run benchat2 400 python3 bench.py --senders 64 --sender-cache 1024 --sender-comb 1 --cpu-sample 0 --e2e 0
              grep '^{' $D/benchat2.txt > $D/benchat2.json ;;
    bench1) run bench1 300 python3 bench.py --pmc-traffic 0 --cpu-sample 0 --e2e 0
            grep '^{' $D/bench1.txt > $D/bench1.json ;;
    torchrun1) run torchrun1 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
                 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 2 --e2e 0
               grep '^{' $D/torchrun1.txt > $D/torchrun1.json ;;
    torchrun3) run torchrun3 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
                 --master-port 29534 bench.py --gpus 1 --steps 10 --warmup 2 --e2e 0 --records-per-gpu 2097152
               grep '^{' $D/torchrun3.txt > $D/torchrun3.json ;;
    rocprof) export AT2V_SCRATCH_SETS=1
             run rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- \
               python3 bench.py --steps 20 --warmup 3 --pmc-traffic 0 --cpu-sample 0 --e2e 0 --churn-legs 0
             unset AT2V_SCRATCH_SETS
             find $D/prof -name '*kernel_stats.csv' -exec cp {} $D/kernel_stats.csv \; ;;
    latab) for r in 1 2; do for v in 0 1; do
             AT2V_QUEUE_DIRECT=$v run lat_d${v}_$r 300 python3 tools/latency_probe.py --reps 100 --comb 1 --sizes 1,20,64
             AT2V_QUEUE_DIRECT=$v run c5_d${v}_$r 200 python3 tools/mininode.py --nodes 4 --rate 20000 --seconds 2 \
               --batch 1024 --delay-us 1000 --eager 1 --comb 1
           done; done ;;
    spinab) for r in 1 2; do for v in 0 2000; do
             AT2V_QUEUE_SPIN_US=$v run lat_s${v}_$r 300 python3 tools/latency_probe.py --reps 100 --comb 1 --sizes 1,20,64
             AT2V_QUEUE_SPIN_US=$v run c5_s${v}_$r 200 python3 tools/mininode.py --nodes 4 --rate 20000 --seconds 2 \
               --batch 1024 --delay-us 1000 --eager 1 --comb 1
           done; done ;;
    zcab) for r in 1 2; do for v in 0 1024; do
             AT2V_QUEUE_ZEROCOPY=$v run lat_z${v}_$r 300 python3 tools/latency_probe.py --reps 100 --comb 1 --sizes 1,64,1024
             AT2V_QUEUE_ZEROCOPY=$v run c5_z${v}_$r 200 python3 tools/mininode.py --nodes 4 --rate 20000 --seconds 2 \
               --batch 1024 --delay-us 1000 --eager 1 --comb 1
           done; done ;;
    lhab) for r in 1 2; do for v in 0 1; do
             AT2V_QUEUE_LAUNCH_HERE=$v run lat_l${v}_$r 300 python3 tools/latency_probe.py --reps 100 --comb 1 --sizes 1,20,64
             AT2V_QUEUE_LAUNCH_HERE=$v run c5_l${v}_$r 200 python3 tools/mininode.py --nodes 4 --rate 20000 --seconds 2 \
               --batch 1024 --delay-us 1000 --eager 1 --comb 1
           done; done ;;
    latprof) run latprof 300 rocprofv3 --kernel-trace --output-format csv -d $D/latprof -o run -- \
               python3 tools/latency_probe.py --reps 20 --comb 1 --sizes 1,64
             find $D/latprof -name '*kernel_trace.csv' -exec cp {} $D/latprof_trace.csv \; ;;
    fresh) run fresh 900 bash tools/fresh_sweep.sh $TAG ;;
    pmc) run pmc 1100 bash tools/profile.sh $TAG ;;
    stallat2) run stallat2 400 bash tools/stall_pmc_at2.sh $TAG ;;
    icache) run icache 400 bash tools/icache_pmc.sh $TAG ;;
    abchurn=*) run abchurn 900 bash tools/ab_churn.sh $TAG $(echo "${st#abchurn=}" | tr ',' ' ') 2 ;;
    ab5=*) run ab5 900 bash tools/ab_config5.sh $TAG $(echo "${st#ab5=}" | tr ',' ' ') 1 ;;
    stall) run stall 300 bash tools/stall_pmc_quick.sh $TAG ;;
    latency) run latency 400 python3 tools/latency_probe.py --reps 100 --comb 1
             grep '^{' $D/latency.txt > $D/latency_comb1.json ;;
    ab=*) libs=""
          for v in $(echo "${st#ab=}" | tr ',' ' '); do libs="$libs at2-node_amd/at2v/variants/libat2v_$v.so"; done
          run ab 900 python3 tools/ab_bench.py $libs --rounds 12 ;;
    abcomb=*) libs=""
          for v in $(echo "${st#abcomb=}" | tr ',' ' '); do libs="$libs at2-node_amd/at2v/variants/libat2v_$v.so"; done
          run abcomb 900 python3 tools/ab_bench.py $libs --rounds 12 --senders 64 --comb ;;
    abx=*) libs=""  # experiment builds (wrong verdicts allowed), distinct keys
          for v in $(echo "${st#abx=}" | tr ',' ' '); do libs="$libs at2-node_amd/at2v/variants/libat2v_$v.so"; done
          run abx 900 python3 tools/ab_bench.py $libs --rounds 12 --no-check ;;
    cprobe=*|cprobex=*) libs=""; chk=""; [ "${st%%=*}" = cprobex ] && chk="--no-check"
          for v in $(echo "${st#*=}" | tr ',' ' '); do libs="$libs at2-node_amd/at2v/variants/libat2v_$v.so"; done
          run ${st%%=*} 900 python3 tools/ab_bench.py $libs --rounds 8 --senders 64 --comb --probe $chk ;;
    abwide=*) libs=""  # AT2 traffic through contexts with the wide comb of B
          for v in $(echo "${st#abwide=}" | tr ',' ' '); do libs="$libs at2-node_amd/at2v/variants/libat2v_$v.so"; done
          run abwide 900 python3 tools/ab_bench.py $libs --rounds 12 --senders 64 --comb --wide ;;
    abcombx=*) libs=""  # experiment builds (wrong verdicts allowed)
          for v in $(echo "${st#abcombx=}" | tr ',' ' '); do libs="$libs at2-node_amd/at2v/variants/libat2v_$v.so"; done
          run abcombx 900 python3 tools/ab_bench.py $libs --rounds 12 --senders 64 --comb --no-check ;;
    *) echo "[gpu_run] unknown stage $st"; exit 2 ;;
  esac
done
echo "[gpu_run] done: $D"
