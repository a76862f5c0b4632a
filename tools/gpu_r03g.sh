# r03g: round-3 build validation: full GPU suite, smoke, the default bench line (with its PMC passes), rocprofv3 kernel
# trace + stats, config 3's per-rank load through libat2v's RCCL gather at world 1 (torchrun), 64-sender traffic with
# and without the sender cache
set -o pipefail
D=gpurun_out/r03g
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -40 $D/gpu_tests.txt; exit 1; }
tail -3 $D/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || { tail -20 $D/smoke.txt; exit 1; }
cat $D/smoke.txt
timeout -k 10 600 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
cat $D/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --pmc-traffic 0 --e2e 0 > $D/bench_under_rocprof.json 2> $D/rocprof.err || { tail -20 $D/rocprof.err; exit 1; }
find $D/prof -name "*kernel_stats.csv" | head -1 | xargs cat | head -3
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --records-per-gpu 2097152 --cpu-sample 0 --pmc-traffic 0 --e2e 0 > $D/bench_torchrun_config3_rank.json 2> $D/tr.err || { tail -20 $D/tr.err; exit 1; }
cat $D/bench_torchrun_config3_rank.json
timeout -k 10 300 python3 bench.py --senders 64 --sender-cache 0 --cpu-sample 0 --pmc-traffic 0 --e2e 0 > $D/bench_s64_nocache.json 2> $D/b1.err || { tail -20 $D/b1.err; exit 1; }
timeout -k 10 300 python3 bench.py --senders 64 --sender-cache 4096 --cpu-sample 0 --pmc-traffic 0 --e2e 0 > $D/bench_s64_cache.json 2> $D/b2.err || { tail -20 $D/b2.err; exit 1; }
python3 -c "
import json
for f in ('bench_s64_nocache','bench_s64_cache'):
    r=json.load(open('$D/'+f+'.json')); print(f, round(r['value']/1e6,2), 'M/s kernel', round(r['kernel_ms'],3), 'ms match', r['verdict_match'])
"
