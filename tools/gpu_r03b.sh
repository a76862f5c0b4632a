# r03b: per-sender A cache (GPU tests), A/B of the cache-off path vs the round-2 kernel, table-traffic experiment
# (waves sharing table slots, wrong verdicts, timing only), bench with 64 repeating senders with and without the cache
set -o pipefail
D=gpurun_out/r03b
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -40 $D/gpu_tests.txt; exit 1; }
tail -3 $D/gpu_tests.txt
V=at2-node_amd/at2v/variants
timeout -k 10 300 python3 tools/ab_bench.py $V/libat2v_base.so $V/libat2v_nopp.so $V/libat2v_pp.so $V/libat2v_park.so $V/libat2v_slot8.so $V/libat2v_slot256.so --rounds 8 --no-check > $D/ab_slots.txt 2>&1 || { tail -20 $D/ab_slots.txt; exit 1; }
cat $D/ab_slots.txt
timeout -k 10 300 python3 tools/latency_probe.py --reps 100 > $D/latency_probe.json 2> $D/latency_probe.err || { tail -20 $D/latency_probe.err; exit 1; }
cat $D/latency_probe.err
timeout -k 10 300 python3 bench.py --senders 64 --sender-cache 0 --cpu-sample 0 --pmc-traffic 0 --e2e 0 --steps 10 > $D/bench_s64_nocache.json 2> $D/b1.err || { tail -20 $D/b1.err; exit 1; }
timeout -k 10 300 python3 bench.py --senders 64 --sender-cache 4096 --cpu-sample 0 --pmc-traffic 0 --e2e 0 --steps 10 > $D/bench_s64_cache.json 2> $D/b2.err || { tail -20 $D/b2.err; exit 1; }
python3 -c "
import json
for f in ('bench_s64_nocache','bench_s64_cache'):
    r=json.load(open('$D/'+f+'.json')); print(f, round(r['value']/1e6,2), 'M/s kernel', round(r['kernel_ms'],3), 'ms match', r['verdict_match'])
"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || { tail -20 $D/smoke.txt; exit 1; }
cat $D/smoke.txt
timeout -k 10 600 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
cat $D/bench.json
