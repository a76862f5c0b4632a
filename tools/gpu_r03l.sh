# r03l: small-batch latency with and without combs (latency probe), rocprofv3 kernel trace (csv) of the default bench
set -o pipefail
D=gpurun_out/r03l
mkdir -p $D
export TMPDIR=/tmp
for c in 0 1; do
timeout -k 10 300 python3 tools/latency_probe.py --reps 100 --comb $c > $D/latency_comb$c.json 2> $D/latency.err || { tail -20 $D/latency.err; exit 1; }
done
python3 -c "
import json
for c in (0,1):
    r=json.load(open('$D/latency_comb%d.json'%c))
    print('comb',c,{B:{k:round(v['p50_us']) for k,v in x.items()} for B,x in r['sizes'].items()})
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 20 --warmup 3 --pmc-traffic 0 --cpu-sample 0 --e2e 0 > $D/bench_under_rocprof.json 2> $D/rocprof.err || { tail -20 $D/rocprof.err; exit 1; }
find $D/prof -name '*kernel_stats.csv' -exec cp {} $D/kernel_stats.csv \;
head -4 $D/kernel_stats.csv
