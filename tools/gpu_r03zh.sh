# r03zh: rocprofv3 kernel trace of the final build, headline and AT2-traffic legs (one scratch set: launches serial)
set -o pipefail
D=gpurun_out/r03zh
mkdir -p $D
export TMPDIR=/tmp
AT2V_SCRATCH_SETS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 20 --warmup 3 --pmc-traffic 0 --cpu-sample 0 --e2e 0 > $D/bench_under_rocprof.json 2> $D/rocprof.err || { tail -20 $D/rocprof.err; exit 1; }
find $D/prof -name '*kernel_stats.csv' -exec cp {} $D/kernel_stats.csv \;
python3 -c "
import csv
for r in csv.DictReader(open('$D/kernel_stats.csv')):
    print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e6, 4), r['Percentage'])
" | head -20
grep -o '"launch_ms_alone": [0-9.]*' $D/bench_under_rocprof.json
