# r03v: comb throughput path restructured (helpers inlined, short live ranges), early tables off again: GPU suite and
# the bench line (headline + AT2-traffic leg)
set -o pipefail
D=gpurun_out/r03v
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1
rc=$?
tail -3 $D/gpu_tests.txt
grep -E "FAILED|ERROR" $D/gpu_tests.txt | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python3 -c "
import json; r=json.load(open('$D/bench.json'))
print('value', r['value'], 'kernel_ms', r['kernel_ms'], 'alone', r['launch_ms_alone'], 'clk', r['effective_clock_ghz'], 'frac', r['roofline']['frac'], 'valu/verify', r['roofline']['valu_measured']['valu_lane_ops_per_verify'], 'traffic/verify', r['roofline']['traffic_detail']['bytes_per_verify'])
print('at2_traffic', r['at2_traffic']['value'], r['at2_traffic']['verdicts_ok'], 'e2e', r.get('e2e_verifies_per_s'))
"
