# r03t: single-product group law as default: GPU suite; A/B of register-pressure options on the new baseline
set -o pipefail
D=gpurun_out/r03t
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1
rc=$?
tail -3 $D/gpu_tests.txt
grep -E "FAILED|ERROR" $D/gpu_tests.txt | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
V=at2-node_amd/at2v/variants
timeout -k 10 700 python3 tools/ab_bench.py $V/libat2v_cur.so $V/libat2v_park1.so $V/libat2v_sqn0.so $V/libat2v_lpp0.so --rounds 12 > $D/ab.txt 2>&1 || { tail -20 $D/ab.txt; exit 1; }
cat $D/ab.txt
