# r03u: tables built right after each decode (AT2V_TABLES_EARLY, R's sign applied per digit): GPU suite; A/B vs the
# round-3 order (early0) and with one lattice state set (early_lpp0)
set -o pipefail
D=gpurun_out/r03u
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1
rc=$?
tail -3 $D/gpu_tests.txt
grep -E "FAILED|ERROR" $D/gpu_tests.txt | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
V=at2-node_amd/at2v/variants
timeout -k 10 700 python3 tools/ab_bench.py $V/libat2v_early0.so $V/libat2v_cur.so $V/libat2v_early_lpp0.so --rounds 14 > $D/ab.txt 2>&1 || { tail -20 $D/ab.txt; exit 1; }
cat $D/ab.txt
