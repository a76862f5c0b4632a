# r03f: shared identity entry (per-lane tables hold [1..8]P): GPU parity + cache tests on it, then A/B vs the build
# without it (sig) and round 2 (base)
set -o pipefail
D=gpurun_out/r03f
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cache.py -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -30 $D/gpu_tests.txt; exit 1; }
tail -2 $D/gpu_tests.txt
V=at2-node_amd/at2v/variants
timeout -k 10 500 python3 tools/ab_bench.py $V/libat2v_base.so $V/libat2v_sig.so $V/libat2v_ident.so --rounds 16 > $D/ab_ident.txt 2>&1 || { tail -20 $D/ab_ident.txt; exit 1; }
cat $D/ab_ident.txt
