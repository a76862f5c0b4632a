# r03h: cache lookup with one leader per distinct key per wave; SHA-512 message reader split (fast path straight-line)
# and early message touch: full GPU suite, then A/B vs round 2 (base) and the r03f build (ident)
set -o pipefail
D=gpurun_out/r03h
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -40 $D/gpu_tests.txt; exit 1; }
tail -3 $D/gpu_tests.txt
V=at2-node_amd/at2v/variants
timeout -k 10 500 python3 tools/ab_bench.py $V/libat2v_base.so $V/libat2v_ident.so $V/libat2v_split.so $V/libat2v_touch.so --rounds 16 > $D/ab_msg.txt 2>&1 || { tail -20 $D/ab_msg.txt; exit 1; }
cat $D/ab_msg.txt
