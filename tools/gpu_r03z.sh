# r03z: A-comb window 8 vs 10 bits on 1M records from 64 senders (one process), and the cache/comb GPU tests on the
# in-tree (8-bit) build
set -o pipefail
D=gpurun_out/r03z
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cache.py -v --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -30 $D/gpu_tests.txt; exit 1; }
tail -2 $D/gpu_tests.txt
V=at2-node_amd/at2v/variants
timeout -k 10 600 python3 tools/ab_bench.py $V/libat2v_comb8.so $V/libat2v_comb10.so --senders 64 --comb --rounds 14 > $D/ab_comb_bits.txt 2>&1 || { tail -20 $D/ab_comb_bits.txt; exit 1; }
cat $D/ab_comb_bits.txt
