# r03q: A/B of the interleaved A/R decode and table build (AT2V_DECODE_X2, AT2V_TABLES_X2) in one process
set -o pipefail
D=gpurun_out/r03q
mkdir -p $D
export TMPDIR=/tmp
V=at2-node_amd/at2v/variants
timeout -k 10 600 python3 tools/ab_bench.py $V/libat2v_base.so $V/libat2v_dec1.so $V/libat2v_tab1.so $V/libat2v_dectab1.so --rounds 12 > $D/ab_interleave.txt 2>&1 || { tail -20 $D/ab_interleave.txt; exit 1; }
cat $D/ab_interleave.txt
