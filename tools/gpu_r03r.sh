# r03r: A/B of one-product-at-a-time group law (AT2V_GU_X2=0) on top of sequential decode/tables (dectab1)
set -o pipefail
D=gpurun_out/r03r
mkdir -p $D
export TMPDIR=/tmp
V=at2-node_amd/at2v/variants
timeout -k 10 700 python3 tools/ab_bench.py $V/libat2v_base.so $V/libat2v_dectab1.so $V/libat2v_gux1.so $V/libat2v_gu1only.so --rounds 12 > $D/ab_gu.txt 2>&1 || { tail -20 $D/ab_gu.txt; exit 1; }
cat $D/ab_gu.txt
