# r03y: A/B of table-build placement: both after the reduction (cur), both early (early1), A early (early2), R early (early3)
set -o pipefail
D=gpurun_out/r03y
mkdir -p $D
export TMPDIR=/tmp
V=at2-node_amd/at2v/variants
timeout -k 10 700 python3 tools/ab_bench.py $V/libat2v_cur.so $V/libat2v_early1.so $V/libat2v_early2.so $V/libat2v_early3.so --rounds 14 > $D/ab.txt 2>&1 || { tail -20 $D/ab.txt; exit 1; }
cat $D/ab.txt
