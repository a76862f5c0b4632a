# r03zd: final inversions shared by 1 / 2 (default) / 3 / 4 chunks per lane, config 2, A/B in one process
set -o pipefail
D=gpurun_out/r03zd
mkdir -p $D
export TMPDIR=/tmp
V=at2-node_amd/at2v/variants
timeout -k 10 600 python3 tools/ab_bench.py $V/libat2v_base.so $V/libat2v_inv1.so $V/libat2v_inv3.so $V/libat2v_inv4.so --rounds 10 > $D/ab_inv_group.txt 2>&1 || { tail -20 $D/ab_inv_group.txt; exit 1; }
cat $D/ab_inv_group.txt
