# r03zb: one wave per SIMD (512 VGPR+AGPR, no spills, 4-wave blocks, no pacing) against the default build, config 2
# and 64-sender comb traffic, A/B in one process
set -o pipefail
D=gpurun_out/r03zb
mkdir -p $D
export TMPDIR=/tmp
V=at2-node_amd/at2v/variants
timeout -k 10 400 python3 tools/ab_bench.py $V/libat2v_base.so $V/libat2v_w1.so --rounds 10 > $D/ab_w1.txt 2>&1 || { tail -20 $D/ab_w1.txt; exit 1; }
cat $D/ab_w1.txt
timeout -k 10 400 python3 tools/ab_bench.py $V/libat2v_base.so $V/libat2v_w1.so --senders 64 --comb --rounds 10 > $D/ab_w1_comb.txt 2>&1 || { tail -20 $D/ab_w1_comb.txt; exit 1; }
cat $D/ab_w1_comb.txt
