# r03w: A/B of the comb throughput path (r03s form vs restructured) on 1M records from 64 senders, in one process
set -o pipefail
D=gpurun_out/r03w
mkdir -p $D
export TMPDIR=/tmp
V=at2-node_amd/at2v/variants
timeout -k 10 600 python3 tools/ab_bench.py $V/libat2v_comb_old.so $V/libat2v_cur.so --senders 64 --comb --rounds 14 > $D/ab_comb.txt 2>&1 || { tail -20 $D/ab_comb.txt; exit 1; }
cat $D/ab_comb.txt
