# r03zc: A-comb windows of 10 (default) / 11 / 12 / 13 bits on 1M records from 64 senders, A/B in one process
set -o pipefail
D=gpurun_out/r03zc
mkdir -p $D
export TMPDIR=/tmp
V=at2-node_amd/at2v/variants
timeout -k 10 600 python3 tools/ab_bench.py $V/libat2v_base.so $V/libat2v_comb11.so $V/libat2v_comb12.so $V/libat2v_comb13.so --senders 64 --comb --rounds 12 > $D/ab_comb_bits.txt 2>&1 || { tail -20 $D/ab_comb_bits.txt; exit 1; }
cat $D/ab_comb_bits.txt
