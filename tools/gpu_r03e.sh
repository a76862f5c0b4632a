# r03e: uncached kernel with round 2's own signature (no extra parameters), with and without the squaring ping-pong,
# vs round 2 (base) and the templated kernel (cur)
set -o pipefail
D=gpurun_out/r03e
mkdir -p $D
export TMPDIR=/tmp
V=at2-node_amd/at2v/variants
timeout -k 10 400 python3 tools/ab_bench.py $V/libat2v_base.so $V/libat2v_cur.so $V/libat2v_sig.so $V/libat2v_signopp.so --rounds 10 > $D/ab_sig.txt 2>&1 || { tail -20 $D/ab_sig.txt; exit 1; }
cat $D/ab_sig.txt
