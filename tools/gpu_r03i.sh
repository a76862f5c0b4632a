# r03i: does the next launch fill the previous launch's drain? (two contexts / two streams vs serial vs 2M launches)
set -o pipefail
D=gpurun_out/r03i
mkdir -p $D
export TMPDIR=/tmp
for st in hip prio; do
timeout -k 10 300 python3 -u tools/overlap_probe.py --rounds 3 --streams $st > $D/overlap_$st.txt 2>&1 || { tail -20 $D/overlap_$st.txt; exit 1; }
echo "== $st"; cat $D/overlap_$st.txt
done
