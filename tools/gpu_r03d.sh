# r03d: table-footprint sweep (waves share K table slots; wrong verdicts, timing only) vs the current build and round 2
set -o pipefail
D=gpurun_out/r03d
mkdir -p $D
export TMPDIR=/tmp
V=at2-node_amd/at2v/variants
timeout -k 10 400 python3 tools/ab_bench.py $V/libat2v_base.so $V/libat2v_cur.so $V/libat2v_slot256.so $V/libat2v_slot512.so $V/libat2v_slot1024.so $V/libat2v_slot1536.so --rounds 8 --no-check > $D/ab_footprint.txt 2>&1 || { tail -20 $D/ab_footprint.txt; exit 1; }
cat $D/ab_footprint.txt
bash tools/gpu_r03c.sh
