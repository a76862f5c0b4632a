# r02l: GPU parity suite + smoke on the build with the fast-reciprocal Lehmer estimate and v_bitop3 SHA-512
set -o pipefail
D=gpurun_out/r02l
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -30 $D/gpu_tests.txt; exit 1; }
tail -2 $D/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || { tail -20 $D/smoke.txt; exit 1; }
tail -1 $D/smoke.txt
