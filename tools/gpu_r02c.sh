set -o pipefail
mkdir -p gpurun_out/r02c
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02c/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r02c/gpu_tests.txt; exit 1; }
tail -3 gpurun_out/r02c/gpu_tests.txt
for n in 32 2048 16384 32768; do
  timeout -k 10 60 ./tools/phase_bench $n 0 2>&1 | grep "^n=" | sed "s/^/throughput /"
  timeout -k 10 60 ./tools/phase_bench $n 1048576 2>&1 | grep "^n=" | sed "s/^/lowlat     /"
done > gpurun_out/r02c/small_batch_latency.txt
cat gpurun_out/r02c/small_batch_latency.txt
cat gpurun_out/config5_eager.json | python3 -c "import json,sys; d=json.load(sys.stdin); print({k:d[k] for k in d if k!='per_node'})"
