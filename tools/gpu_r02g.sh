# r02g: GPU parity suite (incl. the ragged long-message test) + config-3 per-GPU rehearsal (2M records per rank,
# torch.distributed.run world 1: libat2v RCCL communicator + verdict all-gather inside the timed loop)
set -o pipefail
D=gpurun_out/r02g
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -30 $D/gpu_tests.txt; exit 1; }
tail -2 $D/gpu_tests.txt
timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 1 --records-per-gpu 2097152 --steps 10 --warmup 2 --cpu-sample 0 --e2e 0 > $D/bench_cfg3_rank_torchrun.json 2> $D/bench_cfg3.err || { tail -20 $D/bench_cfg3.err; exit 1; }
cat $D/bench_cfg3_rank_torchrun.json
