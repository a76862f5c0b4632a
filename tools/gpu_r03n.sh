# r03n: full bench line with the AT2-traffic leg; world-1 torchrun bench (RCCL gathers of overlapped steps); rocprofv3
# kernel trace of the bench with one scratch set (serial launches: per-launch durations comparable to launch_ms_alone)
set -o pipefail
D=gpurun_out/r03n
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
cat $D/bench.json
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 3 --pmc-traffic 0 --cpu-sample 0 > $D/bench_torchrun_n1.json 2> $D/torchrun.err || { tail -20 $D/torchrun.err; exit 1; }
cat $D/bench_torchrun_n1.json
AT2V_SCRATCH_SETS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 20 --warmup 3 --pmc-traffic 0 --cpu-sample 0 --e2e 0 --traffic-leg 0 > $D/bench_serial_under_rocprof.json 2> $D/rocprof.err || { tail -20 $D/rocprof.err; exit 1; }
find $D/prof -name '*kernel_stats.csv' -exec cp {} $D/kernel_stats_serial.csv \;
head -3 $D/kernel_stats_serial.csv
grep -o '"launch_ms_alone": [0-9.]*' $D/bench_serial_under_rocprof.json
