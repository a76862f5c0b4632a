#!/bin/bash
# Run one command on the GPU box via gpurun; re-submit ONLY when the box could not be acquired
# (status=transient / rc 3: nothing ran, nothing charged). A command that ran is never retried.
# usage: tools/gpu.sh <timeout_s> '<command>'
T=$1; shift
for attempt in 1 2 3 4; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpurun_last.log 2>&1
  rc=$?
  if grep -q "status=transient" /tmp/gpurun_last.log || [ $rc -eq 3 ]; then
    echo "[gpu.sh] box not acquired (attempt $attempt), waiting" >&2
    sleep 45
    continue
  fi
  break
done
tail -3 /tmp/gpurun_last.log
exit $rc
