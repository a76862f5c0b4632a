#!/usr/bin/env python3
"""Where the end-to-end (pinned host buffers) rate goes below the kernel rate: times, on one GPU and 1M records per
step, (a) kernel only, (b) uploads only (4 arrays, copy stream), (c) upload + kernel serial, (d) pipelined (uploads
of step k+1 on a copy stream under the kernel of step k), each over --steps steps. Prints one JSON object."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "at2-node_amd"))
import at2v  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    n, L = a.n, 100
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    v = at2v.BatchVerifier(device=0)
    st = torch.cuda.current_stream(dev)
    s = st.cuda_stream
    d = [torch.empty(n * 32, dtype=torch.uint8, device=dev), torch.empty(n * 64, dtype=torch.uint8, device=dev),
         torch.empty(n * L, dtype=torch.uint8, device=dev), torch.empty(n + 1, dtype=torch.int32, device=dev)]
    ver = torch.zeros(n // 32, dtype=torch.int32, device=dev)
    v.gen_records_device(0x4154325F, 0, n, L, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), s)
    torch.cuda.synchronize()
    h = [t.cpu().pin_memory() for t in d]
    sets = [[torch.empty_like(t) for t in d] for _ in range(2)]
    copy = torch.cuda.Stream(dev)
    h_out = torch.empty(ver.numel(), dtype=torch.int32).pin_memory()

    def verify(b, strm):
        v.verify_batch_device(b[0].data_ptr(), b[1].data_ptr(), b[2].data_ptr(), n * L, b[3].data_ptr(), n,
                              ver.data_ptr(), strm)

    def upload(b, strm):
        with torch.cuda.stream(strm):
            for x, y in zip(b, h):
                x.copy_(y, non_blocking=True)

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e3

    out = {"n": n, "steps": a.steps}
    verify(d, s)
    upload(sets[0], copy)
    upload(sets[1], copy)
    torch.cuda.synchronize()
    out["kernel_ms"] = timed(lambda: [verify(d, s) for _ in range(a.steps)])
    out["upload_ms"] = timed(lambda: [upload(sets[k % 2], copy) for k in range(a.steps)])
    out["upload_gbs"] = sum(t.numel() * t.element_size() for t in d) / out["upload_ms"] / 1e6

    def serial():
        for _ in range(a.steps):
            upload(sets[0], st)
            verify(sets[0], s)
            with torch.cuda.stream(st):
                h_out.copy_(ver, non_blocking=True)
    out["serial_ms"] = timed(serial)

    def piped():
        up = [torch.cuda.Event() for _ in range(2)]
        free = [torch.cuda.Event() for _ in range(2)]
        for e in free:
            e.record(st)
        for k in range(a.steps):
            b = sets[k % 2]
            copy.wait_event(free[k % 2])
            upload(b, copy)
            up[k % 2].record(copy)
            st.wait_event(up[k % 2])
            verify(b, s)
            free[k % 2].record(st)
            with torch.cuda.stream(st):
                h_out.copy_(ver, non_blocking=True)
    out["pipelined_ms"] = timed(piped)
    for k in ("kernel_ms", "serial_ms", "pipelined_ms"):
        out[k.replace("_ms", "_Mps")] = n / out[k] / 1e3
    out["verdicts_ok"] = bool((h_out == -1).all())
    v.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
