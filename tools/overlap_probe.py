#!/usr/bin/env python3
"""Does the next batch's launch fill the end-of-launch drain of the previous one?  (DESIGN §5 load balance)

Back-to-back verify launches of config 2 batches (1M records each), timed over K launches with a sync on both sides:
  serial:   one context, one stream (every launch waits for the previous one: the drain is paid per batch);
  overlap2: two contexts (two scratch sets), two streams, launches alternate, so launch k+1's blocks take the CUs
            launch k's blocks leave;
  big:      one launch of 2x the records (the drain paid once per 2M), for reference.
Rounds interleave the modes in one process. Prints M verifies/s per mode (median over rounds)."""
import argparse
import ctypes
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
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--streams", default="torch", choices=["torch", "prio", "hip"])
    a = ap.parse_args()
    torch.cuda.set_device(0)
    n, L, K = a.n, 100, a.k
    vs = [at2v.BatchVerifier(device=0) for _ in range(2)]
    if a.streams == "torch":
        streams = [torch.cuda.Stream() for _ in range(2)]
    elif a.streams == "prio":
        streams = [torch.cuda.Stream(priority=0), torch.cuda.Stream(priority=-1)]
    else:  # raw HIP streams (non-blocking), wrapped for torch
        hip = ctypes.CDLL("libamdhip64.so")
        streams = []
        for _ in range(2):
            h = ctypes.c_void_p()
            assert hip.hipStreamCreateWithFlags(ctypes.byref(h), 1) == 0
            streams.append(torch.cuda.ExternalStream(h.value))
    d_pk = torch.empty(2 * n * 32, dtype=torch.uint8, device="cuda")
    d_sig = torch.empty(2 * n * 64, dtype=torch.uint8, device="cuda")
    d_msg = torch.empty(2 * n * L, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(2 * n + 1, dtype=torch.int32, device="cuda")
    vers = [torch.zeros(2 * n // 32, dtype=torch.int32, device="cuda") for _ in range(2)]
    s0 = torch.cuda.current_stream()
    vs[0].gen_records_device(0x4154325F, 0, 2 * n, L, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                             d_off.data_ptr(), s0.cuda_stream)
    torch.cuda.synchronize()
    P = (d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr())

    def run(mode):
        for v in vers:
            v.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode == "serial":
            for k in range(K):
                vs[0].verify_batch_device(*P, n * L, d_off.data_ptr(), n, vers[0].data_ptr(), streams[0].cuda_stream)
        elif mode == "overlap2":
            for k in range(K):
                j = k & 1
                vs[j].verify_batch_device(*P, n * L, d_off.data_ptr(), n, vers[j].data_ptr(), streams[j].cuda_stream)
        else:  # big: K/2 launches of 2n
            for k in range(K // 2):
                vs[0].verify_batch_device(*P, 2 * n * L, d_off.data_ptr(), 2 * n, vers[0].data_ptr(),
                                          streams[0].cuda_stream)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        m = n // 32
        ok = bool((vers[0][:m] == -1).all().item()) and (mode != "overlap2" or bool((vers[1][:m] == -1).all().item()))
        return K * n / dt / 1e6, ok

    modes = ["serial", "overlap2", "big"]
    res = {m: [] for m in modes}
    for r in range(a.rounds + 1):
        for m in modes:
            rate, ok = run(m)
            assert ok, f"{m}: wrong verdicts"
            if r:
                res[m].append(rate)
    for m in modes:
        x = np.array(res[m])
        print(f"{m:9s} median {np.median(x):8.2f} M verifies/s  (min {x.min():.2f} max {x.max():.2f}, {K} x {n})")


if __name__ == "__main__":
    main()
