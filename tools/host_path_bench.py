#!/usr/bin/env python3
"""host_path_bench.py — throughput of the verify path when records start in HOST memory (PCIe-inclusive),
the case a Rust server handing over its own buffers is in:

  * sync   : one at2v_verify_batch call per batch (H2D, kernel, D2H serialised on one stream);
  * queue  : the ingest queue (at2v_queue_*), which overlaps the upload of batch k+1 with the verify of
             batch k on separate streams.

Records are generated on the GPU (at2v_gen_records_device) and copied to host once, untimed.
usage: python tools/host_path_bench.py [--n 4194304] [--batch 262144]   -> one JSON line
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "at2-node_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 22)
    ap.add_argument("--batch", type=int, default=1 << 18)
    ap.add_argument("--msg-len", type=int, default=100)
    a = ap.parse_args()
    import numpy as np
    import torch

    import at2v
    from at2v.node import IngestQueue

    n, L, B = a.n, a.msg_len, a.batch
    v = at2v.BatchVerifier(device=0)
    dev = "cuda:0"
    d_pk = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_sig = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    d_msg = torch.empty(n * L, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    v.gen_records_device(0x4154325F, 0, n, L, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), None, s)
    torch.cuda.synchronize()
    pk = d_pk.cpu().numpy().reshape(n, 32)
    sig = d_sig.cpu().numpy().reshape(n, 64)
    msg = d_msg.cpu().numpy()
    del d_pk, d_sig, d_msg
    off = (np.arange(B + 1, dtype=np.uint64) * L).astype(np.uint32)
    out = {"metric": "host-buffer verify throughput (PCIe-inclusive)", "n": n, "batch": B, "msg_len": L}

    # sync: one call per batch
    v.verify_batch(pk[:B], sig[:B], msg[:B * L], off)  # warm
    t0 = time.perf_counter()
    ok = 0
    for b0 in range(0, n, B):
        ok += int(v.verify_batch(pk[b0:b0 + B], sig[b0:b0 + B], msg[b0 * L:(b0 + B) * L], off).sum())
    dt = time.perf_counter() - t0
    out["sync"] = {"verifies_per_s": n / dt, "seconds": dt, "all_valid": ok == n}
    v.close()

    # queue: batches sealed at B records, depth 3 (upload/verify/download overlapped)
    with IngestQueue(device=0, max_batch=B, max_delay_us=200, max_msg_bytes=L, depth=3) as q:
        q.submit(pk[:B], sig[:B], msg[:B * L], off)  # warm
        q.flush()
        got = 0
        while got < B:
            t, _ = q.poll(1 << 20, 100000)
            got += len(t)
        t0 = time.perf_counter()
        for b0 in range(0, n, B):
            q.submit(pk[b0:b0 + B], sig[b0:b0 + B], msg[b0 * L:(b0 + B) * L], off)
        q.flush()
        got, valid = 0, 0
        while got < n:
            t, vv = q.poll(1 << 20, 100000)
            got += len(t)
            valid += int(vv.sum())
        dt = time.perf_counter() - t0
        out["queue"] = {"verifies_per_s": n / dt, "seconds": dt, "all_valid": valid == n, "stats": q.stats()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
