#!/usr/bin/env python3
"""abi_probe.py — the library's host-buffer call (at2v_verify_batch on pageable numpy arrays) under chunk-schedule
variants, for tuning the HostPipe staging (at2v_api.hip). Each variant sets the test hooks AT2V_TEST_STAGE_FIRST /
AT2V_TEST_STAGE_MAX / AT2V_TEST_COPY_THREADS (AT2V_TEST_HOOKS=1) before creating its context; variants alternate over
`--rounds` rounds so box drift hits them alike. Also prints the device-API kernel time of the same batch and a
single-thread numpy copy rate of the batch (host memory bandwidth).
usage: python tools/abi_probe.py [--n 1048576] [--calls 8] [--rounds 2] [--variants first:max:threads[:streams[:staged]],...]
-> one JSON line"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "at2-node_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--calls", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--msg-len", type=int, default=100)
    ap.add_argument("--variants", default="32768:131072:8")
    ap.add_argument("--host-only", action="store_true", help="skip the device-API timings (for kernel traces)")
    ap.add_argument("--lib", default="", help="a libat2v variant (tools/build_variant.sh) instead of the product")
    a = ap.parse_args()
    os.environ["AT2V_TEST_HOOKS"] = "1"
    if "--trace" in sys.argv[1:] or os.environ.get("ABI_PROBE_TRACE"):
        os.environ["AT2V_TEST_PIPE_TRACE"] = "1"
    import numpy as np
    import torch

    import at2v

    if a.lib:
        at2v.load_library(a.lib)
    n, L = a.n, a.msg_len
    dev = "cuda:0"
    g = at2v.BatchVerifier()
    s = torch.cuda.current_stream().cuda_stream
    d_pk = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_sig = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    d_msg = torch.empty(n * L, dtype=torch.uint8, device=dev)
    d_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    d_ver = torch.empty((n + 31) // 32, dtype=torch.int32, device=dev)
    g.gen_records_device(0x4154325F, 0, n, L, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(), s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.verify_batch_device(d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), n * L, d_off.data_ptr(), n,
                          d_ver.data_ptr(), s)
    e0.record()
    for _ in range(3):
        g.verify_batch_device(d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), n * L, d_off.data_ptr(), n,
                              d_ver.data_ptr(), s)
    e1.record()
    torch.cuda.synchronize()
    kernel_ms = e0.elapsed_time(e1) / 3
    # the same 1M records as back-to-back device-API launches of `sub` records (one stream, and two streams whose
    # launches may overlap): what chunking a batch into launches costs without any host work
    subs = {}
    ls = at2v.launch_streams(2)
    for sub in () if a.host_only else (65536, 131072, 262144, 524288):
        for nst in (1, 2):
            e0.record(ls[0])
            ls[1].wait_event(e0)
            ends = []
            for k in range(n // sub):
                st = ls[k % nst]
                g.verify_batch_device(d_pk.data_ptr() + k * sub * 32, d_sig.data_ptr() + k * sub * 64, d_msg.data_ptr(),
                                      n * L, d_off.data_ptr() + k * sub * 4, sub, d_ver.data_ptr() + k * sub // 8,
                                      st.cuda_stream)
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(st)
                ends.append(ev)
            torch.cuda.synchronize()
            subs[f"{sub}x{nst}"] = max(e0.elapsed_time(e) for e in ends)
    print(f"[abi_probe] device-API 1M as launches of sub records (ms): {subs}", file=sys.stderr, flush=True)
    # cold records: four distinct 1M batches (800 MB, beyond the 256 MB MALL) verified round robin, against the same
    # batch re-verified (the headline bench's case: its 200 MB stay MALL-resident)
    cold = []
    for b in range(0 if a.host_only else 4):
        bufs = [torch.empty(n * 32, dtype=torch.uint8, device=dev), torch.empty(n * 64, dtype=torch.uint8, device=dev),
                torch.empty(n * L, dtype=torch.uint8, device=dev), torch.empty(n + 1, dtype=torch.int32, device=dev)]
        g.gen_records_device(0x4154325F, (b + 1) * n, n, L, *(x.data_ptr() for x in bufs), s)
        cold.append(bufs)
    torch.cuda.synchronize()
    e0.record()
    for k in range(8 if cold else 0):
        b = cold[k % 4]
        g.verify_batch_device(b[0].data_ptr(), b[1].data_ptr(), b[2].data_ptr(), n * L, b[3].data_ptr(), n,
                              d_ver.data_ptr(), s)
    e1.record()
    torch.cuda.synchronize()
    cold_ms = e0.elapsed_time(e1) / 8 if cold else 0.0
    del cold
    print(f"[abi_probe] device-API kernel: hot {kernel_ms:.3f} ms, cold {cold_ms:.3f} ms", file=sys.stderr, flush=True)
    # the same launch after the device sat idle (a host-buffer call's copies leave it so between calls): clock ramp
    gaps = {}
    for gap_ms in (0.0, 1.0, 3.0, 6.0):
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            time.sleep(gap_ms / 1e3)
            e0.record()
            g.verify_batch_device(d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), n * L, d_off.data_ptr(), n,
                                  d_ver.data_ptr(), s)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        gaps[gap_ms] = sorted(ts)[2]
    print(f"[abi_probe] device-API kernel after an idle gap (ms -> ms): {gaps}", file=sys.stderr, flush=True)
    pk, sig, msg = d_pk.cpu().numpy(), d_sig.cpu().numpy(), d_msg.cpu().numpy()
    off = d_off.cpu().numpy().view(np.uint32)
    g.close()
    tmp = np.empty(n * (96 + L), np.uint8)
    src = np.concatenate([pk, sig, msg])
    t0 = time.perf_counter()
    np.copyto(tmp, src)
    copy_gbs = src.nbytes / (time.perf_counter() - t0) / 1e9
    words = np.zeros(n // 32 + 1, np.uint32)
    out = {"n": n, "kernel_ms_after_gap": gaps, "kernel_ms_device_api": kernel_ms, "kernel_ms_device_api_cold": cold_ms, "device_api_split_ms": subs, "numpy_copy_gbs_1thread": copy_gbs, "variants": {}}
    for r in range(a.rounds):
        for var in a.variants.split(","):
            first, mx, th, ps, st = (var.split(":") + ["1", "0"])[:5]
            os.environ["AT2V_TEST_PIPE_STREAMS"] = ps
            os.environ["AT2V_TEST_STAGED"] = st  # 1: the staged single launch, 0: chunk launches
            os.environ["AT2V_TEST_STAGE_FIRST"] = first
            os.environ["AT2V_TEST_STAGE_MAX"] = mx
            os.environ["AT2V_TEST_COPY_THREADS"] = th
            v = at2v.BatchVerifier()
            lib = v._lib
            ptrs = (pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, off.ctypes.data)
            assert lib.at2v_verify_batch(v._h, *ptrs, n, words.ctypes.data) == 0
            times = []
            for _ in range(a.calls):
                t0 = time.perf_counter()
                assert lib.at2v_verify_batch(v._h, *ptrs, n, words.ctypes.data) == 0
                times.append((time.perf_counter() - t0) * 1e3)
            ok = bool((words[: n // 32] == 0xFFFFFFFF).all())
            chunks = v.info()["host_chunks"]
            v.close()
            d = out["variants"].setdefault(var, {"ms": [], "ok": True})
            d["ms"].append(sorted(times)[len(times) // 2])
            d["ok"] &= ok
            d["chunks_per_call"] = chunks / (a.calls + 1)
            print(f"[abi_probe] round {r} {var}: median {d['ms'][-1]:.3f} ms (min {min(times):.3f}) ok={ok}",
                  file=sys.stderr, flush=True)
    for var, d in out["variants"].items():
        d["best_ms"] = min(d["ms"])
        d["rate_mps"] = n / d["best_ms"] / 1e3
        d["vs_kernel"] = kernel_ms / d["best_ms"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
