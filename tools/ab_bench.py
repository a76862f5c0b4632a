#!/usr/bin/env python3
"""A/B kernel-time comparison of libat2v builds, interleaved rounds in ONE process (guide rule 24).
usage: python3 tools/ab_bench.py lib1.so lib2.so ... [--n 1048576] [--rounds 5]
Also checks every build returns all-valid verdicts for the generated batch."""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "at2-node_amd"))
import at2v  # noqa: E402


class Opts(ctypes.Structure):  # include/at2v.h at2v_opts (ABI v6)
    _fields_ = [("device", ctypes.c_int), ("num_gpus", ctypes.c_int), ("policy", ctypes.c_int),
                ("small_batch_max", ctypes.c_uint32), ("sender_cache", ctypes.c_uint32), ("sender_comb", ctypes.c_uint32),
                ("cpu_threads", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


def open_lib(path, comb=False, wide=False):
    lib = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL)
    P = ctypes.c_void_p
    lib.at2v_create.argtypes = [P, ctypes.POINTER(P)]
    lib.at2v_verify_batch_device.argtypes = [P, P, P, P, ctypes.c_size_t, P, ctypes.c_size_t, P, P]
    lib.at2v_gen_records_senders_device.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t,
                                                    ctypes.c_uint32, ctypes.c_uint64, P, P, P, P, P]
    h = P()
    o = Opts(0, 1, 0, 0, 1024 if comb else 0, 1 if comb else 0, 0, 4 if (comb and wide) else 0)
    assert lib.at2v_create(ctypes.byref(o), ctypes.byref(h)) == 0
    return lib, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--msg-len", type=int, default=100)
    ap.add_argument("--no-check", action="store_true", help="perf-only experiment builds: skip the verdict check")
    ap.add_argument("--senders", type=int, default=0, help="records signed by this many repeating senders (0 = distinct)")
    ap.add_argument("--comb", action="store_true", help="contexts with sender_cache 1024 + sender_comb (AT2 traffic)")
    ap.add_argument("--wide", action="store_true", help="with --comb: the wide comb of B (AT2V_CTX_BCOMB_WIDE)")
    ap.add_argument("--probe", action="store_true",
                    help="builds with -DAT2V_COMB_PROBE: print the comb kernel's per-wait cycle sums (rounds 2..)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    n, L = a.n, a.msg_len
    libs = [open_lib(p, a.comb, a.wide) for p in a.libs]
    s = torch.cuda.current_stream()
    d_pk = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    d_sig = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    d_msg = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(n + 1, dtype=torch.int32, device="cuda")
    d_ver = torch.zeros((n + 31) // 32, dtype=torch.int32, device="cuda")
    lib0, h0 = libs[0]
    assert lib0.at2v_gen_records_senders_device(h0, 0x4154325F, 0, n, L, a.senders, d_pk.data_ptr(), d_sig.data_ptr(),
                                                d_msg.data_ptr(), d_off.data_ptr(), s.cuda_stream) == 0
    torch.cuda.synchronize()
    times = {p: [] for p in a.libs}
    for r in range(a.rounds + 1):
        for p, (lib, h) in zip(a.libs, libs):
            d_ver.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            assert lib.at2v_verify_batch_device(h, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), n * L,
                                                d_off.data_ptr(), n, d_ver.data_ptr(), s.cuda_stream) == 0
            e1.record(s)
            torch.cuda.synchronize()
            ok = bool((d_ver == -1).all().item())
            if r > 0:
                times[p].append(e0.elapsed_time(e1))
            assert ok or a.no_check, f"{p}: wrong verdicts"
        if a.probe and r == 1:  # the warm-up launches (sighting, claims) are not counted
            for lib, _ in libs:
                if hasattr(lib, "at2v_probe_read"):
                    probe_read(lib)
    for p in a.libs:
        t = np.array(times[p])
        print(f"{os.path.basename(p):28s} median {np.median(t):8.3f} ms  min {t.min():8.3f}  -> {n / np.median(t) / 1e3:8.2f} M verifies/s")
    if a.probe:
        for p, (lib, _) in zip(a.libs, libs):
            if hasattr(lib, "at2v_probe_read"):
                print_probe(os.path.basename(p), probe_read(lib))


PROBE_NAMES = ["A-comb entry waits (vmcnt)", "B-comb entry waits (vmcnt)", "stage refill waits (lgkmcnt)",
               "record loads + prechecks", "SHA-512 + recode (msg loads incl.)", "comb additions (waits incl.)",
               "slot + inversion + encodes", "list loads + verdicts + ticket", "chunk total", "chunks",
               "comb-entry LDS reads (lgkmcnt, forced)", "slot + R loads in the finish (vmcnt, forced)"]


def probe_read(lib):
    buf = (ctypes.c_ulonglong * 16)()
    k = lib.at2v_probe_read(buf, 16)
    assert k > 0, k
    return [int(buf[i]) for i in range(k)]


def print_probe(name, v):
    """the comb kernel's wave-cycle sums (s_memtime) per phase and wait, as a share of the chunk total"""
    tot, chunks = v[8], max(1, v[9])
    print(f"probe {name}: {chunks} chunks of 256 records, {tot / chunks:.0f} wave-cycles per chunk")
    for i in list(range(8)) + list(range(10, len(v))):
        print(f"  {PROBE_NAMES[i]:36s} {100.0 * v[i] / max(1, tot):6.2f} %  ({v[i] / chunks:10.0f} cycles per chunk)")


if __name__ == "__main__":
    main()
