#!/usr/bin/env python3
"""bcomb_build_probe.py — context creation with per-sender combs (VERDICT r5 "Next" 3): the combs of B (16-bit and
20-bit windows, or 24-bit with AT2V_CTX_BCOMB_WIDE) are built by additions in short launches and shared by the contexts
of a process. Prints one JSON line: creation time of a first comb context, of a second one (shares the tables), of a
wide one, and of one after all were closed (builds again). Run under rocprofv3 --kernel-trace --stats for the launch
durations (bcomb_base_kernel / bcomb_fill_kernel)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "at2-node_amd"))


def main():
    import torch  # noqa: F401

    import at2v
    out = {}

    def make(**kw):
        t0 = time.perf_counter()
        v = at2v.BatchVerifier(device=0, sender_cache=1024, sender_comb=True, **kw)
        return v, time.perf_counter() - t0

    plain, out["plain_context_s"] = (lambda t0: (at2v.BatchVerifier(device=0), time.perf_counter() - t0))(
        time.perf_counter())
    a, out["first_comb_context_s"] = make()
    b, out["second_comb_context_s"] = make()
    w, out["wide_comb_context_s"] = make(bcomb_wide=True)
    for v in (a, b, w):
        v.close()
    c, out["comb_context_after_close_s"] = make()
    c.close()
    plain.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
