#!/usr/bin/env python3
"""cache_debug.py — per-launch sender-cache counters for the sliding-window workload of tests/test_gpu_cache.py
test_senders_4x_capacity (diagnostics; prints one line per launch)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "at2-node_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import at2v
    import test_gpu_cache as t
    S, L = 256, 48
    pk, sig, msg, off = t._gen_senders(at2v, S * 16, L, S)
    snd = np.arange(S * 16) % S
    for comb in (False, True):
        for small in (0xFFFFFFFF, 0):
            with at2v.BatchVerifier(small_batch_max=small, sender_cache=64, sender_comb=comb) as v:
                for launch in range(6):
                    window = set(((np.arange(64) + 16 * launch) % S).tolist())
                    idx = np.array(sorted((i for i in range(S * 16) if snd[i] in window), key=lambda i: (snd[i], i)))
                    m2 = np.concatenate([msg[off[i]:off[i + 1]] for i in idx])
                    o2 = (np.arange(len(idx) + 1) * L).astype(np.uint32)
                    h0 = v.info()
                    got = v.verify_batch(pk[idx], sig[idx], m2, o2)
                    h1 = v.info()
                    d = {k: h1[k] - h0[k] for k in ("cache_chunks", "cache_chunk_hits", "cache_claims", "cache_evicted",
                                                     "cache_compactions")}
                    print(f"comb={comb} small={small:#x} launch {launch}: all valid {bool(got.all())} {d} "
                          f"entries {h1['cache_entries']}", flush=True)


if __name__ == "__main__":
    main()
