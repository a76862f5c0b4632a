"""Multi-GPU plumbing for the at2v verdict bitmap.

One process per GPU. A node-level batch of n records is split by contiguous index range into
`world` shards, each a multiple of 64 records (one wave chunk = two verdict words), so every rank's
verdict words land at a word-aligned offset of the node bitmap and one all-gather of equal-sized
word buffers (RCCL over xGMI when the group backend is "nccl") returns the full bitmap on every rank.
There is no other data-path collective: verification itself is embarrassingly parallel.
"""
from __future__ import annotations

from typing import List, Tuple

CHUNK = 64  # records per wave chunk


def shard_bounds(n: int, world: int) -> List[Tuple[int, int]]:
    """[lo, hi) record range of every rank: contiguous, 64-aligned starts, equal padded size."""
    per = -(-n // world)           # ceil
    per = -(-per // CHUNK) * CHUNK  # round up to a chunk
    return [(min(n, r * per), min(n, (r + 1) * per)) for r in range(world)]


def padded_words_per_rank(n: int, world: int) -> int:
    """verdict words each rank contributes to the all-gather (equal counts; pad bits are 0)."""
    lo, hi = shard_bounds(n, world)[0]
    per = -(-n // world)
    per = -(-per // CHUNK) * CHUNK
    return per // 32


def gather_verdicts(local_words, world: int, group=None):
    """All-gather equal-sized per-rank verdict word tensors (int32) into the node bitmap.

    local_words: 1-D int32 tensor of padded_words_per_rank() words on this rank's device.
    Returns a tensor of world * len(local_words) words (rank r's words at offset r * len)."""
    import torch
    import torch.distributed as dist

    out = torch.empty(world * local_words.numel(), dtype=local_words.dtype, device=local_words.device)
    dist.all_gather_into_tensor(out, local_words.contiguous(), group=group)
    return out


def bitmap_to_bool(words, n: int):
    """node bitmap words (torch int32 or numpy) -> numpy bool[n]"""
    import numpy as np

    w = words.cpu().numpy() if hasattr(words, "cpu") else words
    bits = np.unpackbits(np.ascontiguousarray(w).view(np.uint8), bitorder="little")
    return bits[:n].astype(bool)


def node_bitmap_from_shards(words, n: int, world: int):
    """Gathered padded words (rank-major) -> bool[n] in global record order."""
    import numpy as np

    per_words = padded_words_per_rank(n, world)
    w = words.cpu().numpy() if hasattr(words, "cpu") else np.asarray(words)
    out = np.zeros(n, dtype=bool)
    for r, (lo, hi) in enumerate(shard_bounds(n, world)):
        if hi <= lo:
            continue
        seg = w[r * per_words:(r + 1) * per_words]
        out[lo:hi] = bitmap_to_bool(seg, hi - lo)
    return out
