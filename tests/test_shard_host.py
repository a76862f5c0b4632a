"""CPU: the index-range sharding of at2-node_amd/csrc/at2v_shard.h — the code at2v_verify_batch_sharded /
at2v_verify_shard_gather_device (one process per GPU + RCCL all-gather) and at2v_verify_batch with num_gpus > 1
(one process, several devices) run — compiled for the host and checked against at2v/dist.py (shard_bounds,
padded_words_per_rank, node_bitmap_from_shards) for world / G = 1..8 and ragged n, including n not a multiple of 64
and ranks with no records. The multi-device paths themselves have not run on more than one GPU (1-GPU pool)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from at2v import dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NS = [0, 1, 2, 31, 32, 33, 63, 64, 65, 127, 128, 129, 1000, 4095, 4096, 4097, 65535, 65536, 65537, 1 << 20,
      (1 << 20) + 17, 16 * (1 << 20) + 17]
SZ = ctypes.c_size_t


@pytest.fixture(scope="module")
def sh():
    so = os.path.join(ROOT, "tests", "host", "shard_host.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I" + os.path.join(ROOT, "at2-node_amd", "csrc"),
                    os.path.join(ROOT, "tests", "host", "shard_host.cpp"), "-o", so], check=True)
    L = ctypes.CDLL(so)
    L.sh_per_rank.restype = SZ
    L.sh_per_rank.argtypes = [SZ, ctypes.c_int]
    L.sh_words_per_rank.restype = SZ
    L.sh_words_per_rank.argtypes = [SZ, ctypes.c_int]
    P = ctypes.POINTER(SZ)
    L.sh_rank_range.argtypes = [SZ, ctypes.c_int, ctypes.c_int, P, P]
    L.sh_rank_words.argtypes = [SZ, ctypes.c_int, ctypes.c_int, P, P, P]
    L.sh_device_range.argtypes = [SZ, SZ, SZ, P, P]
    L.sh_offsets_valid.argtypes = [ctypes.c_void_p, SZ]
    L.sh_rebase.argtypes = [ctypes.c_void_p, SZ, SZ, ctypes.c_void_p]
    return L


def _range(L, n, w, r):
    lo, hi = SZ(), SZ()
    L.sh_rank_range(n, w, r, ctypes.byref(lo), ctypes.byref(hi))
    return lo.value, hi.value


@pytest.mark.parametrize("world", range(1, 9))
def test_rank_ranges_match_dist_py(sh, world):
    for n in NS:
        want = dist.shard_bounds(n, world)
        got = [_range(sh, n, world, r) for r in range(world)]
        if n:
            assert got == want, (n, world)
            assert sh.sh_words_per_rank(n, world) == dist.padded_words_per_rank(n, world)
        else:  # an empty node batch still all-gathers 2 zero words per rank (RCCL needs a count > 0)
            assert got == [(0, 0)] * world and sh.sh_words_per_rank(0, world) == 2
        per = sh.sh_per_rank(n, world)
        assert per % 64 == 0 and per * world >= n
        # contiguous cover of [0, n), 64-aligned starts
        assert got[0][0] == 0 and got[-1][1] == n
        for (a, b), (c, _) in zip(got, got[1:]):
            assert b == c and (a % 64 == 0 or a == n)


@pytest.mark.parametrize("world", [2, 3, 5, 8])
def test_gathered_word_placement_reassembles_bitmap(sh, world):
    """rank q's words land at word lo_q/32 of the caller's array (at2v_verify_batch_sharded's D2H copies); the result
    equals dist.node_bitmap_from_shards of the rank-major gathered words, for random verdicts"""
    rng = np.random.default_rng(world)
    for n in NS[:-1]:
        bits = rng.integers(0, 2, n).astype(np.uint8)
        wpr = sh.sh_words_per_rank(n, world)
        gathered = np.zeros(world * wpr, np.uint32)
        for q in range(world):
            lo, hi = _range(sh, n, world, q)
            slab = np.zeros(wpr * 32, np.uint8)
            slab[:hi - lo] = bits[lo:hi]
            gathered[q * wpr:(q + 1) * wpr] = np.packbits(slab, bitorder="little").view(np.uint32)
        out = np.zeros((n + 31) // 32, np.uint32)
        for q in range(world):
            d, s, k = SZ(), SZ(), SZ()
            sh.sh_rank_words(n, world, q, ctypes.byref(d), ctypes.byref(s), ctypes.byref(k))
            assert s.value == q * wpr
            out[d.value:d.value + k.value] = gathered[s.value:s.value + k.value]
        got = np.unpackbits(out.view(np.uint8), bitorder="little")[:n]
        assert np.array_equal(got, bits), (n, world)
        if n:
            assert np.array_equal(dist.node_bitmap_from_shards(gathered.view(np.int32), n, world), bits.astype(bool))


@pytest.mark.parametrize("G", range(1, 9))
def test_device_ranges_cover_in_whole_chunks(sh, G):
    for n in NS:
        rs = []
        for g in range(G):
            lo, hi = SZ(), SZ()
            sh.sh_device_range(n, G, g, ctypes.byref(lo), ctypes.byref(hi))
            rs.append((lo.value, hi.value))
        assert rs[0][0] == 0 and rs[-1][1] == n
        chunks = (n + 63) // 64
        for g, (a, b) in enumerate(rs):
            assert a % 64 == 0 and a <= b
            # balanced: shard sizes differ by at most one chunk (the last may be ragged)
            assert (b - a + 63) // 64 in (chunks // G, chunks // G + 1)
        for (a, b), (c, _) in zip(rs, rs[1:]):
            assert b == c


def test_offsets_check_and_rebase(sh):
    rng = np.random.default_rng(1)
    lens = rng.integers(0, 300, 1000)
    off = np.concatenate([[7], 7 + np.cumsum(lens)]).astype(np.uint32)
    assert sh.sh_offsets_valid(off.ctypes.data, 1000) == 1
    for a, m in [(0, 1000), (64, 100), (999, 1), (500, 0)]:
        out = np.zeros(m + 1, np.uint32)
        sh.sh_rebase(off.ctypes.data, a, m, out.ctypes.data)
        assert np.array_equal(out, off[a:a + m + 1] - off[a])
    bad = off.copy()
    bad[600] = bad[599] - 1  # one decreasing offset anywhere in the batch: every rank rejects the whole batch
    assert sh.sh_offsets_valid(bad.ctypes.data, 1000) == 0
    assert sh.sh_offsets_valid(off.ctypes.data, 0) == 1
