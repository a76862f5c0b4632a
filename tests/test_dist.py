"""CPU: the multi-rank verdict path (shard bounds + all-gather of verdict words) with world_size 2 on
gloo, exactly as bench.py / a node with one process per GPU uses it over RCCL. Verdict words are
produced by the oracle here (CPU), standing in for each rank's GPU launch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from at2v import dist as at2dist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_bounds_cover_and_align():
    for n in (1, 63, 64, 65, 1000, 4096, 1 << 20, 16_777_216):
        for world in (1, 2, 3, 4, 8):
            b = at2dist.shard_bounds(n, world)
            assert b[0][0] == 0 and b[-1][1] == n
            for (lo, hi), (lo2, _) in zip(b, b[1:]):
                assert hi == lo2 or hi == n
            assert all(lo % 64 == 0 or lo == n for lo, _ in b)
            per = at2dist.padded_words_per_rank(n, world)
            assert all(hi - lo <= per * 32 for lo, hi in b)


def _worker(rank, world, port, n, pk, sig, msg, off, want, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle_py

    o = oracle_py.Oracle()
    lo, hi = at2dist.shard_bounds(n, world)[rank]
    per = at2dist.padded_words_per_rank(n, world)
    words = np.zeros(per, np.uint32)
    if hi > lo:
        v = o.verify_batch(pk[lo:hi], sig[lo:hi], msg, off[lo:hi + 1], 0, 2)
        bits = np.zeros(per * 32, np.uint8)
        bits[: hi - lo] = v
        words = np.packbits(bits, bitorder="little").view(np.uint32)
    local = torch.from_numpy(words.view(np.int32).copy())
    full = at2dist.gather_verdicts(local, world)
    got = at2dist.node_bitmap_from_shards(full, n, world)
    q.put((rank, bool(np.array_equal(got, want))))
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [1000, 4096])
def test_gloo_world2_gather_matches_oracle(golden, n):
    g = golden["adversarial"]
    pk, sig, msg, off = g.pk[:n], g.sig[:n], g.msg, g.off[: n + 1]
    want = g.dalek[:n]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, pk, sig, msg, off, want, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True)]
