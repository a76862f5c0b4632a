"""GPU: the pieces around the verify kernel, through the C ABI of libat2v.so —
  * at2v_decode_points (GPU dalek decompression check) vs the oracle;
  * the ingest/batching queue (HIP backend) vs the oracle, with concurrent producers and every flush path;
  * end to end: wire SendAssetRequests -> packer -> recipient decode -> queue verify -> ledger apply, for
    the config-1 AT2 traffic with corrupted signatures mixed in (balances checked against a direct
    computation from the records the oracle accepts);
  * BASELINE config 4 at full size: 1M adversarial records, bit-exact against the oracle."""
import ctypes
import json
import os
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def at2v_mod():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import at2v
    return at2v


@pytest.fixture(scope="module")
def verifier(at2v_mod):
    v = at2v_mod.BatchVerifier(device=0)
    yield v
    v.close()


def test_decode_points_matches_oracle(verifier, oracle, golden):
    oracle.L.oracle_decompress_ok.argtypes = [ctypes.c_void_p]
    oracle.L.oracle_decompress_ok.restype = ctypes.c_int
    rng = np.random.default_rng(3)
    pts = [g.pk for g in golden.values()] + [rng.integers(0, 256, (3000, 32), dtype=np.uint8)]
    pts += [np.frombuffer(b"".join(oracle.small_order_encoding(i) for i in range(14)), np.uint8).reshape(14, 32)]
    pts = np.concatenate(pts)
    got = verifier.decode_points(pts)
    want = np.array([bool(oracle.L.oracle_decompress_ok(p.tobytes())) for p in pts])
    assert np.array_equal(got, want)
    assert 0 < want.sum() < len(want)
    assert verifier.decode_points(np.zeros((0, 32), np.uint8)).size == 0


def _drain(q, n, timeout_s=60):
    tickets, verdicts = [], []
    t0 = time.time()
    while sum(len(t) for t in tickets) < n and time.time() - t0 < timeout_s:
        t, v = q.poll(65536, 20000)
        tickets.append(t)
        verdicts.append(v)
    return np.concatenate(tickets), np.concatenate(verdicts)


def test_queue_matches_oracle_with_concurrent_producers(at2v_mod, oracle):
    from at2v.node import IngestQueue
    n, L = 20000, 100
    pk, sig, msg, off, cls = oracle.gen_adversarial(0x77, 0, n, L)
    want = oracle.verify_batch(pk, sig, msg, off)
    ticket_of = np.full(n, -1, np.int64)
    with IngestQueue(device=0, max_batch=4096, max_delay_us=500, max_msg_bytes=128, depth=3) as q:
        lock = threading.Lock()
        nxt = [0]

        def producer(seed):
            rng = np.random.default_rng(seed)
            while True:
                with lock:
                    a = nxt[0]
                    m = int(rng.integers(1, 700))
                    nxt[0] += m
                if a >= n:
                    return
                b = min(n, a + m)
                first = q.submit(pk[a:b], sig[a:b], msg[a * L:b * L], off[a:b + 1] - off[a])
                ticket_of[a:b] = np.arange(first, first + (b - a))

        th = [threading.Thread(target=producer, args=(s,)) for s in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        q.flush()
        tickets, verdicts = _drain(q, n)
        st = q.stats()
    assert len(tickets) == n and np.array_equal(tickets, np.arange(n))  # every ticket, in order
    assert (ticket_of >= 0).all()
    assert not (verdicts == 0xFF).any()
    got = verdicts[ticket_of] == 1
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    assert st["completed"] == n and st["batches"] >= n // 4096


def test_queue_deadline_flush_small_batches(at2v_mod, oracle):
    from at2v.node import IngestQueue
    pk, sig, msg, off = oracle.gen_records(0x78, 0, 40, 48)
    with IngestQueue(device=0, max_batch=65536, max_delay_us=2000, max_msg_bytes=64, depth=2) as q:
        t0 = time.time()
        q.submit(pk[:10], sig[:10], msg[:480], off[:11])  # never fills: sealed by the deadline
        t, v = _drain(q, 10, 10)
        dt = time.time() - t0
        assert len(t) == 10 and v.all() and dt < 5
        first = q.submit(pk[10:], sig[10:], msg[480:], off[10:] - off[10])
        q.flush()
        t, v = _drain(q, 30, 10)
        assert list(t) == list(range(first, first + 30)) and v.all()
        st = q.stats()
    assert st["batches"] == 2 and st["p50_us"] > 0


def test_end_to_end_config1_pack_verify_apply(at2v_mod, verifier, oracle):
    """config 1 (4096 AT2 send-asset txs) through the whole host path, 1 in 16 signatures corrupted"""
    from at2v.node import IngestQueue, Ledger, SendAssetRequest, pack_send_asset, wire_key, wire_signature
    pk, sig, msg, off, snd, seq = oracle.gen_at2_transactions()
    n = len(seq)
    sig = sig.copy()
    bad = np.arange(n) % 16 == 5
    sig[bad, 40] ^= 0x10
    reqs = []
    for i in range(n):
        m = msg[off[i]:off[i + 1]].tobytes()
        reqs.append(SendAssetRequest(wire_key(pk[i].tobytes()), int(seq[i]), wire_key(m[8:40]),
                                     int.from_bytes(m[40:48], "little"), wire_signature(sig[i].tobytes())))
    rec = pack_send_asset(reqs)
    assert (rec["status"] == 0).all()
    assert verifier.decode_points(rec["recipient"]).all()  # rpc.rs:265 recipient decode
    with IngestQueue(device=0, max_batch=1024, max_delay_us=1000, max_msg_bytes=48, depth=3) as q:
        first = q.submit(rec["pk"], rec["sig"], rec["msg"], rec["off"])
        q.flush()
        t, v = _drain(q, n)
    assert np.array_equal(t, np.arange(first, first + n))
    want = oracle.verify_batch(rec["pk"], rec["sig"], rec["msg"], rec["off"])
    assert set(np.unique(v)) <= {0, 1}
    assert np.array_equal(v == 1, want) and (want == ~bad).all()
    led = Ledger()
    st = led.deliver(rec["pk"], rec["sequence"], rec["recipient"], rec["amount"], v)  # queue bytes, fail closed
    assert st["rejected"] == bad.sum()
    # expected: per sender, sequences apply up to the first rejected one (a gap blocks the rest)
    bal = {}
    for i in range(n):
        bal.setdefault(pk[i].tobytes(), 100000)
    applied = np.zeros(n, bool)
    order = np.lexsort((seq, snd))
    blocked = set()
    for i in order:
        s = int(snd[i])
        if bad[i]:
            blocked.add(s)
        elif s not in blocked:
            applied[i] = True
    for i in np.nonzero(applied)[0]:
        a = int(rec["amount"][i])
        bal[pk[i].tobytes()] -= a
        r = rec["recipient"][i].tobytes()
        bal[r] = bal.get(r, 100000) + a
    assert st["applied"] == applied.sum() and led.pending() == (~bad & ~applied).sum()
    for k, b in bal.items():
        assert led.balance(k) == b
    led.close()


def test_config4_adversarial_1m_bit_exact(verifier, oracle):
    """BASELINE config 4: 1M records, 10% adversarial classes (bit flips, S+l, high S bits, non-canonical
    R, small-order and mixed-order A incl. crafted accepting cases, off-curve A), device path, vs the oracle"""
    import torch
    n, L = 1 << 20, 100
    threads = min(16, os.cpu_count() or 1)
    t0 = time.time()
    pk, sig, msg, off, cls = oracle.gen_adversarial(0xC0F4, 0, n, L, threads=threads)
    t_gen = time.time() - t0
    dev = "cuda:0"
    d_pk = torch.from_numpy(pk.reshape(-1)).to(dev)
    d_sig = torch.from_numpy(sig.reshape(-1)).to(dev)
    d_msg = torch.from_numpy(msg).to(dev)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_ver = torch.zeros(n // 32, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    verifier.verify_batch_device(d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), n * L, d_off.data_ptr(), n,
                                 d_ver.data_ptr(), s)
    torch.cuda.synchronize()
    import at2v
    got = at2v.unpack_verdicts(d_ver.cpu().numpy().view(np.uint32), n)
    t0 = time.time()
    want = oracle.verify_batch(pk, sig, msg, off, 0, threads)
    t_oracle = time.time() - t0
    mism = int((got != want).sum())
    per_class = {int(c): {"n": int((cls == c).sum()), "valid": int(want[cls == c].sum()),
                          "mismatch": int((got[cls == c] != want[cls == c]).sum())} for c in np.unique(cls)}
    summary = {"config": "BASELINE config 4: adversarial 1M", "n": n, "valid": int(want.sum()), "mismatches": mism,
               "verdict_match": 1.0 - mism / n, "per_class": per_class, "oracle_threads": threads,
               "gen_s": round(t_gen, 2), "oracle_s": round(t_oracle, 2)}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "config4_adversarial.json"), "w") as fp:
        json.dump(summary, fp, indent=1)
    assert mism == 0, summary
    assert 0.85 * n < want.sum() < 0.95 * n
