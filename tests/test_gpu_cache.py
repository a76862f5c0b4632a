"""GPU: the per-sender A cache (at2v_opts.sender_cache; VERDICT r2 item 6, SURVEY §7 "reusing per-sender A tables").

AT2 senders issue consecutive sequences (/root/reference/src/bin/server/accounts/account.rs:36-43), so one key signs many
payloads of a node batch (client.rs:77-78). With the cache on, a wave whose 64 records all find their A in the cache
(fingerprint nominates an entry, then all 32 key bytes are compared) skips decoding A and building [j]A. The verdict
must stay a pure function of (A, R||S, M): every test here compares with the oracle or the golden fixtures, through
the C ABI, in every cache state — key claimed in this launch (entry still being built on the build stream: the launch
verifies it without the cache), warm, fingerprint collisions (forced with AT2V_TEST_CACHE_FP_BITS), cache full
(compaction: the least recently used entries are replaced), undecodable / small-order / non-canonical senders cached
together with their decode verdict, and both policies. Every test runs twice: with the [j]A tables (sender_comb off) and
with per-key combs (sender_comb on: all-hit chunks verify by table additions only, at2v_comb.h). `v.info()` waits for the
context's build stream, so a launch after it finds every key claimed before it built and valid."""
import os

import numpy as np
import pytest

import golden_io

pytestmark = pytest.mark.gpu

CFG_SEED = 0x4154325F
OFF = 0xFFFFFFFF  # small_batch_max: the cache serves the throughput kernel, so run it at every size


@pytest.fixture(params=[False, True], ids=["tables", "comb"])
def comb(request):
    return request.param


@pytest.fixture(scope="module")
def at2v_mod():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import at2v
    return at2v


def _mutate(pk, sig, msg, off, rng, k, kinds=4):
    """k records mutated in R, S, M or A (a bit flip; kinds=3: never A): each then has exactly one verdict the oracle
    decides"""
    pk, sig, msg = pk.copy(), sig.copy(), msg.copy()
    for i in rng.choice(len(pk), k, replace=False):
        kind = rng.integers(0, kinds)
        if kind == 0:
            sig[i, rng.integers(0, 32)] ^= 1 << rng.integers(0, 8)
        elif kind == 1:
            sig[i, 32 + rng.integers(0, 31)] ^= 1 << rng.integers(0, 8)
        elif kind == 2 and off[i + 1] > off[i]:
            msg[off[i] + rng.integers(0, off[i + 1] - off[i])] ^= 1
        else:
            pk[i, rng.integers(0, 32)] ^= 1 << rng.integers(0, 8)
    return pk, sig, msg


def test_config1_traffic_every_chunk_hits(at2v_mod, oracle, comb):
    """BASELINE config 1 traffic (64 senders x sequences 1..64): every entry is built by the first launch's build pass,
    so every chunk of every launch takes the cached path; verdicts equal the oracle's, mutated records included."""
    pk, sig, msg, off, snd, seq = oracle.gen_at2_transactions()
    rng = np.random.default_rng(3)
    pk2, sig2, msg2 = _mutate(pk, sig, msg, off, rng, 300)
    want = oracle.verify_batch(pk, sig, msg, off)
    want2 = oracle.verify_batch(pk2, sig2, msg2, off)
    assert want.all() and 0 < want2.sum() < len(want2)
    with at2v_mod.BatchVerifier(small_batch_max=OFF, sender_cache=1024, sender_comb=comb, admit_first=True) as v:
        assert np.array_equal(v.verify_batch(pk, sig, msg, off), want)  # claims the 64 senders, verified uncached
        info = v.info()  # (waits for the build stream: the 64 entries are built and valid)
        assert info["cache_entries"] == 64 and info["cache_claims"] == 64
        assert info["cache_chunks"] == 64 and info["cache_chunk_hits"] == 0
        assert np.array_equal(v.verify_batch(pk, sig, msg, off), want)  # every chunk from the cache
        info = v.info()
        assert info["cache_chunks"] == 2 * 64 and info["cache_chunk_hits"] == 64
        got2 = v.verify_batch(pk2, sig2, msg2, off)  # mutated A's are new keys: new entries, some undecodable
        assert np.array_equal(got2, want2), np.nonzero(got2 != want2)[0][:10]
        assert v.info()["cache_entries"] > 64
        assert np.array_equal(v.verify_batch(pk2, sig2, msg2, off), want2)  # ... now cached, undecodable ones too


@pytest.mark.parametrize("policy", ["dalek", "libsodium"])
def test_golden_sets_with_cache(at2v_mod, golden, policy, comb):
    """every golden fixture set, three times (cold: first sightings; second pass: admission claims and builds; third:
    warm), both policies, with the default admission: the small-order, non-canonical and off-curve senders of the
    adversarial/edge sets are cached with their decode verdicts and served from the cache (default 20-bit comb of B on
    the hit list with combs; [j]A tables without) — ADVICE r5: two passes never reached the warm path"""
    # 16,384 keys hold every set's senders (<= 9,200 distinct); with combs that is 16,384 x 1.7 MB = 28 GB of HBM
    with at2v_mod.BatchVerifier(policy=policy, small_batch_max=OFF, sender_cache=1 << 14, sender_comb=comb) as v:
        for name in golden_io.SETS:
            g = golden[name]
            want = g.dalek if policy == "dalek" else g.sodium
            for rep in range(3):
                h0 = v.info()["cache_record_hits"]
                got = v.verify_batch(g.pk, g.sig, g.msg, g.off)
                assert np.array_equal(got, want), (name, rep, np.nonzero(got != want)[0][:10])
                hits = v.info()["cache_record_hits"] - h0  # (waits for the build stream: this pass's claims are built)
            assert hits > 0.9 * g.n, (name, hits, g.n)  # the warm pass: (nearly) every record from the cache


def test_repeated_adversarial_senders(at2v_mod, oracle, comb):
    """an adversarial batch whose senders repeat: 512 distinct records (every class of config 4) tiled 32x with fresh
    mutations, so entries for small-order / undecodable keys are hit by many records"""
    pk, sig, msg, off, cls = oracle.gen_adversarial(CFG_SEED + 21, 0, 512, 100)
    L = 100
    pk_t = np.tile(pk, (32, 1))
    sig_t = np.tile(sig, (32, 1))
    msg_t = np.tile(msg, 32)
    off_t = (np.arange(512 * 32 + 1) * L).astype(np.uint32)
    pk_t, sig_t, msg_t = _mutate(pk_t, sig_t, msg_t, off_t, np.random.default_rng(5), 1500)
    want = oracle.verify_batch(pk_t, sig_t, msg_t, off_t)
    with at2v_mod.BatchVerifier(small_batch_max=OFF, sender_cache=4096, sender_comb=comb) as v:
        for rep in range(3):
            got = v.verify_batch(pk_t, sig_t, msg_t, off_t)
            assert np.array_equal(got, want), (rep, np.nonzero(got != want)[0][:10])
            if rep == 1:
                v.info()


def test_fingerprint_collisions_fall_back(at2v_mod, oracle, monkeypatch, comb):
    """3 fingerprint bits (test hook): distinct senders share fingerprints, so the lookup nominates entries of other
    keys; the byte comparison must send those waves down the uncached path with identical verdicts"""
    monkeypatch.setenv("AT2V_TEST_CACHE_FP_BITS", "3")
    pk, sig, msg, off, snd, seq = oracle.gen_at2_transactions()
    pk2, sig2, msg2 = _mutate(pk, sig, msg, off, np.random.default_rng(7), 200)
    want = oracle.verify_batch(pk2, sig2, msg2, off)
    with at2v_mod.BatchVerifier(small_batch_max=OFF, sender_cache=1024, sender_comb=comb) as v:
        for rep in range(3):
            assert np.array_equal(v.verify_batch(pk2, sig2, msg2, off), want)
            v.info()
        info = v.info()
        assert info["cache_entries"] <= 4 and info["cache_chunk_hits"] < info["cache_chunks"]


def test_cache_full_compacts(at2v_mod, oracle, comb):
    """capacity 16 < 64 senders: the first launch hands out all 16 payloads (the other claims stay without one), so
    the cache is compacted before a later launch (at most 3/4 of the entries stay, the least recently used go back to
    the free list); verdicts exact throughout, the cache never holds more than its capacity."""
    pk, sig, msg, off, snd, seq = oracle.gen_at2_transactions()
    pk2, sig2, msg2 = _mutate(pk, sig, msg, off, np.random.default_rng(9), 100)
    want = oracle.verify_batch(pk2, sig2, msg2, off)
    with at2v_mod.BatchVerifier(small_batch_max=OFF, sender_cache=16, sender_comb=comb, admit_first=True) as v:
        for rep in range(5):
            assert np.array_equal(v.verify_batch(pk2, sig2, msg2, off), want), rep
            assert v.info()["cache_entries"] <= 16
        info = v.info()
        assert info["cache_chunk_hits"] < info["cache_chunks"]  # waves had senders left out
        assert info["cache_compactions"] >= 1 and info["cache_evicted"] >= 1 and info["cache_capacity"] == 16, info


def _gen_senders(at2v_mod, n, L, senders):
    """n valid records (GPU generator), record i signed by sender i % senders, as host arrays"""
    import torch
    dev = "cuda:0"
    d_pk = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
    d_sig = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
    d_msg = torch.zeros(n * L, dtype=torch.uint8, device=dev)
    d_off = torch.zeros(n + 1, dtype=torch.int32, device=dev)
    with at2v_mod.BatchVerifier() as g:
        g.gen_records_device(CFG_SEED, 0, n, L, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(),
                             torch.cuda.current_stream().cuda_stream, senders=senders)
        torch.cuda.synchronize()
    return (d_pk.cpu().numpy().reshape(n, 32), d_sig.cpu().numpy().reshape(n, 64), d_msg.cpu().numpy(),
            d_off.cpu().numpy().astype(np.uint32))


def test_senders_4x_capacity(at2v_mod, oracle, comb):
    """VERDICT r3 "Next" 5: 4x more senders than the cache holds. 256 senders, capacity 64; launch k carries the 1024
    records (16 per sender, 4 senders per 64-record chunk) of the 64 senders in a window that slides by 16 senders per
    launch over the 256, mutated, so
    a quarter of the working set changes every launch and the whole sender set cycles through the cache 3 times.
    Verdicts equal the oracle's in every launch; the cache compacts (least recently used entries replaced) instead of
    restarting empty, it never holds more than 64 keys, and the senders still in the window hit (hit rate printed)."""
    S, L = 256, 48
    pk, sig, msg, off = _gen_senders(at2v_mod, S * 16, L, S)
    snd = np.arange(S * 16) % S
    rng = np.random.default_rng(17)
    hits, chunks = [], []
    with at2v_mod.BatchVerifier(small_batch_max=OFF, sender_cache=64, sender_comb=comb) as v:
        for launch in range(12):
            window = set(((np.arange(64) + 16 * launch) % S).tolist())
            # grouped by sender (a 64-record chunk holds 4 senders), so chunks of cached senders hit
            idx = np.array(sorted((i for i in range(S * 16) if snd[i] in window), key=lambda i: (snd[i], i)))
            p2, s2 = pk[idx], sig[idx]
            m2 = np.concatenate([msg[off[i]:off[i + 1]] for i in idx])
            o2 = (np.arange(len(idx) + 1) * L).astype(np.uint32)
            p2, s2, m2 = _mutate(p2, s2, m2, o2, rng, 40, kinds=3)  # (a mutated A is one more sender)
            want = oracle.verify_batch(p2, s2, m2, o2)
            h0 = v.info()
            got = v.verify_batch(p2, s2, m2, o2)
            assert np.array_equal(got, want), (launch, np.nonzero(got != want)[0][:10])
            h1 = v.info()
            hits.append(h1["cache_chunk_hits"] - h0["cache_chunk_hits"])
            chunks.append(h1["cache_chunks"] - h0["cache_chunks"])
            assert h1["cache_entries"] <= 64
        info = v.info()
        print(f"4x senders: chunk hit rate {sum(hits)}/{sum(chunks)}, per launch {hits}; {info}")
        assert info["cache_compactions"] >= 2 and info["cache_evicted"] >= 64, info
        assert sum(hits) > 0, hits


def test_generator_with_repeating_senders(at2v_mod, oracle):
    """at2v_gen_records_senders_device: record i signed by sender i % senders, M_i per record, all valid (oracle)"""
    import torch
    n, L, S = 4096, 100, 64
    dev = "cuda:0"
    d_pk = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
    d_sig = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
    d_msg = torch.zeros(n * L, dtype=torch.uint8, device=dev)
    d_off = torch.zeros(n + 1, dtype=torch.int32, device=dev)
    with at2v_mod.BatchVerifier() as v:
        v.gen_records_device(CFG_SEED, 0, n, L, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(),
                             torch.cuda.current_stream().cuda_stream, senders=S)
        torch.cuda.synchronize()
    pk = d_pk.cpu().numpy().reshape(n, 32)
    sig = d_sig.cpu().numpy().reshape(n, 64)
    msg = d_msg.cpu().numpy()
    off = d_off.cpu().numpy().astype(np.uint32)
    assert (pk == np.tile(pk[:S], (n // S, 1))).all() and len({bytes(r) for r in pk[:S]}) == S
    assert oracle.verify_batch(pk, sig, msg, off).all()
    # the sender keys are the distinct-key generator's keys 0..S-1
    with at2v_mod.BatchVerifier() as v:
        d2 = torch.zeros(S * 32, dtype=torch.uint8, device=dev)
        ds = torch.zeros(S * 64, dtype=torch.uint8, device=dev)
        dm = torch.zeros(S * L, dtype=torch.uint8, device=dev)
        v.gen_records_device(CFG_SEED, 0, S, L, d2.data_ptr(), ds.data_ptr(), dm.data_ptr(), None,
                             torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    assert (d2.cpu().numpy().reshape(S, 32) == pk[:S]).all()


LAT_SLICES = (1, 63, 65, 640, 4096, 32_768)  # launch sizes <= AT2V_SMALL_BATCH_DEFAULT: the four-wave comb kernel


def _slices(n, rng):
    """cut [0, n) into launches whose sizes cycle through LAT_SLICES (every one <= the default small_batch_max)"""
    out, a, k = [], 0, int(rng.integers(0, len(LAT_SLICES)))
    while a < n:
        b = min(n, a + LAT_SLICES[k % len(LAT_SLICES)])
        out.append((a, b))
        a, k = b, k + 1
    return out


def _verify_slice(v, g, a, b):
    o = g.off[a:b + 1]
    return v.verify_batch(g.pk[a:b], g.sig[a:b], g.msg[o[0]:o[-1]], (o - o[0]).astype(np.uint32))


@pytest.mark.parametrize("policy", ["dalek", "libsodium"])
def test_golden_sets_comb_lat_kernel(at2v_mod, golden, policy):
    """VERDICT r3 "Next" 1: every golden set through verify_comb_lat_kernel, the four-wave kernel whose verdict rule is
    a projective comparison of R' with the decoded R (at2v_comb.h comb_check_split) instead of dalek's byte compare.
    Default small_batch_max, sender_comb on, each set cut into launches of 1..32,768 records (every one takes the
    four-wave kernel), cold (the launch that first sees a key builds its comb, then verifies from it) and warm; the
    edge / adversarial sets carry non-canonical R, x = 0 with the sign bit, small-order and off-curve R and A."""
    rng = np.random.default_rng(11)
    with at2v_mod.BatchVerifier(policy=policy, sender_cache=1 << 14, sender_comb=True, admit_first=True) as v:
        for name in golden_io.SETS:
            g = golden[name]
            want = g.dalek if policy == "dalek" else g.sodium
            for rep in range(2):
                h0 = v.info()  # (the second pass finds the first pass's keys built)
                got = np.concatenate([_verify_slice(v, g, a, b) for a, b in _slices(g.n, rng)])
                assert np.array_equal(got, want), (name, rep, np.nonzero(got != want)[0][:10])
                h1 = v.info()
                chunks, hits = h1["cache_chunks"] - h0["cache_chunks"], h1["cache_chunk_hits"] - h0["cache_chunk_hits"]
                if rep == 0:  # cold: a chunk with a key not seen before runs the two-wave half-size split
                    assert hits < chunks, (name, h1)
                else:  # warm: every chunk takes the comb branch of the four-wave kernel
                    assert chunks > 0 and hits == chunks, (name, h1)


def test_comb_lat_kernel_mixed_hit_and_fallback_chunks(at2v_mod, oracle, golden):
    """one four-wave launch whose chunks mix all-hit comb chunks with chunks that hold senders beyond the cache's
    capacity (their claims stay invalid): those chunks take wave 0's half-size ladder beside the comb chunks of the same
    grid. Verdicts equal the oracle's / golden's, in three cache states (warm, full, restarted)."""
    pk, sig, msg, off, snd, seq = oracle.gen_at2_transactions()  # 64 senders
    g = golden["adversarial"]
    rng = np.random.default_rng(13)
    # records: [cfg1 64 | adversarial 64 | cfg1 64 | ...]: 16 chunks of each kind, adversarial keys mostly distinct
    L = 48
    n_ad = 16 * 64
    ad = rng.choice(g.n, n_ad, replace=False)
    parts_pk, parts_sig, parts_msg, lens = [], [], [], []
    for c in range(32):
        if c % 2 == 0:
            idx = np.arange((c // 2) * 64, (c // 2) * 64 + 64) % len(pk)
            parts_pk.append(pk[idx]); parts_sig.append(sig[idx])
            parts_msg += [msg[off[i]:off[i + 1]] for i in idx]
        else:
            idx = ad[(c // 2) * 64:(c // 2) * 64 + 64]
            parts_pk.append(g.pk[idx]); parts_sig.append(g.sig[idx])
            parts_msg += [g.msg[g.off[i]:g.off[i + 1]] for i in idx]
    P = np.concatenate(parts_pk)
    S = np.concatenate(parts_sig)
    M = np.concatenate(parts_msg) if parts_msg else np.zeros(0, np.uint8)
    O = np.concatenate([[0], np.cumsum([len(m) for m in parts_msg])]).astype(np.uint32)
    want = oracle.verify_batch(P, S, M, O)
    assert 0 < want.sum() < len(want)
    # capacity 96: the 64 cfg1 senders fit, most adversarial keys do not (their chunks fall back)
    with at2v_mod.BatchVerifier(sender_cache=96, sender_comb=True, admit_first=True) as v:
        assert np.array_equal(v.verify_batch(pk, sig, msg, off), oracle.verify_batch(pk, sig, msg, off))  # warm
        h0 = v.info()  # (waits for the 64 senders' combs)
        for rep in range(3):
            got = v.verify_batch(P, S, M, O)
            assert np.array_equal(got, want), (rep, np.nonzero(got != want)[0][:10])
        info = v.info()
        chunks = info["cache_chunks"] - h0["cache_chunks"]
        hits = info["cache_chunk_hits"] - h0["cache_chunk_hits"]
        assert 0 < hits < chunks, info  # both branches ran in the same launches


@pytest.mark.parametrize("n", [1, 20, 64, 100, 2048, 40_000])
def test_comb_small_and_ragged_launches(at2v_mod, oracle, n):
    """with combs on, launches of every size take the comb kernel (the low-latency pair kernel is not used): config-1
    traffic cut to n records, mutated, cold then warm, against the oracle"""
    pk, sig, msg, off, snd, seq = oracle.gen_at2_transactions()
    reps = (n + len(pk) - 1) // len(pk)
    L = 48
    pk = np.tile(pk, (reps, 1))[:n]
    sig = np.tile(sig, (reps, 1))[:n]
    msg = np.tile(msg, reps)[: n * L]
    off = (np.arange(n + 1) * L).astype(np.uint32)
    # (R, S and M mutations only: 4,000 mutated keys would be 4,000 more senders than the 64 whose chunks should hit)
    pk, sig, msg = _mutate(pk, sig, msg, off, np.random.default_rng(n), max(1, n // 10), kinds=3)
    want = oracle.verify_batch(pk, sig, msg, off)
    with at2v_mod.BatchVerifier(sender_cache=1024, sender_comb=True, admit_first=True) as v:
        for rep in range(2):
            got = v.verify_batch(pk, sig, msg, off)
            assert np.array_equal(got, want), (rep, np.nonzero(got != want)[0][:10])
            info = v.info()
        assert info["cache_chunk_hits"] > 0


@pytest.mark.parametrize("n", [2048, 40000])
def test_device_launches_while_combs_build(at2v_mod, oracle, golden, n):
    """VERDICT r3 "Next" 4, the chunks whose comb is still building: device launches on a caller stream go back to back,
    so the second and third launch of the same records start while the context's stream may still be building the
    combs the first launch claimed. Their chunks then find entries that are claimed but not valid and fall back to the
    half-size check. n = 2048: the four-wave kernel; n = 40000: the four-records-per-lane throughput kernel. Records
    from 64 senders with every fourth one mutated (oracle verdicts), plus the adversarial golden set the same way."""
    import torch
    rng = np.random.default_rng(n)
    pk, sig, msg, off = _gen_senders(at2v_mod, n, 100, 64)
    sig = sig.copy()
    bad = rng.choice(n, n // 4, replace=False)
    sig[bad, 3] ^= 0x10  # R changes: those records must be rejected
    want = oracle.verify_batch(pk, sig, msg, off)
    g = golden["adversarial"]
    sets = [(pk, sig, msg, off, want), (g.pk, g.sig, g.msg, g.off, g.dalek)]
    stream = torch.cuda.Stream()
    for (p_, s_, m_, o_, w_) in sets:
        m = len(p_)
        with at2v_mod.BatchVerifier(sender_cache=1024, sender_comb=True) as v:
            d = [torch.from_numpy(np.array(x, copy=True).reshape(-1)).cuda() for x in (p_, s_)]
            d_msg = torch.from_numpy(np.concatenate([m_, np.zeros(16, np.uint8)])).cuda()
            d_off = torch.from_numpy(np.array(o_, copy=True).view(np.int32)).cuda()
            outs = [torch.zeros((m + 31) // 32, dtype=torch.int32, device="cuda") for _ in range(3)]
            torch.cuda.synchronize()
            for o in outs:  # back to back on one caller stream: no wait for the context's comb builds
                v.verify_batch_device(d[0].data_ptr(), d[1].data_ptr(), d_msg.data_ptr(), int(o_[-1]), d_off.data_ptr(),
                                      m, o.data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize()
            for k, o in enumerate(outs):
                got = at2v_mod.unpack_verdicts(o.cpu().numpy().view(np.uint32), m)
                assert np.array_equal(got, w_), (m, k, np.nonzero(got != w_)[0][:10])
            v.info()  # combs built: a fourth launch takes the comb path where every key is cached
            last = torch.zeros((m + 31) // 32, dtype=torch.int32, device="cuda")
            v.verify_batch_device(d[0].data_ptr(), d[1].data_ptr(), d_msg.data_ptr(), int(o_[-1]), d_off.data_ptr(), m,
                                  last.data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize()
            got = at2v_mod.unpack_verdicts(last.cpu().numpy().view(np.uint32), m)
            assert np.array_equal(got, w_)


# ---------------------------------------------------------------- round 5: admission, asynchronous compaction


def test_admission_one_shot_senders_claim_nothing(at2v_mod, oracle, comb):
    """VERDICT r4 "missing" 3: distinct keys through a cache context. Every key is seen once, so none claims a payload
    (no build, no compaction): the launch records sightings only. Seen again in a later launch, a key claims; verdicts
    equal the oracle's throughout."""
    n, L = 20_000, 100
    pk, sig, msg, off = _gen_senders(at2v_mod, n, L, 0)
    pk2, sig2, msg2 = _mutate(pk, sig, msg, off, np.random.default_rng(41), 500)
    want = oracle.verify_batch(pk2, sig2, msg2, off)
    with at2v_mod.BatchVerifier(small_batch_max=OFF, sender_cache=1024, sender_comb=comb) as v:
        assert np.array_equal(v.verify_batch(pk2, sig2, msg2, off), want)
        info = v.info()
        distinct = len({bytes(r) for r in pk2})
        assert info["cache_claims"] == 0 and info["cache_compactions"] == 0, info
        assert info["cache_sightings"] == distinct, (info, distinct)
        assert np.array_equal(v.verify_batch(pk2, sig2, msg2, off), want)  # second sighting: claims (and fills up)
        info = v.info()
        assert info["cache_claims"] >= 1024, info
        for _ in range(2):
            assert np.array_equal(v.verify_batch(pk2, sig2, msg2, off), want)
        assert v.info()["cache_entries"] <= 1024


def test_admission_repeating_senders_become_hits(at2v_mod, oracle, comb):
    """config-1 traffic (sender = record % 64, so no chunk holds a key twice): the first launch only sights most keys,
    the next claims them, and from the third launch on every chunk hits; mutated records keep the oracle's verdicts."""
    pk, sig, msg, off, snd, seq = oracle.gen_at2_transactions()
    pk2, sig2, msg2 = _mutate(pk, sig, msg, off, np.random.default_rng(43), 200, kinds=3)
    want = oracle.verify_batch(pk2, sig2, msg2, off)
    with at2v_mod.BatchVerifier(small_batch_max=OFF, sender_cache=1024, sender_comb=comb) as v:
        rates = []
        for rep in range(4):
            h0 = v.info()
            assert np.array_equal(v.verify_batch(pk2, sig2, msg2, off), want), rep
            h1 = v.info()
            rates.append((h1["cache_chunk_hits"] - h0["cache_chunk_hits"], h1["cache_chunks"] - h0["cache_chunks"]))
        info = v.info()
    print("admission, hits per launch:", rates, info)
    assert info["cache_claims"] == 64 and info["cache_sightings"] >= 1, info
    assert rates[0][0] == 0 and rates[3][0] == rates[3][1] == 64, rates


# (without combs, launches up to small_batch_max take the pair kernel, which does not use the cache: no tables-lat case)
@pytest.mark.parametrize("comb,small", [(False, OFF), (True, OFF), (True, 0)],
                         ids=["tables-throughput", "comb-throughput", "comb-lat"])
def test_compaction_while_launches_overlap_on_two_streams(at2v_mod, oracle, comb, small):
    """device launches alternate over two streams (the two scratch sets let them overlap) while a
    16-key cache fills and compacts again and again. A compaction runs on the context's stream; launches issued meanwhile
    read the old table and claim nothing, and the first launch after it swaps the tables. Every launch's verdicts equal
    the oracle's (a launch that probed a half-built table or popped a payload still held by a kept key would verify
    records against another key's comb or table)."""
    import torch
    pk, sig, msg, off, snd, seq = oracle.gen_at2_transactions()  # 64 senders > 16 keys of capacity
    rng = np.random.default_rng(47)
    batches = []
    for k in range(6):  # six record sets: the same 64 senders, different mutations (some rejected)
        p2, s2, m2 = _mutate(pk, sig, msg, off, rng, 150)
        batches.append((p2, s2, m2, oracle.verify_batch(p2, s2, m2, off)))
    n = len(pk)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    dev = [tuple(torch.from_numpy(np.array(x, copy=True).reshape(-1)).cuda() for x in b[:3]) for b in batches]
    d_off = torch.from_numpy(off.view(np.int32).copy()).cuda()
    with at2v_mod.BatchVerifier(small_batch_max=small, sender_cache=16, sender_comb=comb, admit_first=True) as v:
        outs = []
        for launch in range(36):
            b = launch % len(batches)
            st = streams[launch % 2]
            o = torch.zeros((n + 31) // 32, dtype=torch.int32, device="cuda")
            d_pk, d_sig, d_msg = dev[b]
            v.verify_batch_device(d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), int(off[-1]), d_off.data_ptr(),
                                  n, o.data_ptr(), st.cuda_stream)
            outs.append((b, o))
            if launch % 4 == 3:
                streams[0].synchronize()  # the host sees the counters' copies: compactions start while stream 1 runs
        torch.cuda.synchronize()
        for k, (b, o) in enumerate(outs):
            got = at2v_mod.unpack_verdicts(o.cpu().numpy().view(np.uint32), n)
            want = batches[b][3]
            assert np.array_equal(got, want), (k, np.nonzero(got != want)[0][:10])
        info = v.info()
    print("two-stream compactions:", info)
    assert info["cache_compactions"] >= 2 and info["cache_entries"] <= 16, info


def test_partitioned_mixed_traffic_record_hits(at2v_mod, oracle, comb):
    """Round 5's partitioned launch: records of 64 cached senders shuffled with records of fresh keys (adversarial set),
    so no 64- or 256-record chunk is all-cached. The classify kernel sends every record of a cached sender down the
    cached path anyway (hit list: comb additions, or [j]A tables) and the rest down the ladder; verdicts equal the
    oracle's, and the cached-record count equals the number of records signed by the 64 senders."""
    pk, sig, msg, off, snd, seq = oracle.gen_at2_transactions()
    p1, s1, m1 = _mutate(pk, sig, msg, off, np.random.default_rng(53), 150, kinds=3)
    pa, sa, ma, oa, cls = oracle.gen_adversarial(CFG_SEED + 57, 0, 4096, 48)
    P = np.concatenate([p1, pa])
    S = np.concatenate([s1, sa])
    msgs = [m1[off[i]:off[i + 1]] for i in range(len(p1))] + [ma[oa[i]:oa[i + 1]] for i in range(len(pa))]
    perm = np.random.default_rng(59).permutation(len(P))
    P, S = P[perm], S[perm]
    msgs = [msgs[i] for i in perm]
    M = np.concatenate(msgs)
    O = np.concatenate([[0], np.cumsum([len(m) for m in msgs])]).astype(np.uint32)
    want = oracle.verify_batch(P, S, M, O)
    assert 0 < want.sum() < len(want)
    cfg1_keys = {bytes(r) for r in pk[:64]}
    n_cfg1 = sum(bytes(r) in cfg1_keys for r in P)
    with at2v_mod.BatchVerifier(small_batch_max=OFF, sender_cache=1 << 14, sender_comb=comb, admit_first=True) as v:
        assert np.array_equal(v.verify_batch(pk, sig, msg, off), oracle.verify_batch(pk, sig, msg, off))
        h0 = v.info()  # (waits for the 64 senders' entries)
        got = v.verify_batch(P, S, M, O)
        assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
        h1 = v.info()
        hits = h1["cache_record_hits"] - h0["cache_record_hits"]
        assert hits >= n_cfg1, (hits, n_cfg1)
        assert h1["cache_chunk_hits"] - h0["cache_chunk_hits"] < (h1["cache_chunks"] - h0["cache_chunks"]) // 4
        for _ in range(2):  # the adversarial keys are cached now too (admit_first): more hits, same verdicts
            assert np.array_equal(v.verify_batch(P, S, M, O), want)
        assert v.info()["cache_record_hits"] - h1["cache_record_hits"] > 2 * hits


@pytest.mark.parametrize("partition", ["0", "1"])
def test_partition_switch_same_verdicts(at2v_mod, golden, monkeypatch, comb, partition):
    """AT2V_CACHE_PARTITION=0 keeps round 4's in-kernel lookup for launches above small_batch_max (A/B switch): both
    forms give the golden verdicts, cold and warm"""
    monkeypatch.setenv("AT2V_CACHE_PARTITION", partition)
    g = golden["adversarial"]
    with at2v_mod.BatchVerifier(small_batch_max=OFF, sender_cache=4096, sender_comb=comb) as v:
        for rep in range(3):
            assert np.array_equal(v.verify_batch(g.pk, g.sig, g.msg, g.off), g.dalek), rep
            v.info()


@pytest.mark.parametrize("wide", [False, True], ids=["bcomb20", "bcomb24"])
def test_comb_hits_staged_and_unstaged_messages(at2v_mod, oracle, wide):
    """The comb hit loop stages a record's message in LDS when every lane's message fits the stage (length up to ~150
    bytes) and ends 8 bytes before the buffer end; any other wave reads word by word (comb2_point_staged returns -1).
    64 cached senders, 4,096 records with message lengths 0..199 at every byte alignment (so some 64-record waves fit
    and some do not), mutated records, and the last records' messages ending exactly at the buffer end: verdicts equal
    the oracle's on the cold launch and on the warm (all-hit) ones."""
    rng = np.random.default_rng(97)
    S, n = 64, 4096
    seeds = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(S)]
    keys = [oracle.public_key(s) for s in seeds]
    lens = rng.integers(0, 200, n)
    lens[: n // 2] = rng.integers(0, 140, n // 2)  # the first half: waves that all fit (the staged path)
    msgs = [bytes(rng.integers(0, 256, int(k), dtype=np.uint8)) for k in lens]
    snd = rng.integers(0, S, n)
    pk = np.array([np.frombuffer(keys[s], np.uint8) for s in snd])
    sig = np.array([np.frombuffer(oracle.sign(seeds[s], m), np.uint8) for s, m in zip(snd, msgs)])
    msg = np.frombuffer(b"".join(msgs), np.uint8).copy()
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint32)
    bad = rng.choice(n, 300, replace=False)
    sig[bad[:150], 5] ^= 0x10  # R changes
    for i in bad[150:]:  # M changes (a byte inside, when there is one)
        if lens[i]:
            msg[off[i] + rng.integers(0, lens[i])] ^= 0x01
    want = oracle.verify_batch(pk, sig, msg, off)
    assert 0 < want.sum() < n
    with at2v_mod.BatchVerifier(small_batch_max=OFF, sender_cache=1024, sender_comb=True, admit_first=True,
                                bcomb_wide=wide) as v:
        for rep in range(3):
            got = v.verify_batch(pk, sig, msg, off)
            assert np.array_equal(got, want), (rep, np.nonzero(got != want)[0][:10])
            info = v.info()
        assert info["cache_record_hits"] >= 2 * n, info


@pytest.mark.parametrize("policy", ["dalek", "libsodium"])
def test_wide_bcomb_golden_sets(at2v_mod, golden, policy):
    """AT2V_CTX_BCOMB_WIDE: the throughput kernel's cached records take [s]B from the 24-bit-window comb of B (11
    entries instead of 16). Every golden set, cold then warm (admit_first: the warm pass is all cached), both policies,
    large launches (the hit-list kernel) and small ones (the low-latency kernel, which keeps the 16-bit comb)."""
    for small in (OFF, 0):
        with at2v_mod.BatchVerifier(policy=policy, small_batch_max=small, sender_cache=1 << 14, sender_comb=True,
                                    admit_first=True, bcomb_wide=True) as v:
            for name in golden_io.SETS:
                g = golden[name]
                want = g.dalek if policy == "dalek" else g.sodium
                for rep in range(2):
                    got = v.verify_batch(g.pk, g.sig, g.msg, g.off)
                    assert np.array_equal(got, want), (small, name, rep, np.nonzero(got != want)[0][:10])
                    v.info()


def test_host_pipeline_chunks_with_combs(at2v_mod, oracle):
    """config-1 traffic (64 senders) tiled to 131,072 records, 1,000 of them mutated, through at2v_verify_batch on a comb
    context: the call stages four chunks (16,384 / 32,768 / 65,536 / 16,384 records), each a cached launch with its own
    claim slot, builds on the context's stream while the next chunk uploads. Cold, then warm: verdicts equal the oracle's and
    the warm call serves its records from the combs"""
    pk, sig, msg, off, snd, seq = oracle.gen_at2_transactions()
    reps, L = 32, 48
    n = 4096 * reps
    pk, sig, msg = np.tile(pk, (reps, 1)), np.tile(sig, (reps, 1)), np.tile(msg, reps)
    off = (np.arange(n + 1) * L).astype(np.uint32)
    pk, sig, msg = _mutate(pk, sig, msg, off, np.random.default_rng(41), 1000, kinds=3)
    want = oracle.verify_batch(pk, sig, msg, off)
    assert want.sum() == n - 1000
    with at2v_mod.BatchVerifier(sender_cache=1024, sender_comb=True) as v:
        for rep in range(3):
            h0 = v.info()["cache_record_hits"]
            got = v.verify_batch(pk, sig, msg, off)
            assert np.array_equal(got, want), (rep, np.nonzero(got != want)[0][:10])
            hits = v.info()["cache_record_hits"] - h0
        assert hits >= n - 64, hits
