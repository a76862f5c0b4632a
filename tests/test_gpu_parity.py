"""GPU parity tests: libat2v.so (HIP, gfx950) through its C ABI vs the golden fixtures and the oracle.

Bar: bit-exact verdicts (integer/byte work). Sizes the oracle checks in seconds are compared record by
record; the full BASELINE sizes (1M) are checked through size-independent properties (every generated
record valid; exactly the mutated records rejected; verdict bits past n zero; shard/tail invariance).
"""
import os

import numpy as np
import pytest

import golden_io

pytestmark = pytest.mark.gpu

CFG_SEED = 0x4154325F


@pytest.fixture(scope="module")
def at2v_mod():
    import at2v
    return at2v


# Both verify kernels: "lowlat" = the library default (launches of <= 32768 records run the two-lanes-per-record
# kernel, larger ones the throughput kernel); "throughput" = the throughput kernel at every size.
KERNELS = {"lowlat": 0, "throughput": 0xFFFFFFFF}


@pytest.fixture(scope="module", params=list(KERNELS))
def verifier(at2v_mod, request):
    v = at2v_mod.BatchVerifier(policy="dalek", small_batch_max=KERNELS[request.param])
    yield v
    v.close()


@pytest.fixture(scope="module", params=list(KERNELS))
def verifier_sodium(at2v_mod, request):
    v = at2v_mod.BatchVerifier(policy="libsodium", small_batch_max=KERNELS[request.param])
    yield v
    v.close()


def _mismatch(got, want, cls=None):
    bad = np.nonzero(got != want)[0]
    return f"{bad.size} mismatches at {bad[:10]}" + (f" classes {cls[bad[:10]]}" if cls is not None else "")


@pytest.mark.parametrize("name", golden_io.SETS)
def test_golden_dalek(verifier, golden, name):
    g = golden[name]
    got = verifier.verify_batch(g.pk, g.sig, g.msg, g.off)
    assert np.array_equal(got, g.dalek), _mismatch(got, g.dalek, g.cls)


@pytest.mark.parametrize("name", golden_io.SETS)
def test_golden_libsodium_policy(verifier_sodium, golden, name):
    g = golden[name]
    got = verifier_sodium.verify_batch(g.pk, g.sig, g.msg, g.off)
    assert np.array_equal(got, g.sodium), _mismatch(got, g.sodium, g.cls)


def test_info(verifier):
    info = verifier.info()
    # 8-wave blocks (both waves of every SIMD in one workgroup, paced), one per CU: 2 waves/SIMD
    assert info["cus"] >= 1 and info["grid_blocks"] >= info["cus"] and info["block_threads"] == 512
    assert info["grid_blocks"] * info["block_threads"] // 64 == 8 * info["cus"]


@pytest.mark.parametrize("n", [1, 2, 31, 32, 33, 63, 64, 65, 127, 1000])
def test_tail_sizes_and_pad_bits(verifier, golden, n):
    """n not a multiple of 64/32: tail lanes are masked and pad bits are zero."""
    g = golden["adversarial"]
    off = g.off[: n + 1]
    got = verifier.verify_batch(g.pk[:n], g.sig[:n], g.msg, off)
    assert np.array_equal(got, g.dalek[:n])
    import ctypes
    lib = verifier._lib
    words = np.full((n + 31) // 32 + 1, 0xFFFFFFFF, np.uint32)
    rc = lib.at2v_verify_batch(verifier._h, g.pk[:n].ctypes.data, g.sig[:n].ctypes.data, g.msg.ctypes.data,
                               np.ascontiguousarray(off).ctypes.data, n, words.ctypes.data)
    assert rc == 0
    if n % 32:
        assert words[(n - 1) // 32] >> (n % 32) == 0
    assert words[-1] == 0xFFFFFFFF  # nothing written past ceil(n/32) words


def test_empty_batch(verifier):
    got = verifier.verify_batch(np.zeros((0, 32), np.uint8), np.zeros((0, 64), np.uint8), np.zeros(0, np.uint8),
                                np.zeros(1, np.uint32))
    assert got.size == 0


def test_unaligned_message_offsets(verifier, golden):
    """messages starting at arbitrary byte offsets (msg_off[0] > 0, odd lengths)"""
    g = golden["ragged"]
    pad = np.zeros(3, np.uint8)
    msg = np.concatenate([pad, g.msg])
    got = verifier.verify_batch(g.pk, g.sig, msg, g.off + 3)
    assert np.array_equal(got, g.dalek)


def test_oracle_adversarial_larger(verifier, oracle):
    """fresh adversarial mix (not the committed fixture) against the oracle, record by record"""
    pk, sig, msg, off, cls = oracle.gen_adversarial(CFG_SEED + 1, 100_000, 16384, 100)
    want = oracle.verify_batch(pk, sig, msg, off)
    got = verifier.verify_batch(pk, sig, msg, off)
    assert np.array_equal(got, want), _mismatch(got, want, cls)
    assert want.sum() > 0.85 * len(want)


def test_verify_one_and_drop_mirror(at2v_mod, golden):
    g = golden["rfc8032"]
    for i in range(g.n):
        assert at2v_mod.verify_one(bytes(g.pk[i]), bytes(g.sig[i]), g.message(i))
        at2v_mod.Signature(bytes(g.sig[i])).verify(g.message(i), at2v_mod.PublicKey(bytes(g.pk[i])))
    bad = bytearray(g.sig[0])
    bad[63] ^= 0x80
    assert not at2v_mod.verify_one(bytes(g.pk[0]), bytes(bad), g.message(0))
    with pytest.raises(at2v_mod.VerifyError):
        at2v_mod.Signature(bytes(bad)).verify(g.message(0), at2v_mod.PublicKey(bytes(g.pk[0])))


def test_gpu_generator_matches_oracle(verifier, oracle):
    """GPU keygen+sign of the deterministic generator is bit-exact with the oracle signer"""
    import torch
    n, L = 4096, 100
    d_pk = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    d_sig = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    d_msg = torch.zeros(n * L, dtype=torch.uint8, device="cuda")
    d_off = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
    verifier.gen_records_device(CFG_SEED, 12345, n, L, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                d_off.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    pk, sig, msg, off = oracle.gen_records(CFG_SEED, 12345, n, L)
    assert np.array_equal(d_pk.cpu().numpy().reshape(n, 32), pk)
    assert np.array_equal(d_msg.cpu().numpy(), msg)
    assert np.array_equal(d_off.cpu().numpy().astype(np.uint32), off)
    assert np.array_equal(d_sig.cpu().numpy().reshape(n, 64), sig)


def test_sign_batch_matches_oracle(verifier, oracle):
    rng = np.random.default_rng(5)
    n = 300
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    lens = rng.integers(0, 300, n)
    msgs = [rng.integers(0, 256, int(k), dtype=np.uint8).tobytes() for k in lens]
    off = np.zeros(n + 1, np.uint32)
    off[1:] = np.cumsum(lens)
    msg = np.frombuffer(b"".join(msgs), np.uint8)
    pk, sig = verifier.sign_batch(seeds, msg, off)
    for i in range(0, n, 7):
        assert bytes(pk[i]) == oracle.public_key(bytes(seeds[i]))
        assert bytes(sig[i]) == oracle.sign(bytes(seeds[i]), msgs[i])
    assert verifier.verify_batch(pk, sig, msg, off).all()


def test_device_api_full_size_properties(verifier):
    """BASELINE config 2 size (1M records, 100-byte messages) on device buffers:
    all valid; flipping one bit in k chosen records rejects exactly those records."""
    import torch
    n, L = 1 << 20, 100
    s = torch.cuda.current_stream().cuda_stream
    d_pk = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    d_sig = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    d_msg = torch.zeros(n * L, dtype=torch.uint8, device="cuda")
    d_off = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
    d_ver = torch.zeros((n + 31) // 32, dtype=torch.int32, device="cuda")
    verifier.gen_records_device(CFG_SEED, 0, n, L, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                d_off.data_ptr(), s)
    verifier.verify_batch_device(d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), n * L, d_off.data_ptr(), n,
                                 d_ver.data_ptr(), s)
    torch.cuda.synchronize()
    assert (d_ver == -1).all().item(), "every generated record must verify"
    rng = np.random.default_rng(9)
    idx = np.unique(rng.integers(0, n, 2000))
    which = rng.integers(0, 3, idx.size)
    for k, (i, w) in enumerate(zip(idx.tolist(), which.tolist())):
        bit = int(rng.integers(0, 8))
        if w == 0:
            d_sig[i * 64 + int(rng.integers(0, 64))] ^= (1 << bit)
        elif w == 1:
            d_msg[i * L + int(rng.integers(0, L))] ^= (1 << bit)
        else:
            d_pk[i * 32 + int(rng.integers(0, 32))] ^= (1 << bit)
    verifier.verify_batch_device(d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), n * L, d_off.data_ptr(), n,
                                 d_ver.data_ptr(), s)
    torch.cuda.synchronize()
    import at2v
    ok = at2v.unpack_verdicts(d_ver.cpu().numpy().view(np.uint32), n)
    rejected = np.nonzero(~ok)[0]
    assert np.array_equal(rejected, idx), f"{rejected.size} rejected vs {idx.size} mutated"


def test_repeat_determinism(verifier, golden):
    g = golden["adversarial"]
    a = verifier.verify_batch(g.pk, g.sig, g.msg, g.off)
    b = verifier.verify_batch(g.pk, g.sig, g.msg, g.off)
    assert np.array_equal(a, b)


def test_multi_gpu_context(at2v_mod, golden, monkeypatch):
    """one context over 8 devices; on a box with fewer, the test hook AT2V_TEST_DEVICE_ALIAS maps shard g to device
    g % ndev so the single-process split still runs (tests/test_gpu_multidev.py has the full matrix)"""
    import torch
    if torch.cuda.device_count() < 8:
        monkeypatch.setenv("AT2V_TEST_DEVICE_ALIAS", "1")
    v = at2v_mod.BatchVerifier(num_gpus=8)
    g = golden["adversarial"]
    assert np.array_equal(v.verify_batch(g.pk, g.sig, g.msg, g.off), g.dalek)
    v.close()


def test_many_chunks_per_wave_adversarial(verifier, oracle):
    """Enough records that every resident wave (2048) takes several chunks from the chunk queue (262,181
    records = 4097 chunks, the last one ragged), adversarial mix, compared record by record."""
    n = (1 << 18) + 37
    pk, sig, msg, off, cls = oracle.gen_adversarial(CFG_SEED + 2, 0, n, 64)
    want = oracle.verify_batch(pk, sig, msg, off)
    got = verifier.verify_batch(pk, sig, msg, off)
    assert np.array_equal(got, want), _mismatch(got, want, cls)
    assert 0.85 * n < want.sum() < n


def test_lowlat_kernel_grid_stride(at2v_mod, oracle):
    """the two-lanes-per-record kernel forced on a batch larger than one pass of its grid (grid-strided 32-record
    chunks), against the oracle"""
    pk, sig, msg, off, cls = oracle.gen_adversarial(CFG_SEED + 7, 0, 100_000, 64)
    want = oracle.verify_batch(pk, sig, msg, off)
    v = at2v_mod.BatchVerifier(policy="dalek", small_batch_max=1 << 20)
    try:
        got = v.verify_batch(pk, sig, msg, off)
    finally:
        v.close()
    assert np.array_equal(got, want), _mismatch(got, want, cls)



def test_ragged_long_messages(verifier, oracle):
    """Messages of very different lengths inside one wave (0 B up to 16 KiB, so lanes need 1 to 130 SHA-512 blocks),
    at packed unaligned offsets, signed by the oracle signer; about a third mutated (message byte, S, R or A). Record by
    record against the oracle; every unmutated record verifies and no mutated one does."""
    import ragged_records
    pk, sig, msg, off, mutated = ragged_records.make(oracle, 2500, seed=20261017)
    want = oracle.verify_batch(pk, sig, msg, off)
    got = verifier.verify_batch(pk, sig, msg, off)
    assert np.array_equal(got, want), _mismatch(got, want)
    assert want[~mutated].all()
    assert not want[mutated].any()


def test_config3_total_size_on_one_gpu(at2v_mod):
    """BASELINE config 3's whole batch (16M signatures, here + 17 for a ragged tail) in ONE launch on one GPU: 262,145
    chunks through the chunk queue, 1.68 GB of messages (offsets near the top of the u32 range the ABI allows).
    Every generated record verifies; after mutating 3,000 random records in S, M or A exactly those are rejected,
    and the pad bits of the last verdict word stay 0."""
    import torch
    n, L = (1 << 24) + 17, 100
    v = at2v_mod.BatchVerifier(policy="dalek", small_batch_max=0xFFFFFFFF)
    try:
        s = torch.cuda.current_stream().cuda_stream
        d_pk = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
        d_sig = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
        d_msg = torch.zeros(n * L, dtype=torch.uint8, device="cuda")
        d_off = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
        words = (n + 31) // 32
        d_ver = torch.zeros(words, dtype=torch.int32, device="cuda")
        v.gen_records_device(CFG_SEED + 3, 0, n, L, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                             d_off.data_ptr(), s)
        v.verify_batch_device(d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), n * L, d_off.data_ptr(), n,
                              d_ver.data_ptr(), s)
        torch.cuda.synchronize()
        ok = at2v_mod.unpack_verdicts(d_ver.cpu().numpy().view(np.uint32), n)
        assert ok.all(), f"{(~ok).sum()} generated records rejected"
        rng = np.random.default_rng(33)
        idx = np.unique(rng.integers(0, n, 3000))
        which = rng.integers(0, 3, idx.size)
        bits = torch.from_numpy((1 << rng.integers(0, 8, idx.size)).astype(np.uint8)).cuda()
        for w, (arr, width) in enumerate(((d_sig, 64), (d_msg, L), (d_pk, 32))):
            sel = np.nonzero(which == w)[0]
            rows = torch.from_numpy(idx[sel]).cuda()
            cols = torch.from_numpy(rng.integers(0, width, sel.size)).cuda()
            view = arr.view(-1, width)
            view[rows, cols] = view[rows, cols] ^ bits[torch.from_numpy(sel).cuda()]
        v.verify_batch_device(d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), n * L, d_off.data_ptr(), n,
                              d_ver.data_ptr(), s)
        torch.cuda.synchronize()
        w_host = d_ver.cpu().numpy().view(np.uint32)
        ok = at2v_mod.unpack_verdicts(w_host, n)
        assert np.array_equal(np.nonzero(~ok)[0], idx)
        assert (int(w_host[-1]) >> (n % 32)) == 0, "pad bits of the last verdict word must be 0"
    finally:
        v.close()


# ---- the host-buffer path's pipeline (at2v_api.hip HostPipe; round 6) ----
# The staged form (test hook AT2V_TEST_STAGED=1): one launch over the shard's part, records uploaded in regions of 65,536
# that the waves wait for. Sizes: one region (32,833 records), two (the second ragged), seven (every staging slot reused).
# The chunked form (the default): the first chunks are 65,536 records,
# later ones 131,072, and a remainder below the first chunk's size joins the chunk before it; its two compute streams
# are created each way (AT2V_TEST_PIPE_STREAMS: one hardware queue or two, so consecutive launches overlap or not).
@pytest.mark.parametrize("form", ["staged", "chunked-plain", "chunked-priority", "chunked-cumask"])
@pytest.mark.parametrize("n", [32_833, 98_437, 400_009])
def test_host_pipeline_chunks_adversarial(at2v_mod, oracle, monkeypatch, n, form):
    """at2v_verify_batch through each form of the pipeline. Adversarial records, record by record against the oracle,
    twice through one context (the second call reuses its staging slots and device arena); a sentinel word after the
    bitmap stays untouched and the pad bits of the last word are 0"""
    monkeypatch.setenv("AT2V_TEST_STAGED", "1" if form == "staged" else "0")
    streams = form.split("-")[-1]
    monkeypatch.setenv("AT2V_TEST_PIPE_STREAMS", {"staged": "0", "plain": "0", "priority": "1", "cumask": "2"}[streams])
    pk, sig, msg, off, cls = oracle.gen_adversarial(CFG_SEED + 101, 0, n, 72)
    want = oracle.verify_batch(pk, sig, msg, off)
    lib = at2v_mod.load_library()
    with at2v_mod.BatchVerifier() as v:
        for rep in range(2):  # (the second call reuses the staging slots and device buffers of the first)
            words = np.full((n + 31) // 32 + 1, 0xA5A5A5A5, np.uint32)
            rc = lib.at2v_verify_batch(v._h, pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, off.ctypes.data, n,
                                       words.ctypes.data)
            assert rc == 0
            assert words[-1] == 0xA5A5A5A5
            got = at2v_mod.unpack_verdicts(words[:-1], n)
            assert np.array_equal(got, want), (rep, _mismatch(got, want, cls))
            if n % 32:
                assert int(words[(n - 1) // 32]) >> (n % 32) == 0


def test_host_pipeline_staged_alternating_batches(at2v_mod, monkeypatch):
    """The staged form reads each region as soon as the host publishes it, from DMA-written device memory the previous
    call's launch also read (same arena, same addresses). Two batches of 1,000,003 records (16 regions, the last one
    ragged) alternate through one context six times: A every record valid, B the same with an S byte flipped in 5,000
    records. Any stale line of the other batch would flip verdicts: exactly B's mutated records are rejected each time,
    and the pad bits stay 0"""
    import torch
    n, L = 1_000_003, 100
    with at2v_mod.BatchVerifier() as g:
        s = torch.cuda.current_stream().cuda_stream
        d_pk = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
        d_sig = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
        d_msg = torch.zeros(n * L, dtype=torch.uint8, device="cuda")
        d_off = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
        g.gen_records_device(CFG_SEED + 131, 0, n, L, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                             d_off.data_ptr(), s)
        torch.cuda.synchronize()
        pk = d_pk.cpu().numpy()
        sig_a = d_sig.cpu().numpy().reshape(n, 64).copy()
        msg = d_msg.cpu().numpy()
        off = d_off.cpu().numpy().view(np.uint32)
    rng = np.random.default_rng(20261019)
    idx = np.sort(rng.choice(n, 5000, replace=False))
    sig_b = sig_a.copy()
    sig_b[idx, 32 + rng.integers(0, 31, idx.size)] ^= 0x04
    lib = at2v_mod.load_library()
    monkeypatch.setenv("AT2V_TEST_STAGED", "1")
    with at2v_mod.BatchVerifier() as v:
        for rep in range(6):
            sig = sig_b if rep % 2 else sig_a
            words = np.full((n + 31) // 32 + 1, 0xA5A5A5A5, np.uint32)
            rc = lib.at2v_verify_batch(v._h, pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, off.ctypes.data, n,
                                       words.ctypes.data)
            assert rc == 0
            assert words[-1] == 0xA5A5A5A5
            ok = at2v_mod.unpack_verdicts(words[:-1], n)
            bad = np.nonzero(~ok)[0]
            if rep % 2:
                assert np.array_equal(bad, idx), (rep, bad.size)
            else:
                assert bad.size == 0, (rep, bad[:10])
            assert int(words[(n - 1) // 32]) >> (n % 32) == 0


@pytest.mark.parametrize("shards", [1, 8])
def test_host_async_submit_wait(at2v_mod, oracle, monkeypatch, shards):
    """at2v_verify_batch_submit / _wait on the device (one shard, and 8 shards through the alias hook): three batches
    with two in flight (A and B submitted, A waited, C submitted while B verifies, then B and C), record by record against
    the oracle; the verdict words of each land in its own array with pad bits 0; a synchronous call between submits
    completes the call in flight; a repeated ticket is AT2V_E_INVALID"""
    if shards > 1:
        monkeypatch.setenv("AT2V_TEST_DEVICE_ALIAS", "1")
    lib = at2v_mod.load_library()
    batches = []
    for k, (n, L) in enumerate(((100_003, 72), (163_841, 100), (40_001, 48))):
        pk, sig, msg, off, cls = oracle.gen_adversarial(CFG_SEED + 211 + k, 0, n, L)
        batches.append((pk, sig, msg, off, oracle.verify_batch(pk, sig, msg, off)))
    with at2v_mod.BatchVerifier(num_gpus=shards) as v:
        for rep in range(2):
            a = v.submit_batch(*batches[0][:4])
            b = v.submit_batch(*batches[1][:4])
            assert np.array_equal(v.wait_batch(a), batches[0][4])
            c = v.submit_batch(*batches[2][:4])
            if rep:  # a synchronous call completes B and C first (their results stay for their waits)
                assert np.array_equal(v.verify_batch(*batches[0][:4]), batches[0][4])
            assert np.array_equal(v.wait_batch(b), batches[1][4])
            assert np.array_equal(v.wait_batch(c), batches[2][4])
            for p_, bt in ((a, batches[0]), (b, batches[1]), (c, batches[2])):
                n = len(bt[4])
                assert int(p_.words[(n - 1) // 32]) >> (n % 32) == 0 if n % 32 else True
            assert lib.at2v_verify_batch_wait(v._h, b.ticket) == -1


def test_host_pipeline_ragged_messages_regrow(at2v_mod, oracle):
    """ragged messages (0 B .. 16 KiB) tiled to 100,000 records at an offset msg_off[0] > 0: the chunks carry very
    different message bytes, so staging slots regrow mid-call; record by record against the oracle"""
    import ragged_records
    pk, sig, msg, off, mutated = ragged_records.make(oracle, 2500, seed=20261018)
    reps = 40
    n = 2500 * reps
    pk = np.tile(pk, (reps, 1))
    sig = np.tile(sig, (reps, 1))
    lens = np.diff(off.astype(np.int64))
    msg = np.concatenate([np.zeros(7, np.uint8), np.tile(msg, reps)])
    offs = np.zeros(n + 1, np.uint32)
    offs[1:] = np.cumsum(np.tile(lens, reps))
    offs += 7
    want = np.tile(oracle.verify_batch(pk[:2500], sig[:2500], msg, offs[:2501]), reps)
    assert want.sum() == reps * (~mutated).sum()
    with at2v_mod.BatchVerifier() as v:
        got = v.verify_batch(pk, sig, msg, offs)
    assert np.array_equal(got, want), _mismatch(got, want)
