"""CPU: the library's CPU batch backend (include/at2v.h ABI v6, at2v_opts.num_gpus = 0; csrc/at2v_cpu.h).

SURVEY §8(b) specifies `num_gpus = 0` = CPU only with `cpu_threads`, and §5 a verdict-identical CPU path. The backend is a
thread pool over the kernels' own verify routine (verify_half_fu, compiled for the host inside libat2v.so), so it runs
here without a GPU; it never links or calls oracle/. It replaces the reference's SystemManager::run(.., num_cpus::get())
workers (/root/reference/src/bin/server/rpc.rs:124-125) that verify each payload broadcast at rpc.rs:275-284.
The GPU-side fallback (AT2V_CTX_CPU_FALLBACK after a device error) is covered in tests/test_gpu_boundary.py."""
import numpy as np
import pytest

import golden_io


@pytest.fixture(scope="module")
def at2v_mod():
    import at2v
    at2v.load_library()
    return at2v


@pytest.fixture(scope="module")
def cpu_ctx(at2v_mod):
    v = at2v_mod.BatchVerifier(num_gpus=0, cpu_threads=4)
    yield v
    v.close()


@pytest.mark.parametrize("name", golden_io.SETS)
@pytest.mark.parametrize("policy", ["dalek", "libsodium"])
def test_cpu_context_golden_sets(at2v_mod, golden, name, policy):
    g = golden[name]
    with at2v_mod.BatchVerifier(num_gpus=0, cpu_threads=3, policy=policy) as v:
        got = v.verify_batch(g.pk, g.sig, g.msg, g.off)
    want = g.dalek if policy == "dalek" else g.sodium
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


def test_cpu_context_info(cpu_ctx):
    inf = cpu_ctx.info()
    assert inf["num_gpus"] == 0 and inf["cpu_threads"] == 4
    assert inf["grid_blocks"] == 0 and inf["cache_capacity"] == 0


@pytest.mark.parametrize("n", [0, 1, 31, 32, 33, 63, 64, 65, 129, 1000])
def test_cpu_context_tail_sizes_and_pad_bits(at2v_mod, cpu_ctx, oracle, n):
    """pad bits stay 0 and no word past ceil(n/32) is written (a sentinel word after them)"""
    pk, sig, msg, off, cls = oracle.gen_adversarial(0x5EED, 7, max(n, 1), 60)
    pk, sig, off = pk[:n], sig[:n], off[:n + 1]
    words = np.full((n + 31) // 32 + 1, 0xDEADBEEF, np.uint32)
    lib = at2v_mod.load_library()
    msg_arg = msg if msg.size else np.zeros(1, np.uint8)
    rc = lib.at2v_verify_batch(cpu_ctx._h, pk.ctypes.data if n else None, sig.ctypes.data if n else None,
                               msg_arg.ctypes.data, off.ctypes.data, n, words.ctypes.data)
    assert rc == 0
    assert words[-1] == 0xDEADBEEF
    if n == 0:
        return
    want = oracle.verify_batch(pk, sig, msg, off)
    got = at2v_mod.unpack_verdicts(words[:-1], n)
    assert np.array_equal(got, want)
    if n % 32:
        assert words[(n - 1) // 32] >> (n % 32) == 0


def test_cpu_context_fresh_adversarial_vs_oracle(at2v_mod, cpu_ctx, oracle):
    pk, sig, msg, off, cls = oracle.gen_adversarial(0xC0B, 0, 5000, 100)
    got = cpu_ctx.verify_batch(pk, sig, msg, off)
    want = oracle.verify_batch(pk, sig, msg, off)
    assert np.array_equal(got, want)
    assert 0 < want.sum() < len(want)


def test_cpu_context_unaligned_offsets(at2v_mod, cpu_ctx, golden):
    """msg_off[0] > 0 and messages at odd byte offsets"""
    g = golden["ragged"]
    msg = np.concatenate([np.zeros(3, np.uint8), g.msg])
    off = g.off + 3
    got = cpu_ctx.verify_batch(g.pk, g.sig, msg, off)
    assert np.array_equal(got, g.dalek)


def test_cpu_context_rejects_device_entry_points(at2v_mod, cpu_ctx):
    lib = at2v_mod.load_library()
    buf = np.zeros(4096, np.uint8)
    p = buf.ctypes.data
    assert lib.at2v_verify_batch_device(cpu_ctx._h, p, p, p, 16, p, 1, p, None) == -2  # AT2V_E_NODEVICE
    assert lib.at2v_gen_records_device(cpu_ctx._h, 1, 0, 1, 16, p, p, p, p, None) == -2
    assert lib.at2v_comm_init_rank(cpu_ctx._h, bytes(128), 0, 1) == -2


def test_cpu_context_decode_points(at2v_mod, cpu_ctx, golden, oracle):
    g = golden["edge"]
    got = cpu_ctx.decode_points(g.pk)
    want = np.array([oracle.decompress_ok(g.pk[i].tobytes()) for i in range(g.n)], dtype=bool)
    assert np.array_equal(got, want)
    assert 0 < got.sum() < g.n


def test_cpu_context_submit_wait(at2v_mod, golden):
    """at2v_verify_batch_submit / _wait on a CPU context (the batch is verified inside the submit): tickets count up,
    each is waited for once, a repeated, unknown or zero ticket is AT2V_E_INVALID, and a submit completes the call two
    tickets back"""
    lib = at2v_mod.load_library()
    with at2v_mod.BatchVerifier(num_gpus=0, cpu_threads=2) as v:
        a = v.submit_batch(golden["adversarial"].pk, golden["adversarial"].sig, golden["adversarial"].msg,
                           golden["adversarial"].off)
        b = v.submit_batch(golden["edge"].pk, golden["edge"].sig, golden["edge"].msg, golden["edge"].off)
        assert b.ticket == a.ticket + 1
        assert np.array_equal(v.wait_batch(b), golden["edge"].dalek)
        assert np.array_equal(v.wait_batch(a), golden["adversarial"].dalek)
        assert lib.at2v_verify_batch_wait(v._h, a.ticket) == -1  # waited already
        assert lib.at2v_verify_batch_wait(v._h, 0) == -1
        assert lib.at2v_verify_batch_wait(v._h, b.ticket + 5) == -1
        r = golden["rfc8032"]
        c = v.submit_batch(r.pk, r.sig, r.msg, r.off)
        d = v.submit_batch(r.pk, r.sig, r.msg, r.off)
        e = v.submit_batch(r.pk, r.sig, r.msg, r.off)  # completes c (its slot), whose result is then gone
        assert lib.at2v_verify_batch_wait(v._h, c.ticket) == -1
        assert np.array_equal(v.wait_batch(d), r.dalek) and np.array_equal(v.wait_batch(e), r.dalek)
        t = __import__("ctypes").c_uint64(7)
        assert lib.at2v_verify_batch_submit(v._h, None, None, None, None, 5, None, t) == -1 and t.value == 0


def test_cpu_context_counts_batches(at2v_mod, golden):
    g = golden["rfc8032"]
    with at2v_mod.BatchVerifier(num_gpus=0, cpu_threads=2) as v:
        for _ in range(3):
            v.verify_batch(g.pk, g.sig, g.msg, g.off)
        inf = v.info()
    assert inf["cpu_batches"] == 3 and inf["cpu_fallbacks"] == 0


def test_cpu_context_bad_args(at2v_mod):
    with pytest.raises(at2v_mod.At2vError):
        at2v_mod.BatchVerifier(num_gpus=-1)
    lib = at2v_mod.load_library()
    assert lib.at2v_create(None, None) == -1  # no out pointer
    bad_flags = at2v_mod._Opts(0, 0, 0, 0, 0, 0, 1, 0x80)
    h = at2v_mod.ctypes.c_void_p()
    assert lib.at2v_create(at2v_mod.ctypes.byref(bad_flags), at2v_mod.ctypes.byref(h)) == -1
    with at2v_mod.BatchVerifier(num_gpus=0, cpu_threads=1) as v:
        g = golden_io.load("rfc8032")
        bad = g.off.copy()
        bad[1] = bad[2] + 1  # decreasing offsets
        with pytest.raises(at2v_mod.At2vError):
            v.verify_batch(g.pk, g.sig, g.msg, bad)


def test_cpu_queue_orders_verdicts(at2v_mod, golden):
    """the ingest queue on the CPU backend (AT2V_QUEUE_CPU): verdicts in ticket order, every golden set"""
    from at2v import node
    with node.IngestQueue(cpu=True, cpu_threads=3, max_batch=700, max_delay_us=500) as q:
        want, first = [], None
        for name in golden_io.SETS:
            g = golden[name]
            t = q.submit(g.pk, g.sig, g.msg, g.off)
            first = t if first is None else first
            want.append(g.dalek)
        q.flush()
        want = np.concatenate(want)
        got_t, got_v = [], []
        while sum(len(x) for x in got_t) < len(want):
            t, v = q.poll(1 << 16, 2_000_000)
            assert len(t), "queue stalled"
            got_t.append(t)
            got_v.append(v)
        t = np.concatenate(got_t)
        v = np.concatenate(got_v)
        st = q.stats()
    assert np.array_equal(t, np.arange(first, first + len(want), dtype=np.uint64))
    assert not (v == 0xFF).any()
    assert np.array_equal(v.astype(bool), want)
    assert st["failed_batches"] == 0 and st["cpu_fallbacks"] == 0


def test_cpu_pool_threads_default(at2v_mod):
    with at2v_mod.BatchVerifier(num_gpus=0) as v:
        assert v.info()["cpu_threads"] >= 1
