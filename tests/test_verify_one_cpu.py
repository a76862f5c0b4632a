"""CPU: at2v_verify_one[_policy] — the per-signature drop-in (include/at2v.h, SURVEY §8(b) "CPU, 1/0") — against
every golden set under both policies. It is the product's own verify code (csrc/ headers) compiled for the host
inside libat2v.so, not the oracle, and it needs no GPU, so it is checked here; tests/test_gpu_parity.py checks it
again on the GPU box next to the kernel. Reference call it replaces: drop::crypto::sign's Signature::verify,
invoked per payload by sieve/murmur for the payloads broadcast at /root/reference/src/bin/server/rpc.rs:275-284."""
import threading

import numpy as np
import pytest

import golden_io


@pytest.fixture(scope="module")
def at2v_mod():
    import at2v
    at2v.load_library()
    return at2v


@pytest.mark.parametrize("name", golden_io.SETS)
def test_verify_one_matches_golden_both_policies(at2v_mod, golden, name):
    g = golden[name]
    got_d = np.array([at2v_mod.verify_one(g.pk[i].tobytes(), g.sig[i].tobytes(), g.message(i)) for i in range(g.n)])
    got_s = np.array([at2v_mod.verify_one(g.pk[i].tobytes(), g.sig[i].tobytes(), g.message(i), policy="libsodium")
                      for i in range(g.n)])
    assert np.array_equal(got_d, g.dalek), np.nonzero(got_d != g.dalek)[0][:10]
    assert np.array_equal(got_s, g.sodium), np.nonzero(got_s != g.sodium)[0][:10]


def test_verify_one_matches_oracle_on_fresh_adversarial(at2v_mod, oracle):
    pk, sig, msg, off, cls = oracle.gen_adversarial(0x1D, 0, 3000, 77)
    want = oracle.verify_batch(pk, sig, msg, off)
    got = np.array([at2v_mod.verify_one(pk[i].tobytes(), sig[i].tobytes(), msg[off[i]:off[i + 1]].tobytes())
                    for i in range(len(pk))])
    assert np.array_equal(got, want)
    assert 0 < want.sum() < len(want)


def test_verify_one_is_reentrant(at2v_mod, golden):
    """no lock, no shared state: threads verifying at once get the golden verdicts"""
    g = golden["adversarial"]
    idx = np.arange(min(g.n, 1200))
    out = np.zeros((4, len(idx)), bool)

    def run(t):
        for k, i in enumerate(idx):
            out[t, k] = at2v_mod.verify_one(g.pk[i].tobytes(), g.sig[i].tobytes(), g.message(i))

    th = [threading.Thread(target=run, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert (out == g.dalek[idx]).all()


def test_drop_signature_mirror(at2v_mod, golden):
    """at2v.Signature.verify(message, PublicKey) raises VerifyError like drop's Result<(), VerifyError>"""
    g = golden["rfc8032"]
    i_ok = int(np.nonzero(g.dalek)[0][0])
    at2v_mod.Signature(g.sig[i_ok].tobytes()).verify(g.message(i_ok), at2v_mod.PublicKey(g.pk[i_ok].tobytes()))
    bad = bytearray(g.sig[i_ok].tobytes())
    bad[3] ^= 1
    with pytest.raises(at2v_mod.VerifyError):
        at2v_mod.Signature(bytes(bad)).verify(g.message(i_ok), at2v_mod.PublicKey(g.pk[i_ok].tobytes()))


def test_verify_one_rejects_bad_arguments(at2v_mod):
    lib = at2v_mod.load_library()
    assert lib.at2v_verify_one(None, None, None, 0) == -1
    assert lib.at2v_verify_one_policy(b"\0" * 32, b"\0" * 64, None, 0, 7) == -1
    assert lib.at2v_verify_one(b"\0" * 32, b"\0" * 64, None, 5) == -1  # msg NULL with len > 0
    assert lib.at2v_verify_one(b"\0" * 32, b"\0" * 64, None, 0) == 0   # empty message is fine


def test_verify_one_ragged_long_messages(at2v_mod, oracle):
    """0 B .. 16 KiB messages (1 to 130 SHA-512 blocks), about a third mutated: the CPU drop-in against the oracle"""
    import ragged_records
    pk, sig, msg, off, mutated = ragged_records.make(oracle, 600, seed=7, n_long=60)
    want = oracle.verify_batch(pk, sig, msg, off)
    got = np.array([at2v_mod.verify_one(pk[i].tobytes(), sig[i].tobytes(), msg[off[i]:off[i + 1]].tobytes())
                    for i in range(len(pk))])
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    assert want[~mutated].all() and not want[mutated].any()
