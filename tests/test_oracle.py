"""CPU: pin the oracle (oracle/ed25519_oracle.c) against the golden fixtures, RFC 8032 §7.1 and hashlib.

The fixture verdicts come from OpenSSL 3.0.2 (dalek-1.x semantics) and libsodium 1.0.18, not from the
oracle (oracle/crosscheck.c). Reference tests hold no vectors for this path."""
import hashlib
import os

import numpy as np
import pytest

import golden_io

RFC8032 = [  # RFC 8032 §7.1 TEST 1-3: (secret seed, public key, message, signature)
    ("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
     "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a", "",
     "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24"
     "655141438e7a100b"),
    ("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
     "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c", "72",
     "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aee"
     "b00d291612bb0c00"),
    ("c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7",
     "fc51cd8e6218a1a38da47ed00230f0580816ed13ba3303ac5deb911548908025", "af82",
     "6291d657deec24024827e69c3abe01a30ce548a284743a445e3680d7db5ac3ac18ff9b538d16f290ae67f760984dc6594a7c15e9716ed28d"
     "c027beceea1ec40a"),
]


@pytest.mark.parametrize("name", golden_io.SETS)
@pytest.mark.parametrize("policy", [0, 1])
def test_oracle_matches_golden(oracle, golden, name, policy):
    g = golden[name]
    got = oracle.verify_batch(g.pk, g.sig, g.msg, g.off, policy)
    want = g.dalek if policy == 0 else g.sodium
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{name} policy {policy}: mismatches at {bad[:10]} classes {g.cls[bad[:10]]}"


@pytest.mark.parametrize("seed,pk,msg,sig", RFC8032)
def test_oracle_rfc8032(oracle, seed, pk, msg, sig):
    seed, pk, msg, sig = (bytes.fromhex(x) for x in (seed, pk, msg, sig))
    assert oracle.public_key(seed) == pk
    assert oracle.sign(seed, msg) == sig
    assert oracle.verify(pk, sig, msg)
    bad = bytearray(sig)
    bad[0] ^= 1
    assert not oracle.verify(pk, bytes(bad), msg)


def test_oracle_sha512_vs_hashlib(oracle):
    rng = np.random.default_rng(1)
    for n in list(range(0, 300, 7)) + [111, 112, 239, 240, 1000]:
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.sha512(data) == hashlib.sha512(data).digest(), n


def test_fixture_sets_cover_every_class(golden):
    adv = golden["adversarial"]
    classes = set(np.unique(adv.cls).tolist())
    assert classes == set(range(8))
    # dalek accepts small-order/mixed-order constructions libsodium rejects (Appendix A.4)
    assert (adv.dalek & ~adv.sodium).any()
    assert not (adv.sodium & ~adv.dalek).any()
    edge = golden["edge"]
    assert edge.dalek.sum() > 100 and edge.sodium.sum() == 1


def test_generator_reproduces_cfg1_fixture(oracle, golden):
    """The committed config-1 fixture is exactly the deterministic AT2 transaction generator's output."""
    pk, sig, msg, off, snd, seq = oracle.gen_at2_transactions()
    g = golden["at2_cfg1"]
    assert np.array_equal(pk, g.pk) and np.array_equal(sig, g.sig) and np.array_equal(msg, g.msg)
    assert np.array_equal(off, g.off)
    # message = bincode(ThinTransaction{recipient, amount}) (src/lib.rs:14-22): u64le(32) || recipient || u64le(amount)
    m = msg.reshape(-1, 48)
    assert (m[:, :8] == np.array([32, 0, 0, 0, 0, 0, 0, 0], np.uint8)).all()
    amounts = m[:, 40:48].copy().view("<u8").ravel()
    assert amounts.min() >= 1 and amounts.max() <= 1000
    assert set(seq.tolist()) == set(range(1, 65)) and set(snd.tolist()) == set(range(64))
    # each recipient is another sender's key
    keys = {bytes(pk[i]) for i in range(64)}
    assert all(bytes(m[i, 8:40]) in keys and bytes(m[i, 8:40]) != bytes(pk[i]) for i in range(len(m)))


def test_adversarial_generator_reproduces_fixture(oracle, golden):
    pk, sig, msg, off, cls = oracle.gen_adversarial(0x4154325F, 0, 8192, 100)
    g = golden["adversarial"]
    assert np.array_equal(pk, g.pk) and np.array_equal(sig, g.sig) and np.array_equal(msg, g.msg)
    assert np.array_equal(cls, g.cls)


def test_generator_records_valid_and_deterministic(oracle):
    a = oracle.gen_records(7, 100, 64, 100)
    b = oracle.gen_records(7, 100, 64, 100)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    pk, sig, msg, off = a
    assert oracle.verify_batch(pk, sig, msg, off).all()
