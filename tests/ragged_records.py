"""Test data: records with ragged, partly long messages (0 B .. 16 KiB), signed by the oracle signer, a share of them
mutated. Used by tests/test_gpu_parity.py (kernel vs oracle) and tests/test_verify_one_cpu.py (CPU drop-in vs oracle).
The oracle is the checker here, never the thing tested."""
import numpy as np

# M lengths where 64 + M (the SHA-512 input R || A || M) sits on either side of a 128-byte block boundary
SHA_EDGES = [0, 1, 47, 48, 63, 64, 111, 112, 127, 128, 239, 240, 255, 256]


def make(oracle, n, seed, n_long=200, max_len=16384):
    """-> pk u8[n,32], sig u8[n,64], msg u8[...], off u32[n+1], mutated bool[n]"""
    rng = np.random.default_rng(seed)
    n_long = min(n_long, max(0, n - len(SHA_EDGES)))
    lens = np.concatenate([SHA_EDGES[:n], rng.integers(0, 300, max(0, n - len(SHA_EDGES) - n_long)),
                           rng.integers(300, max_len + 1, n_long)])[:n]
    rng.shuffle(lens)
    pks, sigs, msgs = [], [], []
    mutated = np.zeros(n, dtype=bool)
    for i, L in enumerate(lens):
        L = int(L)
        seed_i = rng.bytes(32)
        m = bytearray(rng.bytes(L))
        pk = bytearray(oracle.public_key(seed_i))
        sig = bytearray(oracle.sign(seed_i, bytes(m)))
        kind = int(rng.integers(0, 6))
        if kind == 1 and L > 0:
            m[int(rng.integers(0, L))] ^= 1 << int(rng.integers(0, 8))  # message byte
        elif kind == 2:
            sig[32 + int(rng.integers(0, 31))] ^= 0x10  # S (byte 63 untouched)
        elif kind == 3:
            sig[int(rng.integers(0, 31))] ^= 0x01  # R
        elif kind == 4:
            pk[int(rng.integers(0, 31))] ^= 0x04  # A (may also stop it decoding)
        else:
            kind = 0
        mutated[i] = kind != 0
        pks.append(bytes(pk))
        sigs.append(bytes(sig))
        msgs.append(bytes(m))
    off = np.zeros(n + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(m) for m in msgs])
    msg = np.frombuffer(b"".join(msgs), dtype=np.uint8)
    pk = np.frombuffer(b"".join(pks), dtype=np.uint8).reshape(n, 32)
    sig = np.frombuffer(b"".join(sigs), dtype=np.uint8).reshape(n, 64)
    return pk, sig, msg, off, mutated
