"""CPU: the OpenSSL leg of bench.py's CPU baseline (oracle/openssl_verify.c) gives the golden dalek
verdicts on every fixture set, so the GPU/CPU comparison in the bench line times the same decisions. Test/bench
infrastructure only."""
import ctypes
import os

import numpy as np
import pytest

import golden_io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "libossl_verify.so")


@pytest.fixture(scope="module")
def ossl():
    if not os.path.exists(LIB):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "openssl"], check=False)
    try:
        lib = ctypes.CDLL(LIB)
    except OSError:
        pytest.skip("libossl_verify.so not built (no OpenSSL development files)")
    P = ctypes.c_void_p
    lib.ossl_verify_batch.argtypes = [P, P, P, P, ctypes.c_size_t, ctypes.c_int, P]
    lib.ossl_verify_batch.restype = ctypes.c_int
    return lib


@pytest.mark.parametrize("name", golden_io.SETS)
def test_openssl_baseline_matches_golden(ossl, golden, name):
    g = golden[name]
    pk = np.ascontiguousarray(g.pk, dtype=np.uint8)
    sig = np.ascontiguousarray(g.sig, dtype=np.uint8)
    msg = np.ascontiguousarray(g.msg, dtype=np.uint8)
    if msg.size == 0:
        msg = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(g.off, dtype=np.uint32)
    out = np.zeros(g.n, dtype=np.uint8)
    assert ossl.ossl_verify_batch(pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, off.ctypes.data, g.n, 4,
                                  out.ctypes.data) == 0
    assert np.array_equal(out.astype(bool), g.dalek.astype(bool)), np.nonzero(out.astype(bool) != g.dalek)[0][:10]
