"""ctypes wrapper of oracle/liboracle.so — the CPU checker (TEST INFRASTRUCTURE ONLY).

Builds the oracle with `make -C oracle` when the .so is missing (gcc only; no GPU)."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
SO = os.path.join(ORACLE_DIR, "liboracle.so")


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR, "all"], check=True)


class Oracle:
    def __init__(self):
        if not os.path.exists(SO):
            build()
        L = ctypes.CDLL(SO)
        P = ctypes.c_void_p
        L.oracle_verify.argtypes = [P, P, P, ctypes.c_size_t, ctypes.c_int]
        L.oracle_verify.restype = ctypes.c_int
        L.oracle_verify_batch.argtypes = [P, P, P, P, ctypes.c_size_t, ctypes.c_int, P, ctypes.c_int]
        L.oracle_gen_records.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_size_t, P, P, P,
                                         ctypes.c_int]
        L.oracle_gen_adversarial.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_size_t, P, P,
                                             P, P, ctypes.c_int]
        L.oracle_gen_at2_transactions.argtypes = [ctypes.c_uint64, P, P, P, P, P]
        L.oracle_public_key.argtypes = [P, P]
        L.oracle_sign.argtypes = [P, P, ctypes.c_size_t, P]
        L.oracle_sha512.argtypes = [P, ctypes.c_size_t, P]
        L.oracle_sc_reduce64.argtypes = [P, P]
        L.oracle_scalarmult_base.argtypes = [P, P]
        L.oracle_point_add.argtypes = [P, P, P]
        L.oracle_point_add.restype = ctypes.c_int
        L.oracle_small_order_encoding.argtypes = [ctypes.c_int, P]
        L.oracle_decompress_ok.argtypes = [P]
        L.oracle_decompress_ok.restype = ctypes.c_int
        self.L = L

    def decompress_ok(self, p: bytes) -> bool:
        """dalek CompressedEdwardsY::decompress succeeds"""
        return bool(self.L.oracle_decompress_ok(bytes(p)))

    @staticmethod
    def _p(a):
        return a.ctypes.data if a.size else None

    def verify(self, pk: bytes, sig: bytes, msg: bytes, policy: int = 0) -> bool:
        return bool(self.L.oracle_verify(pk, sig, msg if msg else b"\0", len(msg), policy))

    def verify_batch(self, pk, sig, msg, off, policy=0, threads=os.cpu_count() or 1):
        pk = np.ascontiguousarray(pk, np.uint8); sig = np.ascontiguousarray(sig, np.uint8)
        msg = np.ascontiguousarray(msg, np.uint8).reshape(-1); off = np.ascontiguousarray(off, np.uint32)
        n = len(off) - 1
        words = np.zeros(max(1, (n + 31) // 32), np.uint32)
        m = msg if msg.size else np.zeros(1, np.uint8)
        self.L.oracle_verify_batch(self._p(pk), self._p(sig), self._p(m), self._p(off), n, policy, self._p(words),
                                   threads)
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:n]
        return bits.astype(bool)

    def gen_records(self, cfg_seed, first, n, msg_len, threads=os.cpu_count() or 1):
        pk = np.zeros((n, 32), np.uint8); sig = np.zeros((n, 64), np.uint8); msg = np.zeros(n * msg_len, np.uint8)
        self.L.oracle_gen_records(cfg_seed, first, n, msg_len, self._p(pk), self._p(sig), self._p(msg), threads)
        off = (np.arange(n + 1, dtype=np.uint64) * msg_len).astype(np.uint32)
        return pk, sig, msg, off

    def gen_adversarial(self, cfg_seed, first, n, msg_len, threads=os.cpu_count() or 1):
        pk = np.zeros((n, 32), np.uint8); sig = np.zeros((n, 64), np.uint8); msg = np.zeros(n * msg_len, np.uint8)
        cls = np.zeros(n, np.uint8)
        self.L.oracle_gen_adversarial(cfg_seed, first, n, msg_len, self._p(pk), self._p(sig), self._p(msg),
                                      self._p(cls), threads)
        off = (np.arange(n + 1, dtype=np.uint64) * msg_len).astype(np.uint32)
        return pk, sig, msg, off, cls

    def gen_at2_transactions(self, cfg_seed=0x4154325F):
        n = 4096
        pk = np.zeros((n, 32), np.uint8); sig = np.zeros((n, 64), np.uint8); msg = np.zeros(n * 48, np.uint8)
        snd = np.zeros(n, np.uint32); seq = np.zeros(n, np.uint32)
        self.L.oracle_gen_at2_transactions(cfg_seed, self._p(pk), self._p(sig), self._p(msg), self._p(snd),
                                           self._p(seq))
        off = (np.arange(n + 1) * 48).astype(np.uint32)
        return pk, sig, msg, off, snd, seq

    def public_key(self, seed: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.L.oracle_public_key(seed, out)
        return out.raw

    def sign(self, seed: bytes, msg: bytes) -> bytes:
        out = ctypes.create_string_buffer(64)
        self.L.oracle_sign(seed, msg if msg else b"\0", len(msg), out)
        return out.raw

    def sha512(self, data: bytes) -> bytes:
        out = ctypes.create_string_buffer(64)
        self.L.oracle_sha512(data if data else b"\0", len(data), out)
        return out.raw

    def scalarmult_base(self, s: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.L.oracle_scalarmult_base(s, out)
        return out.raw

    def small_order_encoding(self, idx: int) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.L.oracle_small_order_encoding(idx, out)
        return out.raw
