"""at2v — Python binding (ctypes) of libat2v.so, the MI355X batch Ed25519 verifier.

Thin plumbing over the C ABI in include/at2v.h, used by the tests and bench.py. The product is the
HIP library. This module has no Python fallback: if libat2v.so is missing, every call raises, and a GPU
context without a gfx950 device raises. The library's own CPU backend (``BatchVerifier(num_gpus=0)``, and the opt-in
``cpu_fallback`` of a GPU context) runs the kernels' verify routine compiled for the host over a thread pool; it never
routes through the oracle. ``verify_one`` is the per-signature entry point, a CPU function by contract.

Reference interface mirrored (drop::crypto::sign, used by at2-node at src/lib.rs:5,19,
src/client.rs:72-78, src/bin/server/rpc.rs:269,281):
  * ``Signature.verify(message, public_key)`` raises ``VerifyError`` on a bad signature, like
    drop's ``Signature::verify(&self, &T, &PublicKey) -> Result<(), VerifyError>``;
  * ``BatchVerifier.verify_batch(...)`` is the batch form the server ingest uses.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libat2v.so")

POLICY_DALEK_V1 = 0
POLICY_LIBSODIUM_1_0_18 = 1
_POLICIES = {"dalek": POLICY_DALEK_V1, "dalek_v1": POLICY_DALEK_V1, "libsodium": POLICY_LIBSODIUM_1_0_18,
             "libsodium_1_0_18": POLICY_LIBSODIUM_1_0_18, POLICY_DALEK_V1: POLICY_DALEK_V1,
             POLICY_LIBSODIUM_1_0_18: POLICY_LIBSODIUM_1_0_18}

# must match include/at2v.h (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = ("at2v_abi_version", "at2v_create", "at2v_destroy", "at2v_verify_batch", "at2v_verify_batch_device",
                    "at2v_verify_one", "at2v_verify_one_policy", "at2v_strerror", "at2v_gen_records_device",
                    "at2v_gen_records_senders_device", "at2v_gen_records_keys_device", "at2v_sign_batch", "at2v_get_info", "at2v_decode_points",
                    "at2v_comm_get_unique_id", "at2v_comm_init_rank", "at2v_verify_shard_gather_device",
                    "at2v_verify_batch_sharded", "at2v_verify_batch_submit", "at2v_verify_batch_wait",
                    "at2v_queue_create", "at2v_queue_destroy", "at2v_queue_submit", "at2v_queue_flush",
                    "at2v_queue_poll", "at2v_queue_get_stats", "at2v_queue_reset_latency",
                    "at2v_pack_send_asset",
                    "at2v_ledger_create", "at2v_ledger_destroy", "at2v_ledger_balance", "at2v_ledger_last_sequence",
                    "at2v_ledger_transfer", "at2v_ledger_recent_put", "at2v_ledger_recent_get",
                    "at2v_ledger_deliver", "at2v_ledger_pending")


class At2vError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        super().__init__(f"at2v error {code}: {strerror(code)}{(' (' + what + ')') if what else ''}")
        self.code = code


class VerifyError(Exception):
    """Signature rejected (drop::crypto::sign::VerifyError)."""


ABI_VERSION = 7  # include/at2v.h AT2V_ABI_VERSION: the struct layouts below are those of this version
E_PEER = -7      # AT2V_E_PEER: another rank of the communicator failed this collective batch


class _Opts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("num_gpus", ctypes.c_int), ("policy", ctypes.c_int),
                ("small_batch_max", ctypes.c_uint32), ("sender_cache", ctypes.c_uint32),
                ("sender_comb", ctypes.c_uint32), ("cpu_threads", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


CTX_CPU_FALLBACK = 1   # include/at2v.h AT2V_CTX_CPU_FALLBACK: a failed GPU batch (host buffers) re-runs on the CPU backend
CTX_ADMIT_FIRST = 2    # include/at2v.h AT2V_CTX_ADMIT_FIRST: sender-cache keys claim a payload at their first sighting
CTX_BCOMB_WIDE = 4     # include/at2v.h AT2V_CTX_BCOMB_WIDE: with combs, also a 24-bit-window comb of B (11.8 GB)


SMALL_BATCH_DEFAULT = 32768     # include/at2v.h AT2V_SMALL_BATCH_DEFAULT
SMALL_BATCH_OFF = 0xFFFFFFFF    # include/at2v.h AT2V_SMALL_BATCH_OFF: never use the low-latency kernel


class _Info(ctypes.Structure):
    _fields_ = [("num_gpus", ctypes.c_int), ("grid_blocks", ctypes.c_int), ("block_threads", ctypes.c_int),
                ("waves_per_cu", ctypes.c_int), ("cus", ctypes.c_int), ("vgprs", ctypes.c_int),
                ("rank", ctypes.c_int), ("world", ctypes.c_int), ("gathers", ctypes.c_uint64),
                ("cache_entries", ctypes.c_uint64), ("cache_chunks", ctypes.c_uint64),
                ("cache_chunk_hits", ctypes.c_uint64), ("cache_capacity", ctypes.c_uint64),
                ("cache_claims", ctypes.c_uint64), ("cache_evicted", ctypes.c_uint64),
                ("cache_compactions", ctypes.c_uint64), ("cpu_threads", ctypes.c_uint64),
                ("cpu_batches", ctypes.c_uint64), ("cpu_fallbacks", ctypes.c_uint64),
                ("cache_sightings", ctypes.c_uint64), ("cache_built", ctypes.c_uint64),
                ("cache_build_us", ctypes.c_uint64), ("cache_record_hits", ctypes.c_uint64),
                ("experiments", ctypes.c_uint64), ("host_chunks", ctypes.c_uint64)]


UNIQUE_ID_BYTES = 128  # AT2V_UNIQUE_ID_BYTES (RCCL ncclUniqueId)


_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libat2v.so (raises if it is missing: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise At2vError(-2, f"{path} not built; run `make -C at2-node_amd` or __graft_entry__.build()")
    # One HIP runtime per process: torch bundles its own libamdhip64 (same SONAME as ROCm's). If torch is
    # present it must be loaded first so libat2v.so binds to the same runtime and torch streams/pointers
    # passed to the *_device entry points belong to the runtime that launches our kernels.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    lib.at2v_abi_version.argtypes = []
    lib.at2v_abi_version.restype = ctypes.c_int
    if lib.at2v_abi_version() != ABI_VERSION:  # the structs below would not match the library's
        raise At2vError(-1, f"{path} has ABI version {lib.at2v_abi_version()}, this binding needs {ABI_VERSION}")
    P, u8p, u32p = ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint32)
    lib.at2v_create.argtypes = [ctypes.POINTER(_Opts), ctypes.POINTER(P)]
    lib.at2v_create.restype = ctypes.c_int
    lib.at2v_destroy.argtypes = [P]
    lib.at2v_destroy.restype = None
    lib.at2v_verify_batch.argtypes = [P, P, P, P, P, ctypes.c_size_t, P]
    lib.at2v_verify_batch.restype = ctypes.c_int
    lib.at2v_verify_batch_submit.argtypes = [P, P, P, P, P, ctypes.c_size_t, P, ctypes.POINTER(ctypes.c_uint64)]
    lib.at2v_verify_batch_submit.restype = ctypes.c_int
    lib.at2v_verify_batch_wait.argtypes = [P, ctypes.c_uint64]
    lib.at2v_verify_batch_wait.restype = ctypes.c_int
    lib.at2v_verify_batch_device.argtypes = [P, P, P, P, ctypes.c_size_t, P, ctypes.c_size_t, P, P]
    lib.at2v_verify_batch_device.restype = ctypes.c_int
    lib.at2v_verify_one.argtypes = [P, P, P, ctypes.c_size_t]
    lib.at2v_verify_one.restype = ctypes.c_int
    lib.at2v_verify_one_policy.argtypes = [P, P, P, ctypes.c_size_t, ctypes.c_int]
    lib.at2v_verify_one_policy.restype = ctypes.c_int
    lib.at2v_comm_get_unique_id.argtypes = [P]
    lib.at2v_comm_get_unique_id.restype = ctypes.c_int
    lib.at2v_comm_init_rank.argtypes = [P, P, ctypes.c_int, ctypes.c_int]
    lib.at2v_comm_init_rank.restype = ctypes.c_int
    lib.at2v_verify_shard_gather_device.argtypes = [P, P, P, P, ctypes.c_size_t, P, ctypes.c_size_t, ctypes.c_size_t,
                                                    P, P]
    lib.at2v_verify_shard_gather_device.restype = ctypes.c_int
    lib.at2v_verify_batch_sharded.argtypes = [P, P, P, P, P, ctypes.c_size_t, P]
    lib.at2v_verify_batch_sharded.restype = ctypes.c_int
    lib.at2v_strerror.argtypes = [ctypes.c_int]
    lib.at2v_strerror.restype = ctypes.c_char_p
    lib.at2v_gen_records_device.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint32,
                                            P, P, P, P, P]
    lib.at2v_gen_records_device.restype = ctypes.c_int
    lib.at2v_gen_records_senders_device.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t,
                                                    ctypes.c_uint32, ctypes.c_uint64, P, P, P, P, P]
    lib.at2v_gen_records_senders_device.restype = ctypes.c_int
    lib.at2v_gen_records_keys_device.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t,
                                                 ctypes.c_uint32, P, P, P, P, P, P]
    lib.at2v_gen_records_keys_device.restype = ctypes.c_int
    lib.at2v_sign_batch.argtypes = [P, P, P, P, ctypes.c_size_t, P, P]
    lib.at2v_sign_batch.restype = ctypes.c_int
    lib.at2v_get_info.argtypes = [P, ctypes.POINTER(_Info)]
    lib.at2v_get_info.restype = ctypes.c_int
    lib.at2v_decode_points.argtypes = [P, P, ctypes.c_size_t, P]
    lib.at2v_decode_points.restype = ctypes.c_int
    from . import node as _node  # queue / packer / ledger signatures
    _node.bind(lib)
    _lib = lib
    return lib


def strerror(code: int) -> str:
    try:
        return load_library().at2v_strerror(code).decode()
    except At2vError:
        return "library not loaded"


def _check(rc: int, what: str = "") -> int:
    if rc < 0:
        raise At2vError(rc, what)
    return rc


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def unpack_verdicts(words: np.ndarray, n: int) -> np.ndarray:
    """verdict words (bit i%32 of word i/32) -> bool[n]"""
    bits = np.unpackbits(np.ascontiguousarray(words, dtype="<u4").view(np.uint8), bitorder="little")
    return bits[:n].astype(bool)


def pack_records(pks: Sequence[bytes], sigs: Sequence[bytes], msgs: Sequence[bytes]):
    """lists of bytes -> (pk[n,32], sig[n,64], msg u8[], off u32[n+1]) in the ABI layout"""
    n = len(pks)
    pk = np.frombuffer(b"".join(pks), dtype=np.uint8).reshape(n, 32) if n else np.zeros((0, 32), np.uint8)
    sig = np.frombuffer(b"".join(sigs), dtype=np.uint8).reshape(n, 64) if n else np.zeros((0, 64), np.uint8)
    off = np.zeros(n + 1, dtype=np.uint32)
    if n:
        off[1:] = np.cumsum([len(m) for m in msgs])
    msg = np.frombuffer(b"".join(msgs), dtype=np.uint8) if n else np.zeros(0, np.uint8)
    return pk, sig, msg, off


def launch_streams(count: int = 2, device: Optional[int] = None) -> list:
    """`count` non-blocking HIP streams (hipStreamCreateWithFlags) on `device` (current if None), as
    torch.cuda.ExternalStream objects. Verify launches alternating over them overlap: the context's scratch sets let
    launch k+1 take the CUs launch k leaves during its end-of-launch drain (at2v_api.hip). Each stream the runtime
    creates gets its own hardware queue in turn, which is what lets the two kernels run side by side."""
    import torch

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    out = []
    with torch.cuda.device(torch.cuda.current_device() if device is None else device):
        for _ in range(count):
            h = ctypes.c_void_p()
            rc = hip.hipStreamCreateWithFlags(ctypes.byref(h), 1)  # hipStreamNonBlocking
            if rc != 0:
                raise At2vError(-3, f"hipStreamCreateWithFlags failed ({rc})")
            out.append(torch.cuda.ExternalStream(h.value))
    return out


class PendingBatch:
    """A submitted host-buffer batch (BatchVerifier.submit_batch): its ticket, verdict words and the arrays the library
    reads until the wait."""

    def __init__(self, ticket: int, n: int, words: np.ndarray, refs: tuple):
        self.ticket, self.n, self.words, self._refs = ticket, n, words, refs


class BatchVerifier:
    """Owns an at2v context: one or more gfx950 devices, or (num_gpus=0) the library's CPU batch backend."""

    def __init__(self, device: int = 0, num_gpus: int = 1, policy="dalek", small_batch_max: int = 0,
                 sender_cache: int = 0, sender_comb: bool = False, cpu_threads: int = 0, cpu_fallback: bool = False,
                 admit_first: bool = False, bcomb_wide: bool = False):
        """small_batch_max: launches of at most this many records run the low-latency kernel (two lanes per record);
        0 = the library default (SMALL_BATCH_DEFAULT), SMALL_BATCH_OFF = always the throughput kernel.
        sender_cache: capacity of the per-sender A cache in distinct public keys (0 = off).
        sender_comb: with sender_cache, also keep a comb of -A per cached key (1.7 MB of HBM each, plus combs of B of 67
        MB and 872 MB per context; include/at2v.h): records whose sender is cached verify by table additions only
        (at2v_comb.h), launches of every size. bcomb_wide: with sender_comb, the throughput kernel's comb of B gets 24-bit
        windows (11.8 GB, two additions fewer per cached record; AT2V_CTX_BCOMB_WIDE).
        num_gpus=0: the CPU batch backend (no device; cpu_threads host threads, 0 = every usable CPU).
        cpu_fallback: a GPU context re-runs a host-buffer batch on the CPU backend after a device error (same verdicts;
        info()["cpu_fallbacks"] counts it). admit_first: cache keys claim a payload at their first sighting."""
        self._lib = load_library()
        self.policy = _POLICIES[policy]
        flags = ((CTX_CPU_FALLBACK if cpu_fallback else 0) | (CTX_ADMIT_FIRST if admit_first else 0)
                 | (CTX_BCOMB_WIDE if bcomb_wide else 0))
        opts = _Opts(device, num_gpus, self.policy, small_batch_max, sender_cache, 1 if sender_comb else 0,
                     cpu_threads, flags)
        h = ctypes.c_void_p()
        _check(self._lib.at2v_create(ctypes.byref(opts), ctypes.byref(h)), "at2v_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.at2v_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def info(self) -> dict:
        inf = _Info()
        _check(self._lib.at2v_get_info(self._h, ctypes.byref(inf)), "at2v_get_info")
        return {f: getattr(inf, f) for f, _ in _Info._fields_}

    def verify_batch(self, pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, msg_off: np.ndarray) -> np.ndarray:
        """host arrays -> bool[n] verdicts"""
        pk = np.ascontiguousarray(pk, dtype=np.uint8)
        sig = np.ascontiguousarray(sig, dtype=np.uint8)
        msg = np.ascontiguousarray(msg, dtype=np.uint8).reshape(-1)
        msg_off = np.ascontiguousarray(msg_off, dtype=np.uint32)
        n = len(msg_off) - 1
        if pk.size != 32 * n or sig.size != 64 * n:
            raise ValueError("pk/sig/msg_off sizes disagree")
        words = np.zeros(max(1, (n + 31) // 32), dtype=np.uint32)
        msg_arg = msg if msg.size else np.zeros(1, np.uint8)
        _check(self._lib.at2v_verify_batch(self._h, _ptr(pk), _ptr(sig), _ptr(msg_arg), _ptr(msg_off), n,
                                           _ptr(words)), "at2v_verify_batch")
        return unpack_verdicts(words, n)

    def submit_batch(self, pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, msg_off: np.ndarray) -> "PendingBatch":
        """at2v_verify_batch_submit: stage the batch and enqueue its verification; returns the pending call (it holds
        the arrays until wait_batch). At most two in flight per context."""
        pk = np.ascontiguousarray(pk, dtype=np.uint8)
        sig = np.ascontiguousarray(sig, dtype=np.uint8)
        msg = np.ascontiguousarray(msg, dtype=np.uint8).reshape(-1)
        msg_off = np.ascontiguousarray(msg_off, dtype=np.uint32)
        n = len(msg_off) - 1
        if pk.size != 32 * n or sig.size != 64 * n:
            raise ValueError("pk/sig/msg_off sizes disagree")
        words = np.zeros(max(1, (n + 31) // 32), dtype=np.uint32)
        msg_arg = msg if msg.size else np.zeros(1, np.uint8)
        t = ctypes.c_uint64(0)
        _check(self._lib.at2v_verify_batch_submit(self._h, _ptr(pk), _ptr(sig), _ptr(msg_arg), _ptr(msg_off), n,
                                                  _ptr(words), ctypes.byref(t)), "at2v_verify_batch_submit")
        return PendingBatch(t.value, n, words, (pk, sig, msg_arg, msg_off))

    def wait_batch(self, pending: "PendingBatch") -> np.ndarray:
        """at2v_verify_batch_wait -> bool[n] verdicts of a submitted batch"""
        _check(self._lib.at2v_verify_batch_wait(self._h, pending.ticket), "at2v_verify_batch_wait")
        return unpack_verdicts(pending.words, pending.n)

    def verify_batch_device(self, d_pk: int, d_sig: int, d_msg: int, msg_bytes: int, d_off: int, n: int,
                            d_verdicts: int, stream: int = 0) -> None:
        """device pointers (e.g. torch tensor data_ptr()), asynchronous on `stream` (a hipStream_t)"""
        _check(self._lib.at2v_verify_batch_device(self._h, d_pk, d_sig, d_msg, msg_bytes, d_off, n, d_verdicts,
                                                  stream or None), "at2v_verify_batch_device")

    # ---- one rank per GPU: RCCL all-gather of the verdict words (include/at2v.h)
    def comm_init_rank(self, unique_id: bytes, rank: int, world: int) -> None:
        """Attach an RCCL communicator (collective over `world` processes; unique_id from comm_unique_id() on
        rank 0, shared out of band)."""
        if len(unique_id) != UNIQUE_ID_BYTES:
            raise ValueError("unique id must be %d bytes" % UNIQUE_ID_BYTES)
        _check(self._lib.at2v_comm_init_rank(self._h, bytes(unique_id), rank, world), "at2v_comm_init_rank")

    def verify_shard_gather_device(self, d_pk: int, d_sig: int, d_msg: int, msg_bytes: int, d_off: int,
                                   n_local: int, words_per_rank: int, d_bitmap: int, stream: int = 0) -> None:
        """verify this rank's n_local device records into its slice of d_bitmap, then all-gather (asynchronous)"""
        _check(self._lib.at2v_verify_shard_gather_device(self._h, d_pk or None, d_sig or None, d_msg or None,
                                                         msg_bytes, d_off or None, n_local, words_per_rank,
                                                         d_bitmap, stream or None),
               "at2v_verify_shard_gather_device")

    def verify_batch_sharded(self, pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, msg_off: np.ndarray) -> np.ndarray:
        """the node batch (same on every rank) -> bool[n] verdicts of the whole batch on every rank"""
        pk = np.ascontiguousarray(pk, dtype=np.uint8)
        sig = np.ascontiguousarray(sig, dtype=np.uint8)
        msg = np.ascontiguousarray(msg, dtype=np.uint8).reshape(-1)
        msg_off = np.ascontiguousarray(msg_off, dtype=np.uint32)
        n = len(msg_off) - 1
        if pk.size != 32 * n or sig.size != 64 * n:
            raise ValueError("pk/sig/msg_off sizes disagree")
        words = np.zeros(max(1, (n + 31) // 32), dtype=np.uint32)
        msg_arg = msg if msg.size else np.zeros(1, np.uint8)
        _check(self._lib.at2v_verify_batch_sharded(self._h, _ptr(pk), _ptr(sig), _ptr(msg_arg), _ptr(msg_off), n,
                                                   _ptr(words)), "at2v_verify_batch_sharded")
        return unpack_verdicts(words, n)

    def gen_records_device(self, cfg_seed: int, first: int, n: int, msg_len: int, d_pk: int, d_sig: int, d_msg: int,
                           d_off: Optional[int], stream: int = 0, senders: int = 0) -> None:
        """GPU generator; senders > 0: record i is signed by sender (first + i) % senders"""
        if senders:
            _check(self._lib.at2v_gen_records_senders_device(self._h, cfg_seed, first, n, msg_len, senders, d_pk, d_sig,
                                                             d_msg, d_off or None, stream or None),
                   "at2v_gen_records_senders_device")
            return
        _check(self._lib.at2v_gen_records_device(self._h, cfg_seed, first, n, msg_len, d_pk, d_sig, d_msg,
                                                 d_off or None, stream or None), "at2v_gen_records_device")

    def gen_records_keys_device(self, cfg_seed: int, first: int, n: int, msg_len: int, d_keys: int, d_pk: int,
                                d_sig: int, d_msg: int, d_off: Optional[int], stream: int = 0) -> None:
        """GPU generator with a key per record: record i signed by seed index d_keys[i] (u64 device array)"""
        _check(self._lib.at2v_gen_records_keys_device(self._h, cfg_seed, first, n, msg_len, d_keys, d_pk, d_sig, d_msg,
                                                      d_off or None, stream or None), "at2v_gen_records_keys_device")

    def decode_points(self, pts: np.ndarray) -> np.ndarray:
        """bool[n]: 32-byte encodings that decode under dalek rules (GPU kernel)"""
        pts = np.ascontiguousarray(pts, dtype=np.uint8).reshape(-1, 32)
        n = len(pts)
        words = np.zeros(max(1, (n + 31) // 32), dtype=np.uint32)
        _check(self._lib.at2v_decode_points(self._h, _ptr(pts), n, _ptr(words)), "at2v_decode_points")
        return unpack_verdicts(words, n)

    def sign_batch(self, seeds: np.ndarray, msg: np.ndarray, msg_off: np.ndarray):
        seeds = np.ascontiguousarray(seeds, dtype=np.uint8)
        msg = np.ascontiguousarray(msg, dtype=np.uint8).reshape(-1)
        msg_off = np.ascontiguousarray(msg_off, dtype=np.uint32)
        n = len(msg_off) - 1
        pk = np.zeros((n, 32), np.uint8)
        sig = np.zeros((n, 64), np.uint8)
        msg_arg = msg if msg.size else np.zeros(1, np.uint8)
        _check(self._lib.at2v_sign_batch(self._h, _ptr(seeds), _ptr(msg_arg), _ptr(msg_off), n, _ptr(pk), _ptr(sig)),
               "at2v_sign_batch")
        return pk, sig


def comm_unique_id() -> bytes:
    """RCCL unique id for at2v_comm_init_rank (rank 0 creates it; hand it to the other ranks out of band)"""
    buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    _check(load_library().at2v_comm_get_unique_id(buf), "at2v_comm_get_unique_id")
    return buf.raw


def verify_one(pk: bytes, sig: bytes, msg: bytes, policy="dalek") -> bool:
    """One signature on the CPU (at2v_verify_one: the product's verify code built for the host; no GPU)."""
    lib = load_library()
    if len(pk) != 32 or len(sig) != 64:
        raise ValueError("public key must be 32 bytes and signature 64 bytes")
    return bool(_check(lib.at2v_verify_one_policy(bytes(pk), bytes(sig), bytes(msg) if msg else None, len(msg),
                                                  _POLICIES[policy]), "at2v_verify_one_policy"))


# ------------------------------------------------ drop::crypto::sign mirror
class PublicKey:
    """32-byte Ed25519 public key (drop::crypto::sign::PublicKey). Decoding is checked by verify."""

    def __init__(self, data: bytes):
        if len(data) != 32:
            raise ValueError("public key must be 32 bytes")
        self.bytes = bytes(data)

    def __bytes__(self):
        return self.bytes

    def __eq__(self, other):
        return isinstance(other, PublicKey) and other.bytes == self.bytes

    def __hash__(self):
        return hash(self.bytes)

    def __repr__(self):
        return f"PublicKey({self.bytes.hex()})"


class Signature:
    """64-byte Ed25519 signature R || S (drop::crypto::sign::Signature)."""

    def __init__(self, data: bytes):
        if len(data) != 64:
            raise ValueError("signature must be 64 bytes")
        self.bytes = bytes(data)

    def verify(self, message: bytes, public_key: PublicKey) -> None:
        """Raise VerifyError unless the signature is valid (at2v_verify_one: the per-signature CPU entry point,
        as drop's synchronous verify is; batches go through BatchVerifier on the GPU)."""
        if not verify_one(public_key.bytes, self.bytes, bytes(message)):
            raise VerifyError("signature verification failed")
