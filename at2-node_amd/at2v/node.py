"""at2v.node — Python binding of the host-side pieces around the verify kernel (include/at2v.h):

* ``IngestQueue``   the server's transaction ingest/batching queue (at2v_queue_*), GPU-backed;
* ``pack_send_asset`` SendAssetRequest fields -> verify records (at2v_pack_send_asset);
* ``Ledger``        accounts + recent transactions + the deliver/apply loop (at2v_ledger_*).

Reference interfaces mirrored (/root/reference):
  * ``Ledger.transfer / balance / last_sequence`` = ``Accounts`` (src/bin/server/accounts/mod.rs:57-117),
    error codes = ``account::Error`` (accounts/account.rs:3-8);
  * ``Ledger.recent_put / recent`` = ``RecentTransactions`` (src/bin/server/recent_transactions.rs:47-109);
  * ``Ledger.deliver`` = one ``deliver()`` batch through ``Service::spawn`` (src/bin/server/rpc.rs:149-211);
  * ``pack_send_asset`` = the decode half of ``At2::send_asset`` (rpc.rs:258-287).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

TX_OK, TX_INCONSECUTIVE_SEQUENCE, TX_OVERFLOW, TX_UNDERFLOW = 0, 1, 2, 3
TX_PENDING, TX_SUCCESS, TX_FAILURE = 0, 1, 2
WIRE_BYTES, WIRE_ARRAY = 0, 1
PACK_OK, PACK_BAD_RECIPIENT, PACK_BAD_SENDER, PACK_BAD_SIGNATURE = 0, 1, 2, 3
INITIAL_BALANCE = 100000  # accounts/account.rs:17


VERDICT_INVALID, VERDICT_VALID, VERDICT_FAILED = 0, 1, 0xFF  # at2v_queue_poll verdict bytes (at2v.h)


class BatchFailedError(RuntimeError):
    """Verdicts from a batch that failed on the device (at2v_queue_poll reports 0xff for each of its records).
    Nothing from such a batch may be treated as verified: the caller re-submits it or drops it."""


def verdict_mask(verdicts, n: int) -> np.ndarray:
    """Per-record verdicts -> bool[n] of VALID records, failing closed.

    Accepts bool[n], or integers [n] that are each 0 (invalid) or 1 (valid) — the queue's uint8 verdicts.
    A 0xff (failed batch) raises BatchFailedError; any other value raises ValueError. Only == 1 counts as
    valid, so a device failure can never turn into an approval."""
    v = np.asarray(verdicts)
    if v.shape != (n,):
        raise ValueError(f"expected {n} per-record verdicts, got shape {v.shape}")
    if v.dtype == bool:
        return v.copy()
    if not np.issubdtype(v.dtype, np.integer):
        raise ValueError(f"verdicts must be bool or integer, not {v.dtype}")
    if (v == VERDICT_FAILED).any():
        raise BatchFailedError(f"{int((v == VERDICT_FAILED).sum())} records come from a batch that failed on the device")
    if ((v != VERDICT_INVALID) & (v != VERDICT_VALID)).any():
        raise ValueError("per-record verdicts must be 0 or 1")
    return v == VERDICT_VALID


class AccountError(Exception):
    """accounts::Error::AccountModification { source: account::Error } (accounts/mod.rs:16-18)."""

    NAMES = {TX_INCONSECUTIVE_SEQUENCE: "InconsecutiveSequence", TX_OVERFLOW: "Overflow", TX_UNDERFLOW: "Underflow"}

    def __init__(self, code: int):
        super().__init__(self.NAMES.get(code, str(code)))
        self.code = code


QUEUE_EAGER = 1  # include/at2v.h AT2V_QUEUE_EAGER: also seal whenever no batch is in flight
QUEUE_SENDER_COMB = 2  # include/at2v.h AT2V_QUEUE_SENDER_COMB: per-sender combs in the queue's context
QUEUE_CPU = 4  # include/at2v.h AT2V_QUEUE_CPU: batches verified by the CPU backend (no device)
QUEUE_CPU_FALLBACK = 8  # include/at2v.h AT2V_QUEUE_CPU_FALLBACK: a batch that fails on the device re-runs on the CPU


class _QueueOpts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("policy", ctypes.c_int), ("max_batch", ctypes.c_uint32),
                ("max_delay_us", ctypes.c_uint32), ("max_msg_bytes", ctypes.c_uint32), ("depth", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("sender_cache", ctypes.c_uint32), ("cpu_threads", ctypes.c_uint32)]


class _QueueStats(ctypes.Structure):
    _fields_ = [("submitted", ctypes.c_uint64), ("completed", ctypes.c_uint64), ("batches", ctypes.c_uint64),
                ("failed_batches", ctypes.c_uint64), ("mean_batch", ctypes.c_double), ("p50_us", ctypes.c_double),
                ("p99_us", ctypes.c_double), ("max_us", ctypes.c_double), ("cpu_fallbacks", ctypes.c_uint64)]


class _SendAsset(ctypes.Structure):
    _fields_ = [("sender", ctypes.c_void_p), ("sender_len", ctypes.c_size_t), ("sequence", ctypes.c_uint32),
                ("recipient", ctypes.c_void_p), ("recipient_len", ctypes.c_size_t), ("amount", ctypes.c_uint64),
                ("signature", ctypes.c_void_p), ("signature_len", ctypes.c_size_t)]


class _FullTx(ctypes.Structure):
    _fields_ = [("timestamp_us", ctypes.c_uint64), ("sender", ctypes.c_uint8 * 32), ("sender_sequence", ctypes.c_uint32),
                ("recipient", ctypes.c_uint8 * 32), ("amount", ctypes.c_uint64), ("state", ctypes.c_int32)]


class _ApplyStats(ctypes.Structure):
    _fields_ = [("delivered", ctypes.c_uint64), ("rejected", ctypes.c_uint64), ("applied", ctypes.c_uint64),
                ("requeued", ctypes.c_uint64), ("expired", ctypes.c_uint64), ("passes", ctypes.c_uint64)]


def bind(lib) -> None:
    P, sz, u32, u64, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    sig = {
        "at2v_queue_create": ([ctypes.POINTER(_QueueOpts), ctypes.POINTER(P)], i32),
        "at2v_queue_destroy": ([P], None),
        "at2v_queue_submit": ([P, P, P, P, P, sz, ctypes.POINTER(u64)], i32),
        "at2v_queue_flush": ([P], i32),
        "at2v_queue_poll": ([P, P, P, sz, u32], ctypes.c_long),
        "at2v_queue_get_stats": ([P, ctypes.POINTER(_QueueStats)], i32),
        "at2v_queue_reset_latency": ([P], i32),
        "at2v_pack_send_asset": ([P, sz, i32, P, P, P, P, P, P], ctypes.c_long),
        "at2v_ledger_create": ([ctypes.POINTER(P)], i32),
        "at2v_ledger_destroy": ([P], None),
        "at2v_ledger_balance": ([P, P, ctypes.POINTER(u64)], i32),
        "at2v_ledger_last_sequence": ([P, P, ctypes.POINTER(u32)], i32),
        "at2v_ledger_transfer": ([P, P, u32, P, u64], i32),
        "at2v_ledger_recent_put": ([P, P, u32, P, u64, u64], i32),
        "at2v_ledger_recent_get": ([P, P, sz], ctypes.c_long),
        "at2v_ledger_deliver": ([P, P, P, P, P, P, sz, u64, ctypes.POINTER(_ApplyStats)], i32),
        "at2v_ledger_pending": ([P], ctypes.c_long),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res


def _lib():
    from . import load_library
    return load_library()


def _chk(rc: int, what: str) -> int:
    from . import _check
    return _check(rc, what)


def _p(a: np.ndarray):
    return a.ctypes.data if a.size else None


# ------------------------------------------------------------------ ingest queue
class IngestQueue:
    """GPU-backed batching queue: submit records, poll (ticket, verdict) in submission order."""

    def __init__(self, device: int = 0, policy="dalek", max_batch: int = 65536, max_delay_us: int = 1000,
                 max_msg_bytes: int = 256, depth: int = 3, eager: bool = False, sender_comb: bool = False,
                 sender_cache: int = 0, cpu: bool = False, cpu_fallback: bool = False, cpu_threads: int = 0):
        """eager: also seal whenever no batch is in flight (latency mode); sender_comb: per-sender combs in the queue's
        context (at2v_comb.h) for `sender_cache` keys (0 = 1024; 1.7 MB of HBM per key); cpu: verify on the library's
        CPU backend (no device); cpu_fallback: a batch that fails on the device is verified on the CPU backend instead"""
        from . import _POLICIES
        self._lib = _lib()
        flags = ((QUEUE_EAGER if eager else 0) | (QUEUE_SENDER_COMB if sender_comb else 0) | (QUEUE_CPU if cpu else 0)
                 | (QUEUE_CPU_FALLBACK if cpu_fallback else 0))
        o = _QueueOpts(device, _POLICIES[policy], max_batch, max_delay_us, max_msg_bytes, depth, flags, sender_cache,
                       cpu_threads)
        h = ctypes.c_void_p()
        _chk(self._lib.at2v_queue_create(ctypes.byref(o), ctypes.byref(h)), "at2v_queue_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.at2v_queue_destroy(self._h)
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

    def submit(self, pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, msg_off: np.ndarray) -> int:
        """n records (ABI layout) -> ticket of the first; the call's records get consecutive tickets"""
        pk = np.ascontiguousarray(pk, np.uint8)
        sig = np.ascontiguousarray(sig, np.uint8)
        msg = np.ascontiguousarray(msg, np.uint8).reshape(-1)
        off = np.ascontiguousarray(msg_off, np.uint32)
        n = len(off) - 1
        if pk.size != 32 * n or sig.size != 64 * n:
            raise ValueError("pk/sig/msg_off sizes disagree")
        first = ctypes.c_uint64(0)
        m = msg if msg.size else np.zeros(1, np.uint8)
        _chk(self._lib.at2v_queue_submit(self._h, _p(pk), _p(sig), _p(m), _p(off), n, ctypes.byref(first)),
             "at2v_queue_submit")
        return first.value

    def flush(self) -> None:
        _chk(self._lib.at2v_queue_flush(self._h), "at2v_queue_flush")

    def poll(self, max_items: int = 65536, timeout_us: int = 0):
        """-> (tickets u64[k], verdicts u8[k]) in ticket order; a verdict is 1 (valid), 0 (invalid) or 0xff
        (its batch failed on the device: not verified either way). Turn them into a valid-mask with
        verdict_mask(), which refuses 0xff, never with astype(bool)."""
        t = np.zeros(max_items, np.uint64)
        v = np.zeros(max_items, np.uint8)
        k = _chk(self._lib.at2v_queue_poll(self._h, _p(t), _p(v), max_items, timeout_us), "at2v_queue_poll")
        return t[:k], v[:k]

    def stats(self) -> dict:
        s = _QueueStats()
        _chk(self._lib.at2v_queue_get_stats(self._h, ctypes.byref(s)), "at2v_queue_get_stats")
        return {f: getattr(s, f) for f, _ in _QueueStats._fields_}

    def reset_latency(self) -> None:
        _chk(self._lib.at2v_queue_reset_latency(self._h), "at2v_queue_reset_latency")


# ------------------------------------------------------------------ record packer
@dataclass
class SendAssetRequest:
    """src/at2.proto:10-16 (bytes fields hold bincode-encoded drop types)."""
    sender: bytes
    sequence: int
    recipient: bytes
    amount: int
    signature: bytes


def wire_key(pk: bytes, wire: int = WIRE_BYTES) -> bytes:
    """bincode(sign::PublicKey) under the assumed serde encoding"""
    return (len(pk).to_bytes(8, "little") + pk) if wire == WIRE_BYTES else bytes(pk)


def wire_signature(sig: bytes, wire: int = WIRE_BYTES) -> bytes:
    return (len(sig).to_bytes(8, "little") + sig) if wire == WIRE_BYTES else bytes(sig)


def thin_transaction(recipient: bytes, amount: int, wire: int = WIRE_BYTES) -> bytes:
    """M = bincode(ThinTransaction{recipient, amount}) (src/lib.rs:14-22)"""
    return wire_key(recipient, wire) + int(amount).to_bytes(8, "little")


def pack_send_asset(reqs: Sequence[SendAssetRequest], wire: int = WIRE_BYTES):
    """-> dict(pk[n,32], sig[n,64], msg u8[], off u32[n+1], recipient[n,32], sequence u32[n], amount u64[n],
    status u8[n]) — the verify records plus the fields the apply step needs"""
    lib = _lib()
    n = len(reqs)
    keep = []
    arr = (_SendAsset * max(1, n))()
    for i, r in enumerate(reqs):
        bufs = [ctypes.create_string_buffer(bytes(b), max(1, len(b))) for b in (r.sender, r.recipient, r.signature)]
        keep.append(bufs)
        arr[i] = _SendAsset(ctypes.addressof(bufs[0]), len(r.sender), r.sequence, ctypes.addressof(bufs[1]),
                            len(r.recipient), r.amount, ctypes.addressof(bufs[2]), len(r.signature))
    mlen = 48 if wire == WIRE_BYTES else 40
    pk = np.zeros((n, 32), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    msg = np.zeros(max(1, n * mlen), np.uint8)
    off = np.zeros(n + 1, np.uint32)
    rcp = np.zeros((n, 32), np.uint8)
    st = np.zeros(max(1, n), np.uint8)
    _chk(lib.at2v_pack_send_asset(ctypes.addressof(arr), n, wire, _p(pk), _p(sig), _p(msg), _p(off), _p(rcp), _p(st)),
         "at2v_pack_send_asset")
    return {"pk": pk, "sig": sig, "msg": msg[: int(off[-1])], "off": off, "recipient": rcp,
            "sequence": np.array([r.sequence for r in reqs], np.uint32),
            "amount": np.array([r.amount for r in reqs], np.uint64), "status": st[:n]}


# ------------------------------------------------------------------ ledger
@dataclass
class FullTransaction:
    timestamp_us: int
    sender: bytes
    sender_sequence: int
    recipient: bytes
    amount: int
    state: int


class Ledger:
    """Accounts + recent transactions + deliver/apply loop of one AT2 node (host C++, libat2v.so)."""

    def __init__(self):
        self._lib = _lib()
        h = ctypes.c_void_p()
        _chk(self._lib.at2v_ledger_create(ctypes.byref(h)), "at2v_ledger_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.at2v_ledger_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def balance(self, pk: bytes) -> int:
        out = ctypes.c_uint64()
        _chk(self._lib.at2v_ledger_balance(self._h, bytes(pk), ctypes.byref(out)), "at2v_ledger_balance")
        return out.value

    def last_sequence(self, pk: bytes) -> int:
        out = ctypes.c_uint32()
        _chk(self._lib.at2v_ledger_last_sequence(self._h, bytes(pk), ctypes.byref(out)), "at2v_ledger_last_sequence")
        return out.value

    def transfer(self, sender: bytes, sequence: int, recipient: bytes, amount: int) -> None:
        """Accounts::transfer; raises AccountError on InconsecutiveSequence / Overflow / Underflow"""
        rc = _chk(self._lib.at2v_ledger_transfer(self._h, bytes(sender), sequence, bytes(recipient), amount),
                  "at2v_ledger_transfer")
        if rc:
            raise AccountError(rc)

    def recent_put(self, sender: bytes, sequence: int, recipient: bytes, amount: int, now_us: int = 0) -> None:
        _chk(self._lib.at2v_ledger_recent_put(self._h, bytes(sender), sequence, bytes(recipient), amount, now_us),
             "at2v_ledger_recent_put")

    def recent(self) -> List[FullTransaction]:
        buf = (_FullTx * 16)()
        k = _chk(self._lib.at2v_ledger_recent_get(self._h, ctypes.addressof(buf), 16), "at2v_ledger_recent_get")
        return [FullTransaction(t.timestamp_us, bytes(t.sender), t.sender_sequence, bytes(t.recipient), t.amount,
                                t.state) for t in buf[:k]]

    def deliver(self, sender: np.ndarray, sequence: np.ndarray, recipient: np.ndarray, amount: np.ndarray,
                verdicts: Optional[np.ndarray] = None, now_us: int = 0, words: Optional[np.ndarray] = None) -> dict:
        """One delivered batch. Which records were verified is given by exactly one of
          * `verdicts`: per-record bool[n] or 0/1 integers (the queue's uint8 verdicts; 0xff = failed batch
            raises BatchFailedError before anything is applied — see verdict_mask);
          * `words`: the verify call's uint32 verdict bitmap (bit i%32 of word i/32), ceil(n/32) words;
          * neither: every record is delivered."""
        sender = np.ascontiguousarray(sender, np.uint8).reshape(-1, 32)
        n = len(sender)
        seq = np.ascontiguousarray(sequence, np.uint32)
        rcp = np.ascontiguousarray(recipient, np.uint8).reshape(-1, 32)
        amt = np.ascontiguousarray(amount, np.uint64)
        if len(seq) != n or len(rcp) != n or len(amt) != n:
            raise ValueError("field lengths disagree")
        if verdicts is not None and words is not None:
            raise ValueError("give per-record verdicts or bitmap words, not both")
        if verdicts is not None:
            ok = verdict_mask(verdicts, n)
            words = np.packbits(ok.astype(np.uint8), bitorder="little")
            words = np.concatenate([words, np.zeros((-len(words)) % 4, np.uint8)]).view("<u4")
        elif words is not None:
            w = np.asarray(words)
            if w.dtype not in (np.uint32, np.int32) or w.shape != ((n + 31) // 32,):
                raise ValueError(f"bitmap words must be {(n + 31) // 32} uint32/int32 words")
            words = np.ascontiguousarray(w).view("<u4")
        st = _ApplyStats()
        _chk(self._lib.at2v_ledger_deliver(self._h, _p(sender), _p(seq), _p(rcp), _p(amt),
                                           _p(words) if words is not None else None, n, now_us, ctypes.byref(st)),
             "at2v_ledger_deliver")
        return {f: getattr(st, f) for f, _ in _ApplyStats._fields_}

    def pending(self) -> int:
        return _chk(self._lib.at2v_ledger_pending(self._h), "at2v_ledger_pending")
