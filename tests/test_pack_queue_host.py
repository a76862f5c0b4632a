"""CPU: the record packer (at2v_pack_send_asset in libat2v.so) and the batching-queue core
(at2-node_amd/csrc/at2v_queue.h) compiled for the host with the oracle as its verify backend
(tests/host/queue_host.cpp). The shipped queue runs on the GPU backend (tests/test_gpu_node.py)."""
import os
import subprocess

import numpy as np
import pytest

from at2v import node
from at2v.node import (PACK_BAD_RECIPIENT, PACK_BAD_SENDER, PACK_BAD_SIGNATURE, PACK_OK, WIRE_ARRAY, WIRE_BYTES,
                       SendAssetRequest, pack_send_asset, thin_transaction, wire_key, wire_signature)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_thin_transaction_layout_matches_oracle(oracle):
    """M = bincode(ThinTransaction) = u64le(32) || recipient || u64le(amount) (oracle_thin_transaction)"""
    import ctypes
    r = bytes(range(32))
    out = ctypes.create_string_buffer(48)
    oracle.L.oracle_thin_transaction.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    oracle.L.oracle_thin_transaction(r, 123456789, out)
    assert thin_transaction(r, 123456789) == out.raw
    assert thin_transaction(r, 7, WIRE_ARRAY) == r + (7).to_bytes(8, "little")


def test_pack_send_asset_round_trip_config1(oracle):
    """config-1 AT2 transactions (oracle generator: 64 senders x sequences 1..64) re-packed from their wire
    form give back exactly the records that were signed"""
    pk, sig, msg, off, snd, seq = oracle.gen_at2_transactions()
    n = 256
    reqs = []
    for i in range(n):
        m = msg[off[i]:off[i + 1]].tobytes()
        recipient, amount = m[8:40], int.from_bytes(m[40:48], "little")
        reqs.append(SendAssetRequest(wire_key(pk[i].tobytes()), int(seq[i]), wire_key(recipient), amount,
                                     wire_signature(sig[i].tobytes())))
    out = pack_send_asset(reqs)
    assert (out["status"] == PACK_OK).all()
    assert np.array_equal(out["pk"], pk[:n]) and np.array_equal(out["sig"], sig[:n])
    assert np.array_equal(out["off"], off[:n + 1]) and np.array_equal(out["msg"], msg[:off[n]])
    assert np.array_equal(out["sequence"], seq[:n])
    # and the oracle accepts every packed record
    assert oracle.verify_batch(out["pk"], out["sig"], out["msg"], out["off"]).all()


def test_pack_send_asset_decode_errors_in_reference_order():
    good_k, good_s = wire_key(b"\x01" * 32), wire_signature(b"\x02" * 64)
    reqs = [
        SendAssetRequest(good_k, 1, good_k, 5, good_s),                       # ok
        SendAssetRequest(good_k, 1, b"\x20" + b"\0" * 7 + b"\x01" * 31, 5, good_s),  # short recipient
        SendAssetRequest(b"\x21" + b"\0" * 7 + b"\x01" * 33, 1, good_k, 5, good_s),  # wrong length prefix
        SendAssetRequest(good_k, 1, good_k, 5, wire_key(b"\x02" * 32)),       # 32-byte "signature"
        SendAssetRequest(b"", 1, b"", 5, b""),                                # recipient is checked first
        SendAssetRequest(good_k + b"trailing", 1, good_k + b"x", 5, good_s + b"y"),  # bincode allows trailing bytes
    ]
    out = pack_send_asset(reqs)
    assert list(out["status"]) == [PACK_OK, PACK_BAD_RECIPIENT, PACK_BAD_SENDER, PACK_BAD_SIGNATURE,
                                   PACK_BAD_RECIPIENT, PACK_OK]
    # failed records keep their index with an empty message
    lens = np.diff(out["off"])
    assert list(lens) == [48, 0, 0, 0, 0, 48]
    assert not out["pk"][1:5].any()


def test_pack_array_wire_encoding():
    r = SendAssetRequest(b"\x03" * 32, 9, b"\x04" * 32, 77, b"\x05" * 64)
    out = pack_send_asset([r], wire=WIRE_ARRAY)
    assert out["status"][0] == PACK_OK and out["msg"].tobytes() == b"\x04" * 32 + (77).to_bytes(8, "little")
    out = pack_send_asset([r], wire=WIRE_BYTES)  # 32 raw bytes are not a valid bincode byte string
    assert out["status"][0] == PACK_BAD_RECIPIENT


def test_pack_empty():
    out = pack_send_asset([])
    assert out["pk"].shape == (0, 32) and list(out["off"]) == [0]


# host builds of the queue core: plain, AddressSanitizer + UBSan, ThreadSanitizer (the product's threaded host
# code; the oracle backend library itself is not instrumented)
SANITIZE = {"plain": [], "asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"],
            "tsan": ["-fsanitize=thread", "-include", os.path.join(ROOT, "tests", "host", "tsan_compat.h")]}


@pytest.fixture(scope="module")
def queue_host():
    oracle_dir = os.path.join(ROOT, "oracle")
    subprocess.run(["make", "-s", "-C", oracle_dir, "all"], check=True)
    exes = {}
    for kind, flags in SANITIZE.items():
        exe = os.path.join(ROOT, "tests", "host", "queue_host" + ("" if kind == "plain" else "_" + kind))
        subprocess.run(["g++", "-O1" if flags else "-O2", "-g", "-std=c++17", "-pthread", *flags,
                        "-I" + os.path.join(ROOT, "at2-node_amd", "csrc"),
                        os.path.join(ROOT, "tests", "host", "queue_host.cpp"), "-L" + oracle_dir, "-loracle",
                        "-Wl,-rpath," + oracle_dir, "-o", f"{exe}.{os.getpid()}"], check=True)
        os.replace(f"{exe}.{os.getpid()}", exe)  # atomic: parallel workers (pytest -n) never run a half-written file
        exes[kind] = exe
    return exes


@pytest.mark.parametrize("build", list(SANITIZE))
@pytest.mark.parametrize("scenario", ["order", "size", "deadline", "flush", "eager", "eager_order", "drain", "startfail", "failed"])
def test_queue_core_on_host(queue_host, scenario, build):
    """order: 4 producer threads, random run lengths, verdicts map back through tickets (oracle backend);
    size: a full batch seals at max_batch; deadline: a partial batch seals at max_delay_us;
    flush: explicit seal, oversized message rejected; eager_order: latency mode with 4 producers, batches launched by
    producers, the completer and the launcher thread, ticket order kept; drain: destroy completes everything submitted;
    startfail: a start() that fails part-way frees every slot; failed: a batch whose launch fails
    reports 0xff for its records and is counted in failed_batches. Each under ASan+UBSan and TSan too."""
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:halt_on_error=1")
    out = subprocess.run([queue_host[build], scenario], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stdout + out.stderr[-4000:]
