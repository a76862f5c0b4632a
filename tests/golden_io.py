"""Reader for tests/golden/*.bin (format: tests/golden/README.md). Data only; no code is loaded."""
import os
import struct
from dataclasses import dataclass

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SETS = ("rfc8032", "at2_cfg1", "adversarial", "edge", "ragged")


@dataclass
class FixtureSet:
    name: str
    pk: np.ndarray      # (n, 32) u8
    sig: np.ndarray     # (n, 64) u8
    off: np.ndarray     # (n+1,) u32
    msg: np.ndarray     # (bytes,) u8
    dalek: np.ndarray   # (n,) bool  — OpenSSL 3.0.2 verdicts (policy DALEK_V1)
    sodium: np.ndarray  # (n,) bool  — libsodium 1.0.18 verdicts
    cls: np.ndarray     # (n,) u8

    @property
    def n(self):
        return len(self.pk)

    def message(self, i):
        return self.msg[self.off[i]:self.off[i + 1]].tobytes()


def load(name: str) -> FixtureSet:
    b = open(os.path.join(GOLDEN_DIR, name + ".bin"), "rb").read()
    magic, ver, n, mb = struct.unpack_from("<4I", b, 0)
    assert magic == 0x56325441 and ver == 1, name
    o = 16
    pk = np.frombuffer(b, np.uint8, 32 * n, o).reshape(n, 32); o += 32 * n
    sig = np.frombuffer(b, np.uint8, 64 * n, o).reshape(n, 64); o += 64 * n
    off = np.frombuffer(b, "<u4", n + 1, o).astype(np.uint32); o += 4 * (n + 1)
    msg = np.frombuffer(b, np.uint8, mb, o); o += mb
    dalek = np.frombuffer(b, np.uint8, n, o).astype(bool); o += n
    sodium = np.frombuffer(b, np.uint8, n, o).astype(bool); o += n
    cls = np.frombuffer(b, np.uint8, n, o); o += n
    assert o == len(b), name
    return FixtureSet(name, pk, sig, off, msg, dalek, sodium, cls)


def load_all():
    return {s: load(s) for s in SETS}
