"""CPU: the per-lane lattice reduction of the half-size verification equation (at2v_lattice.h, host build)
against Python integers: c0 = c1*k (mod 8l), c1 odd, sizes close to the Euclid/Gauss optimum, and
t = c1*s mod l — for random k and for the corner cases (k = 0, 1, small, l - 1, powers of two, k with a
huge first quotient)."""
import os
import random
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

L = 2**252 + 27742317777372353535851937790883648493
N8 = 8 * L


@pytest.fixture(scope="module")
def exe():
    out = os.path.join(ROOT, "tests", "host", "lattice_host")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "at2-node_amd", "csrc"),
                    os.path.join(ROOT, "tests", "host", "lattice_host.cpp"), "-o", out], check=True)
    return out


def run(exe, pairs):
    inp = "".join(f"{k:064x} {s:064x}\n" for k, s in pairs)
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True, timeout=300).stdout.split("\n")
    res = []
    for line in out:
        if not line.strip():
            continue
        c0, c1, neg, bits, t = line.split()
        res.append((int(c0, 16), int(c1, 16) * (-1 if int(neg) else 1), int(bits), int(t, 16)))
    return res


def check(pairs, res, slack):
    from halfscalar_proto import lattice
    worst = 0
    for (k, s), (c0, c1, bits, t) in zip(pairs, res):
        assert c0 >= 0 and c1 % 2 == 1, (k, c0, c1)
        assert (c0 - c1 * k) % N8 == 0, k
        assert abs(c1) < 5 * 2**252 and c0 < 5 * 2**252  # top radix-16 digit cannot carry out
        assert bits == max(c0.bit_length(), abs(c1).bit_length())
        assert t == (c1 * s) % L
        ref_bits = lattice(k)[0]
        assert bits <= ref_bits + slack, (k, bits, ref_bits)
        worst = max(worst, bits)
    return worst


def test_random_k(exe):
    rng = random.Random(7)
    pairs = [(rng.randrange(L), rng.randrange(L)) for _ in range(20000)]
    res = run(exe, pairs)
    assert len(res) == len(pairs)
    worst = check(pairs, res, slack=1)
    assert worst <= 140


def test_corner_k(exe):
    rng = random.Random(8)
    ks = [0, 1, 2, 3, 7, 8, 9, 16, L - 1, L - 2, (L - 1) // 2, 2**126, 2**127, 2**128, 2**200, 2**252 - 1,
          (1 << 128) + 1, 5, 12345678901234567890, N8 // 7 % L, N8 // 2**40 % L, N8 // 2**100 % L]
    ks += [rng.randrange(2**64) for _ in range(50)]               # tiny k: one huge first quotient
    ks += [L - rng.randrange(2**64) for _ in range(50)]
    ks += [(N8 // rng.randrange(2, 2**60)) % L for _ in range(100)]  # huge quotients deeper in the run
    pairs = [(k, rng.randrange(L)) for k in ks]
    res = run(exe, pairs)
    worst = check(pairs, res, slack=4)
    # the kernel's 64 radix-16 windows need bits <= 255 (verify_half fails a lane closed above that): the
    # largest scalars come from tiny/huge first quotients, where the odd-c1 row is (k, 1) itself
    assert worst <= 253, worst


def test_bits_bound_near_lehmer_threshold(exe):
    """k whose Euclid remainders straddle the stopping threshold ceil(sqrt(8l)) at every depth the
    Lehmer rounds reach: the chosen vector must stay short (no candidate built from the huge row)"""
    import math
    rng = random.Random(9)
    thr = math.isqrt(N8) + 1
    ks = []
    for _ in range(300):  # k = 8l / (thr + small) lands the first remainder next to the threshold
        d = thr + rng.randrange(-2**20, 2**20)
        ks.append((N8 // d) % L)
        ks.append((N8 // d + rng.randrange(1, 2**16)) % L)
    pairs = [(k, rng.randrange(L)) for k in ks]
    res = run(exe, pairs)
    worst = check(pairs, res, slack=4)
    assert worst <= 253, worst
