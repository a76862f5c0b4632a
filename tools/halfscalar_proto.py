#!/usr/bin/env python3
"""halfscalar_proto.py — Python-integer prototype of the half-size-scalar verification equation the
verify kernel uses, checked against the golden fixtures' dalek verdicts.

dalek: accept iff enc([s]B - [k]A) == R_bytes, k = H(R||A||M) mod l, s < l.
Half-size form (after T. Pornin, "Optimized lattice basis reduction in dimension 2, and fast Schnorr and
EdDSA signature verification", 2020), made exactly cofactorless by reducing modulo N = 8l instead of l:
  find (c0, c1) with c0 = c1*k (mod 8l), c1 odd, |c0|, |c1| ~ sqrt(8l) ~ 2^127.5  (Euclid on (8l, k));
  every curve point P has [8l]P = 0, so [c1*k]A = [c0]A exactly, and [c1*s]B = [c1*s mod l]B;
  hence V = [c1]R + [c0]A - [t]B, t = c1*s mod l, equals [c1](R - R') exactly, R' = [s]B - [k]A;
  c1 odd and 0 < |c1| < l make [c1] injective on E = Z/8 x Z/l, so V = 0  <=>  R = R'.
  enc(R') == R_bytes  <=>  R_bytes canonical (y < p, not (x = 0 and sign)) and dec(R_bytes) == R'.
usage: python tools/halfscalar_proto.py [max_records_per_set]
"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
N8 = 8 * L
D = (-121665 * pow(121666, P - 2, P)) % P
SQRTM1 = pow(2, (P - 1) // 4, P)
BY = 4 * pow(5, P - 2, P) % P


def decompress(b: bytes):
    """dalek CompressedEdwardsY::decompress: y = LE255 mod p (no canonicity check), sign bit -> x parity,
    x = 0 with sign bit accepted. Returns extended (X, Y, Z, T) or None."""
    v = int.from_bytes(b, "little")
    sign = v >> 255
    y = (v & ((1 << 255) - 1)) % P
    u = (y * y - 1) % P
    w = (D * y * y + 1) % P
    x2 = u * pow(w, P - 2, P) % P
    x = pow(x2, (P + 3) // 8, P)
    if (x * x - x2) % P:
        x = x * SQRTM1 % P
    if (x * x - x2) % P:
        return None
    if (x & 1) != sign:
        x = (P - x) % P
    return (x, y, 1, x * y % P)


def canonical(b: bytes) -> bool:
    v = int.from_bytes(b, "little")
    y = v & ((1 << 255) - 1)
    if y >= P:
        return False
    pt = decompress(b)
    return not (pt is not None and pt[0] == 0 and (v >> 255))


def add(p1, p2):
    X1, Y1, Z1, T1 = p1
    X2, Y2, Z2, T2 = p2
    A = (Y1 - X1) * (Y2 - X2) % P
    B = (Y1 + X1) * (Y2 + X2) % P
    C = T1 * 2 * D * T2 % P
    DD = Z1 * 2 * Z2 % P
    E, F, G, H = B - A, DD - C, DD + C, B + A
    return (E * F % P, G * H % P, F * G % P, E * H % P)


def neg(p):
    return ((-p[0]) % P, p[1], p[2], (-p[3]) % P)


def mul(k, p):
    r = (0, 1, 1, 0)
    if k < 0:
        k, p = -k, neg(p)
    while k:
        if k & 1:
            r = add(r, p)
        p = add(p, p)
        k >>= 1
    return r


def is_identity(p):
    return p[0] % P == 0 and (p[1] - p[2]) % P == 0


B_PT = decompress(BY.to_bytes(32, "little"))


def lattice(k: int):
    """Euclid on (8l, k) stopped below sqrt(8l): consecutive remainders (r_i, t_i) with r_i = t_i k mod 8l.
    Returns the shortest candidate (c0, c1) with c1 odd among the last two rows and their sum/difference."""
    r0, t0, r1, t1 = N8, 0, k, 1
    while r1 * r1 >= N8:
        q = r0 // r1
        r0, t0, r1, t1 = r1, t1, r0 - q * r1, t0 - q * t1
    q = r0 // r1 if r1 else 0
    r2, t2 = (r0 - q * r1, t0 - q * t1) if r1 else (r0, t0)
    cands = [(r1, t1), (r2, t2), (r0, t0), (r1 + r2, t1 + t2), (r1 - r2, t1 - t2)]
    best = None
    for c0, c1 in cands:
        if c1 % 2 == 0:
            continue
        assert (c0 - c1 * k) % N8 == 0
        size = max(abs(c0), abs(c1)).bit_length()
        if best is None or size < best[0]:
            best = (size, c0, c1)
    return best


def verify_half(pk: bytes, sig: bytes, msg: bytes):
    Rb, Sb = sig[:32], sig[32:]
    s = int.from_bytes(Sb, "little")
    if s >= L:
        return False, None
    A = decompress(pk)
    if A is None:
        return False, None
    if not canonical(Rb):
        return False, None
    R = decompress(Rb)
    if R is None:
        return False, None
    k = int.from_bytes(hashlib.sha512(Rb + pk + msg).digest(), "little") % L
    size, c0, c1 = lattice(k)
    t = (c1 * s) % L
    V = add(add(mul(c1, R), mul(c0, A)), neg(mul(t, B_PT)))
    return is_identity(V), size


def main():
    import golden_io
    lim = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    worst, total, mism = 0, 0, 0
    for name in golden_io.SETS:
        g = golden_io.load(name)
        for i in range(min(g.n, lim)):
            ok, size = verify_half(g.pk[i].tobytes(), g.sig[i].tobytes(), g.message(i))
            total += 1
            if ok != bool(g.dalek[i]):
                mism += 1
                print("MISMATCH", name, i, ok, bool(g.dalek[i]), g.cls[i])
            if size:
                worst = max(worst, size)
        print(f"{name}: checked {min(g.n, lim)}")
    print(f"total {total} mismatches {mism} widest |c0|,|c1| {worst} bits")
    return 1 if mism else 0


if __name__ == "__main__":
    sys.exit(main())
