#!/usr/bin/env python3
"""Generate at2-node_amd/csrc/at2v_fe_gen.h: GF(2^255-19) multiply/square kernels and constant tables.

Representation: 10 signed int32 limbs, radix 2^25.5 (limb i holds bits
[ceil(25.5 i), ceil(25.5 (i+1))) - 26 bits for even i, 25 for odd i). "Carried" limbs are balanced:
|v_i| <= 2^(w_i - 1) (+ a small spill on limb 1). Field mul/square accumulate 10 column sums
with v_mad_i64_i32 (32x32+64 -> 64, one half-rate VALU op on gfx950, see
profiles/r01_ubench_valu.txt), with 19*g pre-multiplied in 32 bits for the wrapped terms
(2^255 = 19 mod p), and each column accumulator starts at its rounding bias 2^(w-1) so a
floor carry chain yields balanced limbs.

This script also proves the bounds: every scaled 32-bit operand fits int32 and every 64-bit
column sum fits int64, for inputs that are sums/differences of up to 3 carried elements.

The B table (fixed base) is computed here with Python integers, independently of oracle/.
"""
import os
import sys

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
D2 = (2 * D) % P
SQRTM1 = pow(2, (P - 1) // 4, P)

OFF = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]
W = [26, 25] * 5

# ----------------------------------------------------------------- limbs


def to_limbs(x):
    """balanced signed limbs of x mod p"""
    x %= P
    v = [(x >> OFF[i]) & ((1 << W[i]) - 1) for i in range(10)]
    for _ in range(3):
        for i in range(10):
            half = 1 << (W[i] - 1)
            c = (v[i] + half) >> W[i]
            v[i] -= c << W[i]
            if i < 9:
                v[i + 1] += c
            else:
                v[0] += 19 * c
    assert sum(v[i] << OFF[i] for i in range(10)) % P == x
    for i in range(10):
        assert abs(v[i]) <= (1 << (W[i] - 1)) + 19, (i, v[i])
    return v


# ------------------------------------------------------------- curve (ints)
def inv(x):
    return pow(x, P - 2, P)


def recover_x(y, sign):
    u = (y * y - 1) % P
    v = (D * y * y + 1) % P
    x2 = u * inv(v) % P
    x = pow(x2, (P + 3) // 8, P)
    if (x * x - x2) % P != 0:
        x = x * SQRTM1 % P
    assert (x * x - x2) % P == 0
    if (x & 1) != sign:
        x = P - x
    return x % P


BY = 4 * inv(5) % P
BX = recover_x(BY, 0)


def ed_add(p1, p2):
    (x1, y1), (x2, y2) = p1, p2
    t = D * x1 * x2 * y1 * y2 % P
    x3 = (x1 * y2 + x2 * y1) * inv(1 + t) % P
    y3 = (y1 * y2 + x1 * x2) * inv(1 - t) % P
    return (x3, y3)


def niels(pt):
    x, y = pt
    return [(y + x) % P, (y - x) % P, 2 * D * x * y % P]


# ------------------------------------------------------- mul/sq generation
MAX32 = 2**31 - 1
MAX64 = 2**63 - 1


def carried_bound(i):
    # balanced limb after carry chain (+ spill on limbs 1 and 5 from the second carries into them)
    return (1 << (W[i] - 1)) + (1 << 16 if i in (1, 5) else 0) + (19 if i == 0 else 0)


def input_bound(i, terms=3):
    return terms * carried_bound(i)


def mul_terms():
    """(k, i, j, coeff) for h = f*g"""
    out = []
    for i in range(10):
        for j in range(10):
            c = 2 if (i % 2 == 1 and j % 2 == 1) else 1
            k = i + j
            if k >= 10:
                c *= 19
                k -= 10
            out.append((k, i, j, c))
    return out


def sq_terms(double=False):
    """(k, i, j, coeff) for h = f^2 (i <= j), optionally 2 f^2"""
    out = []
    for i in range(10):
        for j in range(i, 10):
            c = (1 if i == j else 2) * (2 if (i % 2 == 1 and j % 2 == 1) else 1)
            k = i + j
            if k >= 10:
                c *= 19
                k -= 10
            if double:
                c *= 2
            out.append((k, i, j, c))
    return out


def split_coeff(c, i, j, sq):
    """choose scalings (a on operand i, b on operand j) with a*b == c and both scaled values in int32"""
    cands = []
    for a in (1, 2, 4, 19, 38, 76):
        if c % a:
            continue
        b = c // a
        if b not in (1, 2, 4, 19, 38, 76):
            continue
        fa = a * input_bound(i)
        fb = b * input_bound(j)
        if fa <= MAX32 and fb <= MAX32:
            cands.append((max(a, b), a, b))
    assert cands, (c, i, j)
    cands.sort()
    return cands[0][1], cands[0][2]


def gen_mul():
    lines = []
    terms = mul_terms()
    # scalings on g only (f scaled by 2 for odd-odd)
    need = set()
    cols = [[] for _ in range(10)]
    for k, i, j, c in terms:
        a = 2 if (i % 2 == 1 and j % 2 == 1) else 1
        b = c // a
        assert a * b == c
        assert a * input_bound(i) <= MAX32 and b * input_bound(j) <= MAX32, (i, j, a, b)
        need.add(("f", i, a))
        need.add(("g", j, b))
        cols[k].append((f"f{i}" + (f"_{a}" if a != 1 else ""), f"g{j}" + (f"_{b}" if b != 1 else ""), a, b, i, j))
    return cols, need


def gen_sq(double):
    cols = [[] for _ in range(10)]
    need = set()
    for k, i, j, c in sq_terms(double):
        a, b = split_coeff(c, i, j, True)
        need.add(("f", i, a))
        need.add(("f", j, b))
        cols[k].append((f"f{i}" + (f"_{a}" if a != 1 else ""), f"f{j}" + (f"_{b}" if b != 1 else ""), a, b, i, j))
    return cols, need


def check_cols(cols, name):
    worst = 0
    for k, col in enumerate(cols):
        s = 1 << (W[k] - 1)  # bias
        for _, _, a, b, i, j in col:
            s += a * input_bound(i) * b * input_bound(j)
        worst = max(worst, s)
        assert s < MAX64 - (1 << 40), (name, k, s.bit_length())
    return worst


def emit_block_asm(cols):
    """device variant: all MADs of one multiply/square in ONE asm statement, column-interleaved
    (step t issues the t-th MAD of every column, so dependent MADs are <= 10 instructions apart),
    with the rounding bias as the SGPR addend of step 0. One hazard pad per field op instead of one
    per MAD; LLVM cannot re-associate the bias out of the chains. Returns C++ lines defining h0..h9."""
    out = []
    nsteps = max(len(c) for c in cols)
    out.append("  int64_t h0, h1, h2, h3, h4, h5, h6, h7, h8, h9;")
    ins = []
    idx = {}

    def opnd(expr, cons):
        key = (expr, cons)
        if key not in idx:
            idx[key] = len(ins)
            ins.append(key)
        return idx[key]
    lines = []
    for t in range(nsteps):
        for k in range(10):
            if len(cols[k]) <= t:
                continue
            fa, gb = cols[k][len(cols[k]) - 1 - t][0], cols[k][len(cols[k]) - 1 - t][1]
            ia, ib = opnd(fa, "v"), opnd(gb, "v")
            if t == 0:
                ic = opnd(f"(int64_t)AT2V_BIAS{W[k]}", "s")
                lines.append(f"v_mad_i64_i32 %{k}, vcc, %{10 + ia}, %{10 + ib}, %{10 + ic}")
            else:
                lines.append(f"v_mad_i64_i32 %{k}, vcc, %{10 + ia}, %{10 + ib}, %{k}")
    outs = ", ".join(f'"=&v"(h{k})' for k in range(10))
    inl = ", ".join(f'"{c}"({e})' for e, c in ins)
    out.append('  asm("' + "\\n\\t".join(lines) + '"')
    out.append('      : ' + outs)
    out.append('      : ' + inl)
    out.append('      : "vcc");')
    return out


def emit_fn(name, cols, need, sig, src_g):
    out = []
    out.append(f"AT2V_HD AT2V_INLINE void {name}{sig} {{")
    out.append("  " + " ".join(f"const int32_t f{i} = f.v[{i}];" for i in range(10)))
    if src_g:
        out.append("  " + " ".join(f"const int32_t g{i} = g.v[{i}];" for i in range(10)))
    for (op, idx, s) in sorted(need):
        if s == 1:
            continue
        if s == 2:
            out.append(f"  const int32_t {op}{idx}_2 = AT2V_X2({op}{idx});")
        elif s == 4 and (op, idx, 2) in need:
            out.append(f"  const int32_t {op}{idx}_4 = AT2V_X2({op}{idx}_2);")
        else:
            out.append(f"  const int32_t {op}{idx}_{s} = {s} * {op}{idx};")
    out.append("#if AT2V_FE_ASM_BLOCKS")
    out += emit_block_asm(cols)
    out.append("#else")
    for k in range(10):
        expr = f"(int64_t)AT2V_BIAS{W[k]}"
        for fa, gb, *_ in cols[k]:
            expr = f"AT2V_MAD({fa}, {gb}, {expr})"
        out.append(f"  int64_t h{k} = {expr};")
    out.append("#endif")
    out.append("  fe_carry_wide(h, h0, h1, h2, h3, h4, h5, h6, h7, h8, h9);")
    out.append("}")
    return "\n".join(out)


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(__file__), "..", "at2-node_amd", "csrc", "at2v_fe_gen.h")
    mcols, mneed = gen_mul()
    scols, sneed = gen_sq(False)
    s2cols, s2need = gen_sq(True)
    wm = check_cols(mcols, "mul")
    ws = check_cols(scols, "sq")
    ws2 = check_cols(s2cols, "sq2")

    hdr = []
    hdr.append("// GENERATED by tools/gen_fe.py -- do not edit. Regenerate: python3 tools/gen_fe.py")
    hdr.append(f"// Bound proof (inputs = sums/differences of <= 3 carried elements): worst |column| "
               f"mul 2^{wm.bit_length()}, sq 2^{ws.bit_length()}, sq2 2^{ws2.bit_length()} (< 2^63); "
               f"every scaled int32 operand < 2^31.")
    hdr.append("#pragma once")
    hdr.append('#include "at2v_fe_base.h"')
    hdr.append("namespace at2v {")
    hdr.append(f"// mul: {sum(len(c) for c in mcols)} v_mad_i64_i32; sq: {sum(len(c) for c in scols)}; "
               f"sq2: {sum(len(c) for c in s2cols)}")
    hdr.append(emit_fn("fe_mul", mcols, mneed, "(fe& h, const fe& f, const fe& g)", True))
    hdr.append(emit_fn("fe_sq", scols, sneed, "(fe& h, const fe& f)", False))
    hdr.append(emit_fn("fe_sq2", s2cols, s2need, "(fe& h, const fe& f)", False))

    def fe_lit(x):
        return "{{" + ", ".join(str(v) for v in to_limbs(x)) + "}}"

    hdr.append(f"AT2V_CONST_FE FE_D = {fe_lit(D)};")
    hdr.append(f"AT2V_CONST_FE FE_D2 = {fe_lit(D2)};")
    hdr.append(f"AT2V_CONST_FE FE_SQRTM1 = {fe_lit(SQRTM1)};")
    hdr.append(f"AT2V_CONST_FE FE_BY = {fe_lit(BY)};")
    hdr.append(f"AT2V_CONST_FE FE_BX = {fe_lit(BX)};")
    # fixed-base table: [j]B, j = 0..128, affine Niels (y+x, y-x, 2dxy), 32 int32 per entry (2 pad)
    pts = [(0, 1)]
    acc = (0, 1)
    for j in range(1, 129):
        acc = ed_add(acc, (BX, BY))
        pts.append(acc)
    hdr.append("// [j]B for j = 0..128 as affine Niels (y+x, y-x, 2d*x*y), balanced limbs, 32 words/entry")
    hdr.append("#define AT2V_BTAB_ENTRIES 129")
    hdr.append("#define AT2V_BTAB_WORDS 32")
    rows = []
    for pt in pts:
        limbs = []
        for x in niels(pt):
            limbs += to_limbs(x)
        limbs += [0, 0]
        rows.append("  " + ", ".join(str(v) for v in limbs))
    hdr.append("AT2V_CONST_ARR int32_t AT2V_BTAB[AT2V_BTAB_ENTRIES * AT2V_BTAB_WORDS] = {\n" + ",\n".join(rows) + "};")
    # y-coordinates of the order-8 points (libsodium 1.0.18 blocklist, policy LIBSODIUM_1_0_18):
    # 2P has y = 0  <=>  x^2 = -y^2  =>  d y^4 + 2 y^2 - 1 = 0  =>  y^2 = (-1 +- sqrt(1 + d)) / d
    def sqrt_mod(a):
        a %= P
        r = pow(a, (P + 3) // 8, P)
        if (r * r - a) % P:
            r = r * SQRTM1 % P
        return r if (r * r - a) % P == 0 else None
    s1d = sqrt_mod(1 + D)
    ys = []
    for sg in (1, -1):
        y2 = (-1 + sg * s1d) * inv(D) % P
        y = sqrt_mod(y2)
        if y is not None:
            ys += [y % P, (P - y) % P]
    ys = sorted(set(ys))
    assert len(ys) == 2, ys
    for y in ys:  # check order exactly 8
        pt = (recover_x(y, 0), y)
        q = pt
        for _ in range(2):
            q = ed_add(q, q)
        assert q != (0, 1)
        q = ed_add(q, q)
        assert q == (0, 1)
    def words(x):
        return "{" + ", ".join(hex((x >> (32 * i)) & 0xffffffff) + "u" for i in range(8)) + "}"
    blk = [0, 1, ys[0], ys[1], P - 1, P, P + 1]
    hdr.append("// libsodium 1.0.18 small-order blocklist (y encodings, sign bit masked): 0, 1, y8a, y8b, p-1, p, p+1")
    hdr.append("AT2V_CONST_ARR uint32_t AT2V_SMALL_ORDER_Y[7][8] = {" + ", ".join(words(x) for x in blk) + "};")
    hdr.append("}  // namespace at2v")
    with open(out_path, "w") as fp:
        fp.write("\n".join(hdr) + "\n")
    print(f"wrote {out_path}: mul worst 2^{wm.bit_length()} sq 2^{ws.bit_length()} sq2 2^{ws2.bit_length()}")


if __name__ == "__main__":
    main()
