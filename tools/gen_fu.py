#!/usr/bin/env python3
"""Generate at2-node_amd/csrc/at2v_fu_gen.h: GF(2^255-19) arithmetic with UNSIGNED limbs and the carry chained
through the MAD addend, plus the constants and the bound proof of the group law in at2v_gu.h.

Representation: 10 uint32 limbs, radix 2^25.5 (limb i holds bits [OFF[i], OFF[i] + W[i])), value = sum v_i 2^OFF[i]
(mod p). Every element is non-negative limb-wise; a subtraction a - b is computed as a + K - b with K a multiple of p
whose limbs dominate b's (constants FU_K*).

Product h = f*g: column k (k = 0..9; wrapped terms premultiplied by 19 in 32 bits, odd*odd terms doubled) is ONE
dependent chain of v_mad_u64_u32 whose first addend is the carry out of column k-1 (column 0: 0):
    h_k = c_{k-1} + sum_{i+j=k (mod 10)} f_i' g_j' ;  c_k = h_k >> W[k] ;  r_k = h_k & (2^W[k] - 1)
then the top carry wraps: t = r_0 + 19 c_9 ; r_0 = t mod 2^26 ; r_1 += t >> 26.
Per column that is one 64-bit shift and one AND: floor limbs need no rounding bias and the carry costs no separate
64-bit add, where the balanced signed form of at2v_fe_gen.h needs shift + add + AND + bias subtract
(profiles/r02b/ubench_fu*.txt: -9% per multiply, -20% per square, -8% per doubling before the formula changes).

Bounds are tracked per limb (odd limbs have twice the headroom of even ones under the x19 premultiplication, so the
subtraction constants put their excess into limb 9). The script checks:
  * every scaled 32-bit operand < 2^32 and every column (with its carry-in) < 2^64, for the declared input classes;
  * the group-law formulas of at2v_gu.h (mirrored below) only feed products with inputs inside those classes;
and derives the carried output class (limb 1 takes the wrap carry).
"""
import os
import re
import sys

P = 2**255 - 19
OFF = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]
W = [26, 25] * 5
U32 = 2**32 - 1
U64 = 2**64 - 1
D = (-121665 * pow(121666, P - 2, P)) % P
D2 = (2 * D) % P
SQRTM1 = pow(2, (P - 1) // 4, P)


def val(limbs):
    return sum(v << OFF[i] for i, v in enumerate(limbs))


def carried_limbs(x):
    x %= P
    return [(x >> OFF[i]) & ((1 << W[i]) - 1) for i in range(10)]


# ------------------------------------------------------------------------------------------------ products

def mul_terms():
    out = []
    for i in range(10):
        for j in range(10):
            a = 2 if (i % 2 == 1 and j % 2 == 1) else 1
            b = 1
            k = i + j
            if k >= 10:
                b = 19
                k -= 10
            out.append((k, i, a, j, b))
    return out


def sq_terms(double, fmax):
    """(k, i, a, j, b): product (a f_i)(b f_j); coefficient split so both scaled operands fit uint32"""
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
            best = None
            for a in (1, 2, 4, 8, 19, 38, 76):
                if c % a:
                    continue
                b = c // a
                if b not in (1, 2, 4, 8, 19, 38, 76):
                    continue
                if a * fmax[i] > U32 or b * fmax[j] > U32:
                    continue
                # prefer small powers of two on the lower-index operand and x19 on the higher one (the scaled
                # copies are then shared across columns: f_i*2, f_i*4 for low i, f_j*19 for high j)
                key = (0 if (a in (1, 2, 4) and b in (1, 2, 19)) else 1, (a != 1) + (b != 1), max(a, b))
                if best is None or key < best[0]:
                    best = (key, a, b)
            assert best, (i, j, c)
            out.append((k, i, best[1], j, best[2]))
    return out


def build_cols(terms):
    cols = [[] for _ in range(10)]
    for (k, i, a, j, b) in terms:
        cols[k].append((i, a, j, b))
    return cols


def prove(cols, fmax, gmax, name):
    """column and carry bounds; returns (worst column, c9 max, limb-1 spill)"""
    carry = 0
    worst = 0
    for k in range(10):
        s = carry
        for (i, a, j, b) in cols[k]:
            assert a * fmax[i] <= U32 and b * gmax[j] <= U32, (name, k, i, a, j, b)
            s += a * fmax[i] * b * gmax[j]
        assert s <= U64, (name, k, s.bit_length())
        worst = max(worst, s)
        carry = s >> W[k]
    c9 = carry
    t = ((1 << 26) - 1) + 19 * c9
    return worst, c9, t >> 26


# ------------------------------------------------------------------------------------------------ classes

def units(u, odd_u=None, l9=None, slack=1 << 16):
    """per-limb maxima: u units on even limbs, odd_u on odd limbs, l9 on limb 9 (plus `slack`)"""
    odd_u = u if odd_u is None else odd_u
    out = []
    for i in range(10):
        uu = u if i % 2 == 0 else odd_u
        if i == 9 and l9 is not None:
            uu = l9
        out.append(int(uu * (1 << W[i])) + slack)
    return out


# generated-function input classes (every use in the group-law model below is checked against them). The x19
# premultiplied operand g needs 19 g_j < 2^32: <= 3.36 units on even limbs, 6.7 on odd ones; f is bounded by the
# column sums only.
MUL_F = units(4.0, 4.5, 6.0)     # operand f of fu_mul
MUL_G = units(3.0, 4.5, 6.0)     # operand g of fu_mul (premultiplied by 19)
SQ_IN = MUL_G                    # operand of fu_sq / fu_sq2


def fmax_add(*xs):
    return [sum(x[i] for x in xs) for i in range(10)]


def kconst(dom):
    """multiple of p (limb form) whose limbs all dominate `dom` with the least excess on limbs 0..8: the excess of
    m p over `dom` goes greedily into the top limb first (odd limb 9 has the most headroom)"""
    best = None
    for m in range(1, 12):
        target = m * P
        rest = target - val(dom)
        if rest < 0:
            continue
        k = list(dom)
        for i in range(9, -1, -1):
            q = rest >> OFF[i]
            k[i] += q
            rest -= q << OFF[i]
        assert rest == 0 and val(k) == target and all(k[i] >= dom[i] for i in range(10)), (m, k)
        if any(v >= 2**32 for v in k):
            continue
        key = (max((k[i] - dom[i]) / (1 << W[i]) for i in range(9)), k[9])
        if best is None or key < best[0]:
            best = (key, k)
    assert best, "no constant"
    return best[1]


MCOLS = build_cols(mul_terms())


class Model:
    """the group-law formulas of at2v_gu.h on per-limb maxima: checks product inputs against the classes, and for
    the products emitted with the one-MAD wrap (`narrow`, the fu_*_n / *_wn / *_nn variants) that the top carry of
    that site's inputs stays below 2^32"""

    def __init__(self, carried):
        self.C = carried

    def mul(self, f, g, where, narrow=False):
        assert all(f[i] <= MUL_F[i] for i in range(10)), (where, "f", f)
        assert all(g[i] <= MUL_G[i] for i in range(10)), (where, "g", g)
        if narrow:
            assert prove(MCOLS, f, g, where)[1] < 2**32, where
        return self.C

    def sq(self, f, where, narrow=False, double=False):
        assert all(f[i] <= SQ_IN[i] for i in range(10)), (where, f)
        if narrow:
            assert prove(build_cols(sq_terms(double, SQ_IN)), f, f, where)[1] < 2**32, where
        return self.C


def pcarry_even(x):
    """gu_pcarry_even: even limbs carried into the next (odd) limb: even limbs < 2^26, odd limbs += x_even >> 26"""
    out = list(x)
    for i in (0, 2, 4, 6, 8):
        out[i + 1] += out[i] >> 26
        out[i] = (1 << 26) - 1
    return out


def check_group_law(C, K):
    """mirror of at2v_gu.h (keep in step); K = dict of the subtraction constants"""
    m = Model(C)
    add = fmax_add
    KC = K["C"]
    dom = lambda k, x: all(k[i] >= x[i] for i in range(10))
    # --- doubling p2 -> p1p1 (gu_p2_dbl): inputs carried.  x3 = N1/D1, y3 = N2/D2 with
    #     N1 = XX + YY + K - t0 (= -2XY), D1 = XX + K - YY (= X^2 - Y^2), N2 = XX + YY, D2 = ZZ2 + D1, even-carried
    X = Y = Z = C
    s = add(X, Y)
    XX = m.sq(X, "dbl XX", True); YY = m.sq(Y, "dbl YY", True)
    t0 = m.sq(s, "dbl (X+Y)^2", True); ZZ2 = m.sq(Z, "dbl 2Z^2", True, True)
    N2 = add(XX, YY)
    assert dom(KC, t0) and dom(KC, YY)
    N1 = add(N2, KC)
    D1 = add(XX, KC)
    D2 = pcarry_even(add(ZZ2, D1))
    dbl = (N1, N2, D1, D2)
    # --- addition p3 + cached -> p1p1 (gu_add); cached entries as stored by gu_p3_to_cached
    ypx, ymx, z2, t2d = add(C, C), add(C, KC), add(C, C), C
    assert dom(KC, C)
    ym = add(C, KC); yp = add(C, C)
    for (pp, mm) in ((ypx, ymx), (ymx, ypx)):    # a negative digit swaps YpX / YmX and negates T2d
        m.mul(ym, mm, "add A"); m.mul(yp, pp, "add B", True)
    tneg = KC                                        # K_C - T2d <= K_C
    m.mul(C, t2d, "add C", True); m.mul(C, tneg, "add C-", True); m.mul(C, z2, "add D", True)
    Ea = add(C, KC); Ha = add(C, C); Ga = add(C, C); Fa = add(C, KC)
    addr = (Ea, Ha, Ga, Fa)
    # --- mixed addition with an affine Niels entry (gu_madd): entries carried; negation as for cached
    m.mul(ym, C, "madd A", True); m.mul(yp, C, "madd B", True); m.mul(C, C, "madd C", True)
    m.mul(C, KC, "madd C-", True)
    d2 = add(C, C)
    Gm = add(d2, C); Fm = pcarry_even(add(d2, KC))
    madd = (Ea, Ha, Gm, Fm)
    # p1p1 (X, Y, Z, T) -> p2 / p3 (gu_p1p1_to_p2 / _p3): X3 = X T (wide), Y3 = Y Z or Z Y (AT2V_GU_SHARE; narrow),
    # Z3 = Z T (wide), T3 = X Y (wide)
    for (x, y, z, t), nm in ((dbl, "dbl"), (addr, "add"), (madd, "madd")):
        m.mul(x, t, nm + " X"); m.mul(y, z, nm + " Y", True); m.mul(z, y, nm + " Y'", True)
        m.mul(z, t, nm + " Z"); m.mul(x, y, nm + " T")
    # --- cached form of a p3 point: YpX = Y + X, YmX = Y + K_C - X, Z2 = 2Z, T2d = T * 2d
    m.mul(C, C, "T2d", True)
    # --- decode: u = y^2 + (p - 1), v = d y^2 + 1; checks on v x^2 -+ u
    u = add(C, K["PM1"])
    v = add(C, [1] + [0] * 9)
    m.sq(v, "decode v^2"); m.mul(C, v, "decode v^3"); m.mul(C, u, "decode u v^7")
    m.mul(u, C, "decode u sqrt(-1)")
    m.mul(C, v, "decode v x^2")
    return True


def emit_fn(name, colsets, is_mul, cheap_wrap):
    """fu_mul / fu_sq (one column set) or the 2-way variants (two independent products, e.g. a square and a
    doubled square; each column's asm block alternates the MADs of both, so the two dependent chains interleave)"""
    nway = len(colsets)
    ps = [""] if nway == 1 else ["0", "1"]
    args = []
    for q in ps:
        args.append(f"fu& h{q}")
        args.append(f"const fu& f{q}")
        if is_mul:
            args.append(f"const fu& g{q}")
    out = [f"AT2V_HD AT2V_INLINE void {name}({', '.join(args)}) {{"]
    gsrc = "g" if is_mul else "f"
    for q in ps:
        out.append("  " + " ".join(f"const uint32_t f{q}_{i} = f{q}.v[{i}];" for i in range(10)))
        if is_mul:
            out.append("  " + " ".join(f"const uint32_t g{q}_{i} = g{q}.v[{i}];" for i in range(10)))
    needs = []
    for cols in colsets:
        need = set()
        for k in range(10):
            for (i, a, j, b) in cols[k]:
                need.add(("f", i, a))
                need.add((gsrc, j, b))
        needs.append(need)

    def nm(q, src, i, s):
        return f"{src}{q}_{i}" + (f"_{s}" if s != 1 else "")
    for q, need in zip(ps, needs):
        for (src, i, s) in sorted(need):
            if s == 1:
                continue
            if s in (2, 4, 8) and (s == 2 or (src, i, s // 2) in need):
                out.append(f"  const uint32_t {nm(q, src, i, s)} = AT2V_UX2({nm(q, src, i, s // 2)});")
            else:
                out.append(f"  const uint32_t {nm(q, src, i, s)} = AT2V_USC({s}u, {src}{q}_{i});")
    out.append("  " + " ".join(f"uint64_t c{q} = 0;" for q in ps))
    if nway == 1:
        out += emit_fused(colsets[0], gsrc, nm)
        out.append("#else")
    for k in range(10):
        cs = [cols[k] for cols in colsets]
        assert all(len(c) == len(cs[0]) for c in cs)
        out.append("#if AT2V_FU_ASM")
        out.append("  {")
        out.append("    " + " ".join(f"uint64_t hk{q};" for q in ps))
        ins = []
        idx = {}

        def reg(e):
            if e not in idx:
                idx[e] = len(ins)
                ins.append(e)
            return idx[e]
        lines = []
        for t in range(len(cs[0])):
            for qi, q in enumerate(ps):
                (i, a, j, b) = cs[qi][t]
                ra, rb = reg(nm(q, "f", i, a)), reg(nm(q, gsrc, j, b))
                if t == 0:
                    addend = "0" if k == 0 else f"CARRY{qi}"
                    lines.append(f"v_mad_u64_u32 %{qi}, vcc, IN{ra}, IN{rb}, {addend}")
                else:
                    lines.append(f"v_mad_u64_u32 %{qi}, vcc, IN{ra}, IN{rb}, %{qi}")
        nout = len(ps)
        if k > 0:
            for q in ps:
                reg(f"c{q}")
        fixed = []
        for l in lines:
            l = re.sub(r"IN(\d+)", lambda mm: f"%{int(mm.group(1)) + nout}", l)
            l = re.sub(r"CARRY(\d)", lambda mm: f"%{idx['c' + ps[int(mm.group(1))]] + nout}", l)
            fixed.append(l)
        outs = ", ".join(f'"=&v"(hk{q})' for q in ps)
        inl = ", ".join(f'"v"({e})' for e in ins)
        out.append('    asm("' + "\\n\\t".join(fixed) + '"')
        out.append('        : ' + outs)
        out.append('        : ' + inl)
        out.append('        : "vcc");')
        for q in ps:
            out.append(f"    c{q} = hk{q} >> {W[k]};")
            out.append(f"    h{q}.v[{k}] = (uint32_t)hk{q} & 0x{(1 << W[k]) - 1:x}u;")
        out.append("  }")
        out.append("#else")
        for q, col in zip(ps, cs):
            expr = f"c{q}"
            for (i, a, j, b) in col:
                expr = f"AT2V_UMAD({nm(q, 'f', i, a)}, {nm(q, gsrc, j, b)}, {expr})"
            out.append(f"  {{ const uint64_t hk = {expr}; c{q} = hk >> {W[k]}; h{q}.v[{k}] = (uint32_t)hk & 0x{(1 << W[k]) - 1:x}u; }}")
        out.append("#endif")
    if nway == 1:
        out.append("#endif  // AT2V_FU_FUSED")
    # wrap: t = r0 + 19 c9
    for q, cw in zip(ps, cheap_wrap):
        out.append("  {")
        if cw:  # c9 < 2^32 (proven): one 32x32+64 MAD
            out.append(f"    const uint64_t t = AT2V_UMAD(AT2V_UNARROW(c{q}), 19u, h{q}.v[0]);")
        else:
            out.append(f"    const uint64_t t = (uint64_t)h{q}.v[0] + 19u * c{q};")
        out.append(f"    h{q}.v[0] = (uint32_t)t & 0x3ffffffu;")
        out.append(f"    h{q}.v[1] += (uint32_t)(t >> 26);")
        out.append("  }")
    out.append("}")
    return "\n".join(out)


def emit_fused(cols, gsrc, nm):
    """AT2V_FU_FUSED: the whole product as ONE asm statement. The column accumulator lives in the clobbered pair
    v[254:255]: column k's MAD chain ends there, v_and_b32 takes limb k out of its low half (into an output operand) and
    v_lshrrev_b64 shifts the pair in place into the carry that starts column k+1's chain; column 9's carry goes to an
    output operand for the wrap. hipcc pads one wait state after every inline asm whose output a VALU reads next (it
    cannot see inside the string); per column that was one s_nop per product column, here it is one per product. No
    VALU->VALU pair inside the string needs a wait state on gfx950 (no DPP, SDWA, trans or readlane consumers)."""
    out = ["#if AT2V_FU_ASM && AT2V_FU_FUSED", "  {"]
    ins, idx = [], {}

    def reg(e):
        if e not in idx:
            idx[e] = len(ins)
            ins.append(e)
        return idx[e]
    lines = []
    nout = 11  # r0..r9, c9
    for k in range(10):
        for t, (i, a, j, b) in enumerate(cols[k]):
            ra, rb = reg(nm("", "f", i, a)), reg(nm("", gsrc, j, b))
            addend = ("0" if k == 0 else "v[254:255]") if t == 0 else "v[254:255]"
            lines.append(f"v_mad_u64_u32 v[254:255], vcc, %{ra + nout}, %{rb + nout}, {addend}")
        lines.append(f"v_and_b32 %{k}, 0x{(1 << W[k]) - 1:x}, v254")
        if k < 9:
            lines.append(f"v_lshrrev_b64 v[254:255], {W[k]}, v[254:255]")
        else:
            lines.append(f"v_lshrrev_b64 %10, {W[k]}, v[254:255]")
    out.append("    uint32_t r0, r1, r2, r3, r4, r5, r6, r7, r8, r9;")
    out.append('    asm("' + "\\n\\t".join(lines) + '"')
    out.append('        : ' + ", ".join(f'"=&v"(r{k})' for k in range(10)) + ', "=&v"(c)')
    out.append('        : ' + ", ".join(f'"v"({e})' for e in ins))
    out.append('        : "vcc", "v254", "v255");')
    out.append("    h.v[0] = r0; h.v[1] = r1; h.v[2] = r2; h.v[3] = r3; h.v[4] = r4;")
    out.append("    h.v[5] = r5; h.v[6] = r6; h.v[7] = r7; h.v[8] = r8; h.v[9] = r9;")
    out.append("  }")
    return out


def lit(limbs):
    return "{{" + ", ".join(f"0x{v:x}u" for v in limbs) + "}}"


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(__file__), "..", "at2-node_amd", "csrc", "at2v_fu_gen.h")
    mcols = build_cols(mul_terms())
    scols = build_cols(sq_terms(False, SQ_IN))
    s2cols = build_cols(sq_terms(True, SQ_IN))
    wm, c9m, spm = prove(mcols, MUL_F, MUL_G, "mul")
    ws, c9s, sps = prove(scols, SQ_IN, SQ_IN, "sq")
    ws2, c9s2, sps2 = prove(s2cols, SQ_IN, SQ_IN, "sq2")
    spill = max(spm, sps, sps2)
    # carried output class; it must lie inside every input class
    C = [(1 << W[i]) - 1 for i in range(10)]
    C[1] += spill
    assert all(C[i] <= MUL_G[i] and C[i] <= SQ_IN[i] for i in range(10))
    K = {"C": kconst(C), "2C": kconst(fmax_add(C, C))}
    pm1 = carried_limbs(P - 1)
    K["PM1"] = pm1
    assert val(pm1) == P - 1
    check_group_law(C, K)

    hdr = []
    hdr.append("// GENERATED by tools/gen_fu.py -- do not edit. Regenerate: python3 tools/gen_fu.py")
    hdr.append("// Bound proof (per limb, tools/gen_fu.py): fu_mul f within 4 carried units on even limbs, 4.5 on odd ones")
    hdr.append("// (limb 9: 6); fu_mul g and fu_sq operands within 3 on even limbs (x19 premultiplied); scaled operands < 2^32; columns with carry-in: mul 2^{wm.bit_length()}, sq 2^{ws.bit_length()}, "
               f"sq2 2^{ws2.bit_length()} (< 2^64);")
    hdr.append(f"// top carry mul 2^{c9m.bit_length()}, sq 2^{c9s.bit_length()}, sq2 2^{c9s2.bit_length()}; "
               f"carried output: limb i < 2^W[i], limb 1 <= 2^25 - 1 + {spill}.")
    hdr.append("// The group law of at2v_gu.h is checked against these classes (check_group_law).")
    hdr.append("#pragma once")
    hdr.append('#include "at2v_fu_base.h"')
    hdr.append("namespace at2v {")
    hdr.append(f"constexpr uint32_t kFuLimb1Spill = {spill}u;")
    hdr.append(f"// mul: {sum(len(c) for c in mcols)} v_mad_u64_u32; sq: {sum(len(c) for c in scols)}; "
               f"sq2: {sum(len(c) for c in s2cols)}")
    # variants for carried inputs (exponentiation chains): the top carry stays below 2^32, so the wrap is one MAD
    sccols = build_cols(sq_terms(False, C))
    wsc, c9sc, spsc = prove(sccols, C, C, "sqc")
    wmc, c9mc, spmc = prove(mcols, C, C, "mulc")
    assert c9sc < 2**32 and c9mc < 2**32 and max(spsc, spmc) <= spill
    cw_m, cw_s, cw_s2 = c9m < 2**32, c9s < 2**32, c9s2 < 2**32
    hdr.append(emit_fn("fu_mul", [mcols], True, [cw_m]))
    hdr.append(emit_fn("fu_sq", [scols], False, [cw_s]))
    hdr.append(emit_fn("fu_sq2", [s2cols], False, [cw_s2]))
    hdr.append(emit_fn("fu_mul_x2", [mcols, mcols], True, [cw_m, cw_m]))
    hdr.append(emit_fn("fu_sq_x2", [scols, scols], False, [cw_s, cw_s]))
    hdr.append("// h0 = f0^2, h1 = 2 f1^2")
    hdr.append(emit_fn("fu_sq_sq2", [scols, s2cols], False, [cw_s, cw_s2]))
    hdr.append(f"// carried inputs only (top carry < 2^{max(c9sc, c9mc).bit_length()}): exponentiation chains")
    hdr.append(emit_fn("fu_mulc", [mcols], True, [True]))
    hdr.append(emit_fn("fu_sqc", [sccols], False, [True]))
    hdr.append(emit_fn("fu_mulc_x2", [mcols, mcols], True, [True, True]))
    hdr.append("// one-MAD wrap at the sites check_group_law proves narrow (n), full wrap where it does not (w)")
    hdr.append(emit_fn("fu_mul_n", [mcols], True, [True]))
    hdr.append(emit_fn("fu_mul_wn", [mcols, mcols], True, [cw_m, True]))
    hdr.append(emit_fn("fu_mul_nn", [mcols, mcols], True, [True, True]))
    hdr.append(emit_fn("fu_sq_sq2_n", [scols, s2cols], False, [True, True]))
    hdr.append(emit_fn("fu_sqc_x2", [sccols, sccols], False, [True, True]))
    hdr.append("// subtraction constants (multiples of p): FU_KC dominates a carried element, FU_K2C a sum of two carried")
    hdr.append(f"AT2V_FU_CONST fu FU_KC = {lit(K['C'])};")
    hdr.append(f"AT2V_FU_CONST fu FU_K2C = {lit(K['2C'])};")
    hdr.append(f"AT2V_FU_CONST fu FU_PM1 = {lit(K['PM1'])};  // p - 1")
    hdr.append(f"AT2V_FU_CONST fu FU_D = {lit(carried_limbs(D))};")
    hdr.append(f"AT2V_FU_CONST fu FU_D2 = {lit(carried_limbs(D2))};")
    hdr.append(f"AT2V_FU_CONST fu FU_SQRTM1 = {lit(carried_limbs(SQRTM1))};")
    hdr.append("}  // namespace at2v")
    with open(out_path, "w") as fp:
        fp.write("\n".join(hdr) + "\n")
    print(f"wrote {out_path}: mul 2^{wm.bit_length()} sq 2^{ws.bit_length()} sq2 2^{ws2.bit_length()}, "
          f"c9 mul 2^{c9m.bit_length()} sq 2^{c9s.bit_length()} sq2 2^{c9s2.bit_length()}, limb-1 spill {spill}")
    for nm_, k in K.items():
        print(f"  K_{nm_} units {[round(k[i] / (1 << W[i]), 3) for i in range(10)]}")


if __name__ == "__main__":
    main()
