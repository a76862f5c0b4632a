#!/usr/bin/env python3
"""isa_loops.py — static instruction mix of a kernel in a hipcc -S listing, per loop body.

usage: python3 tools/isa_loops.py listing.s kernel_substring [--top N]

Finds backward branches (loops), and for each loop prints its line span, instruction count and the mix
by class (64-bit VALU = half rate on gfx950, 32-bit VALU, SALU, LDS, VMEM, scratch). Used to see where a
kernel's dynamic instruction count comes from (the ladder window loop, the fe_sqn loops of the two
exponentiations, SHA-512 rounds, ...)."""
import re
import sys
from collections import Counter

HALF = re.compile(r"^v_(mad_i64_i32|mad_u64_u32|ashrrev_i64|lshrrev_b64|lshlrev_b64|lshl_add_u64|add_co_u32|addc_co_u32|"
                  r"sub_co_u32|subb_co_u32|subrev_co_u32|mul_lo_u32|mul_hi_u32|mul_hi_i32|mul_u32_u24|mul_i32_i24|bfe_u32|"
                  r"bfe_i32|alignbit_b32|lshlrev_b32|lshrrev_b32|ashrrev_i32|lshl_add_u32|add3_u32|mov_b64|cndmask_b32|"
                  r"mad_u32_u24|lshl_or_b32|and_or_b32|or3_b32|xad_u32|mov_b64|add_nc_u64|ashr_i64)")


def classify(op):
    if op.startswith("scratch_") or op.startswith("buffer_store") and "off" in op:
        return "scratch"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu_half" if HALF.match(op) else "valu_full"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and name in l and l.rstrip().endswith(":") or
                 (l.split(":")[0].startswith("_Z") and name in l.split(":")[0]))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {}
    insts = []  # (line index in body, opcode)
    for i, l in enumerate(body):
        s = l.strip()
        m = re.match(r"^(\.LBB\d+_\d+):", s)
        if m:
            labels[m.group(1)] = i
            continue
        if not s or s.startswith((";", ".")):
            continue
        insts.append((i, s.split()[0]))
    total = Counter(classify(op) for _, op in insts)
    print(f"kernel lines {start}..{end}: {len(insts)} instructions: {dict(total)}")
    loops = []
    for i, op in insts:
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = body[i].split()[-1]
            if tgt in labels and labels[tgt] < i:
                loops.append((labels[tgt], i, tgt))
    for a, b, tgt in sorted(loops):
        ops = [op for j, op in insts if a <= j <= b]
        c = Counter(classify(op) for op in ops)
        cycles = 4 * c["valu_half"] + 2 * c["valu_full"]
        print(f"loop {tgt} body lines {a}..{b}: {len(ops)} insts, nominal VALU cycles {cycles}: {dict(c)}")
        if "--ops" in sys.argv:
            for op, k in Counter(ops).most_common(top):
                print(f"    {k:6d} {op}")


if __name__ == "__main__":
    main()
