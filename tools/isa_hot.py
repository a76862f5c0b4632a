#!/usr/bin/env python3
"""isa_hot.py — the largest loops of a kernel in a hipcc -S listing with their MAD / scratch / s_nop / LDS counts.
usage: python3 tools/isa_hot.py listing.s kernel_substring [N]"""
import collections
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    lines = open(path).read().split("\n")
    st = next(i for i, l in enumerate(lines) if l.startswith("_Z") and name in l.split(":")[0])
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    b = lines[st:en]
    labels = {}
    for i, l in enumerate(b):
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, l in enumerate(b):
        s = l.strip()
        if s.startswith(("s_cbranch", "s_branch")):
            t = s.split()[-1]
            if t in labels and labels[t] < i:
                loops.append((labels[t], i, t))

    def ops(a, z):
        return [l.split()[0] for l in b[a:z + 1] if l.strip() and not l.strip().startswith((";", "."))]
    for a, z, t in sorted(loops, key=lambda x: -(x[1] - x[0]))[:top]:
        o = ops(a, z)
        c = collections.Counter(o)
        print(f"{t:14s} lines {a + st:6d}..{z + st:6d} insts {len(o):6d} mad {c['v_mad_u64_u32'] + c['v_mad_i64_i32']:5d} "
              f"scratch {sum(v for k, v in c.items() if k.startswith('scratch')):3d} nop {c['s_nop']:3d} "
              f"lds {sum(v for k, v in c.items() if k.startswith('ds_')):3d} "
              f"vmem {sum(v for k, v in c.items() if k.startswith(('global_', 'buffer_'))):3d} "
              f"salu {sum(v for k, v in c.items() if k.startswith('s_')):4d}")


if __name__ == "__main__":
    main()
