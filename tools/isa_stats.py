#!/usr/bin/env python3
"""isa_stats.py — resource usage of one kernel in a hipcc -S listing (VGPRs, AGPRs, spills, scratch) and the
scratch ops inside its loops.   usage: python3 tools/isa_stats.py listing.s kernel_substring"""
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    s = open(path).read()
    metas = s.split("\n  - ")
    for m in metas:
        nm = re.search(r"\.name:\s+(\S+)", m)
        if not nm or name not in nm.group(1):
            continue
        out = {"kernel": nm.group(1)}
        for k in ("vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size"):
            v = re.search(r"\." + k + r":\s+(\d+)", m)
            out[k] = int(v.group(1)) if v else None
        print(out)


if __name__ == "__main__":
    main()
