"""Instruction mix of the hot basic blocks of a kernel in a hipcc -S dump.

usage: python scripts/micro/isa_blocks.py FILE.s NAME_SUBSTRING [--all]

Prints, per kernel whose symbol contains NAME_SUBSTRING, its VGPR count and
the blocks that hold a v_rsq_f64 and no v_div_scale_f64 (the shared-reciprocal
pair loops of the strict kernels), or every block with --all.
"""
import re
import sys
from collections import Counter


def main():
    path, sub = sys.argv[1], sys.argv[2]
    show_all = "--all" in sys.argv
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and sub in l]
    for st in starts:
        end = st
        while not lines[end].startswith(".Lfunc_end"):
            end += 1
        blocks, cur = [], None
        for l in lines[st:end]:
            if re.match(r"^\.LBB\d+_\d+:", l):
                cur = [l.split()[0], []]
                blocks.append(cur)
            elif cur and l.startswith("\t") and not l.strip().startswith((";", ".")):
                cur[1].append(l.strip().split()[0])
        vg = next((l.strip() for l in lines[end:end + 400] if "NumVgprs:" in l), "")
        print(lines[st].split(":")[0][-70:], vg)
        for name, ins in blocks:
            c = Counter(ins)
            if show_all or (c.get("v_rsq_f64_e32", 0) and not c.get("v_div_scale_f64", 0)):
                print("  ", name, len(ins), sorted(c.items(), key=lambda x: -x[1])[:16])


if __name__ == "__main__":
    main()
