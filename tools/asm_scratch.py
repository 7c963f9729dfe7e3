"""Where a kernel instance spills: scratch loads/stores of one trace_kernel
instance in the -S output, grouped by basic block, with each block's loop
depth from the compiler's '; Loop Depth' annotations.

    python tools/asm_scratch.py inverse_path_tracer_amd/lib/obj/ipt_hip.s 0 0 1   # MODE SPEC BVH
"""
import re
import sys


def main():
    path, mode, spec, bvh = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
    s = open(path).read().split("\n")
    tag = "_ZN3ipt12trace_kernelILi%sELb%sELb%sE" % (mode, spec, bvh)
    i = next(k for k, l in enumerate(s) if l.startswith(tag) and re.match(re.escape(tag) + r"\S*:", l))
    j = i
    while "s_endpgm" not in s[j]:
        j += 1
    body = s[i:j]
    block, depth, counts, valu = "entry", 0, {}, {}
    for l in body:
        m = re.match(r"^(\.LBB\d+_\d+):\s*(;.*Loop Depth (\d+))?", l)
        if m:
            block, depth = m.group(1), int(m.group(3) or 0)
            continue
        t = l.strip()
        if t.startswith("scratch_"):
            key = (block, depth)
            counts.setdefault(key, [0, 0])[0 if "store" in t else 1] += 1
    tot = [0, 0]
    for (b, d), (st, ld) in counts.items():
        print("%-12s depth %d  stores %3d  loads %3d" % (b, d, st, ld))
        tot[0] += st
        tot[1] += ld
    print("total stores %d loads %d in %d lines" % (tot[0], tot[1], len(body)))


if __name__ == "__main__":
    main()
