"""Static instruction histogram of one trace_kernel instance in the -S output.

    python tools/asm_hist.py inverse_path_tracer_amd/lib/obj/ipt_hip.s 0 0 0 [top]
"""
import collections
import sys


def body(path, mode, spec, bvh):
    s = open(path).read().split("\n")
    tag = "_ZN3ipt12trace_kernelILi%sELb%sELb%sE" % (mode, spec, bvh)
    i = next(k for k, l in enumerate(s) if l.startswith(tag) and ": ;" in l)
    j = i
    while "s_endpgm" not in s[j]:
        j += 1
    return s[i:j]


def main():
    b = body(*sys.argv[1:5])
    top = int(sys.argv[5]) if len(sys.argv) > 5 else 60
    c = collections.Counter()
    for l in b:
        t = l.strip().split()
        if t and t[0][:2] in ("v_", "s_", "ds", "gl", "sc", "bu"):
            c[t[0]] += 1
    print(sum(v for k, v in c.items() if k.startswith("v_")), "static VALU")
    for k, v in c.most_common(top):
        print("%-28s %d" % (k, v))


if __name__ == "__main__":
    main()
