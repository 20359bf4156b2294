#!/usr/bin/env python3
"""tools/asm_mix.py ASM [VARIANT] [BVH] [LIST] — static instruction mix of one
trace_samples_kernel instantiation in a `make asm` listing (build/rtg_trace_sS.s):
instruction classes, f64 opcodes, scratch accesses and the register/occupancy
summary the compiler prints after the function."""
import collections
import re
import sys


def kernel_body(text, sym):
    i = text.index(sym + ":")
    j = text.index(".Lfunc_end", i)
    return text[i:j], text[j:j + 4000]


def main():
    path = sys.argv[1]
    variant = sys.argv[2] if len(sys.argv) > 2 else "0"
    bvh = sys.argv[3] if len(sys.argv) > 3 else "0"
    lst = sys.argv[4] if len(sys.argv) > 4 else "1"  # kList: the compacted launch
    text = open(path).read()
    s = re.search(r"_ZN3rtg20trace_samples_kernelILi(\d+)E", text).group(1)
    sym = "_ZN3rtg20trace_samples_kernelILi%sELb0ELi%sELb%sELb%sEEEvNS_10KernelArgsE" % (
        s, variant, bvh, lst)
    body, tail = kernel_body(text, sym)
    ops = [l.split()[0] for l in body.split("\n")
           if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
    cls = collections.Counter()
    f64 = collections.Counter()
    for o in ops:
        if o.startswith("v_") and "f64" in o:
            cls["valu_f64"] += 1
            f64[o] += 1
        elif o.startswith("v_"):
            cls["valu"] += 1
        elif o.startswith(("s_load", "s_buffer_load")):
            cls["smem"] += 1
        elif o.startswith(("s_cbranch", "s_branch")):
            cls["branch"] += 1
        elif o.startswith("s_"):
            cls["salu"] += 1
        elif o.startswith("scratch_"):
            cls["scratch"] += 1
        elif o.startswith(("buffer_", "global_", "flat_")):
            cls["vmem"] += 1
        elif o.startswith("ds_"):
            cls["lds"] += 1
        else:
            cls[o] += 1
    print(sym)
    print("instructions", len(ops), dict(cls))
    print("f64", dict(f64.most_common()))
    for k in ("NumVgprs", "NumAgprs", "NumSgprs", "ScratchSize", "Occupancy"):
        mm = re.search(r"; %s: (\d+)" % k, tail)
        print(k, mm and mm.group(1))


if __name__ == "__main__":
    main()
