#!/usr/bin/env python3
"""Static instruction mix of a kernel's loops in a device .s file (hipcc --cuda-device-only -S):
    tools/isa_loop.py file.s <substring of the mangled kernel name>
Per top-level loop (\"This Loop Header\" in the compiler's block comments): VALU / SALU / SMEM / VMEM / LDS counts
and the vector memory instructions in it."""
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if l.split(":")[0].startswith("_Z") and key in l.split(":")[0]
              and ":" in l and not l.startswith("\t")]
    if not starts:
        sys.exit("no kernel matching %r" % key)
    a = starts[0]
    b = next(i for i in range(a, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[a:b]
    heads = [i for i, l in enumerate(body) if "This Loop Header" in l and "Depth=1" in l]
    heads.append(len(body))
    for h0, h1 in zip(heads[:-1], heads[1:]):
        cnt = {"valu": 0, "salu": 0, "smem": 0, "vmem": 0, "lds": 0}
        vm = []
        for l in body[h0:h1]:
            t = l.strip()
            if not t or t[0] in ";." or t.endswith(":"):
                continue
            op = t.split()[0]
            if op.startswith(("global_", "buffer_", "flat_")):
                cnt["vmem"] += 1
                vm.append(t[:80])
            elif op.startswith("ds_"):
                cnt["lds"] += 1
            elif op.startswith(("s_load", "s_buffer_load")):
                cnt["smem"] += 1
            elif op.startswith("v_"):
                cnt["valu"] += 1
            elif op.startswith("s_"):
                cnt["salu"] += 1
        print("loop at +%d (%d lines): %s" % (h0, h1 - h0, cnt))
        for t in vm:
            print("   ", t)


if __name__ == "__main__":
    main()
