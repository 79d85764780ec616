#!/usr/bin/env python3
"""Per-basic-block instruction counts of one kernel in a gfx950 assembly listing (CPU, no GPU):

    hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S prometheus_amd/csrc/prom_mol.hip -o /tmp/m.s
    python tools/isa_blocks.py /tmp/m.s k_tau_molILi0ELi1ELb1 [--min 20] [--dump .LBB3_12]

Counts VALU (v_*), SALU (s_*), VMEM (global_/buffer_), LDS (ds_) and SMEM (s_load/s_buffer) per block, marks
loop back-edges, so a kernel's hot loop body can be read off before a GPU run.
"""
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 0
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    lines = open(path).read().split("\n")
    names = [l.split(":")[0] for l in lines if l.startswith("_Z") and key in l and l.rstrip().endswith(tuple(":;")) or
             (l.startswith("_Z") and key in l and ":" in l)]
    if not names:
        sys.exit("no kernel matching %s" % key)
    name = names[0]
    i0 = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    i1 = next(i for i in range(i0, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur = [], None
    for l in lines[i0:i1]:
        m = re.match(r"^(\.LBB\S+):", l)
        if m or cur is None:
            cur = {"name": m.group(1) if m else "entry", "v": 0, "s": 0, "vmem": 0, "ds": 0, "smem": 0, "br": [],
                   "text": []}
            blocks.append(cur)
            if m:
                continue
        t = l.strip()
        if not t or t.startswith(";") or t.startswith("."):
            continue
        cur["text"].append(t)
        op = t.split()[0]
        if op.startswith("v_"):
            cur["v"] += 1
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            cur["smem"] += 1
        elif op.startswith("s_"):
            cur["s"] += 1
            if op.startswith("s_cbranch") or op == "s_branch":
                cur["br"].append(t.split()[-1])
        elif op.startswith("global_") or op.startswith("buffer_"):
            cur["vmem"] += 1
        elif op.startswith("ds_"):
            cur["ds"] += 1
    order = {b["name"]: k for k, b in enumerate(blocks)}
    print(name)
    for k, b in enumerate(blocks):
        back = [t for t in b["br"] if t in order and order[t] <= k]
        if (b["v"] + b["s"] < mn and not back) or (dump and b["name"] != dump):
            continue
        print("%-14s V %4d  S %4d  SMEM %3d  VMEM %3d  DS %3d %s" % (
            b["name"], b["v"], b["s"], b["smem"], b["vmem"], b["ds"], ("<- loop to " + ",".join(back)) if back else ""))
        if dump and b["name"] == dump:
            print("\n".join("    " + t for t in b["text"]))


if __name__ == "__main__":
    main()
