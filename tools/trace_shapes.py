#!/usr/bin/env python3
"""Per-dispatch-shape time of the kernels in a rocprofv3 --kernel-trace CSV.

Groups dispatches by (kernel, grid, workgroup, LDS bytes) and prints calls per step, the
average duration and the share of the step, largest first — the split-fp16 GEMM launches of
one step differ only in their grids, so this separates e.g. the layer-2 projection from the
Set2Set gates product.  `--match` keeps kernel names containing that substring.

    python tools/trace_shapes.py <dir with *kernel_trace.csv> --steps 20 --match gemm
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("mvml::", "").replace("void ", "")
    depth, cut = 0, len(name)
    for i, ch in enumerate(name):  # drop the argument list: the first '(' outside <...>
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    return name[:cut][:120]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20, help="divide totals by this many steps")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--bucket", action="store_true", help="round grids to 2 significant digits")
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True) \
        if os.path.isdir(a.trace) else [a.trace]
    tot, cnt = defaultdict(int), defaultdict(int)
    everything = 0
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                everything += d
                nm = r["Kernel_Name"]
                if a.match and a.match not in nm:
                    continue
                grid = tuple(int(r.get(f"Grid_Size_{c}", 0) or 0) for c in "XYZ")
                if a.bucket:  # batches of different sizes: bucket the grid to 2 significant digits
                    grid = tuple(int(float(f"{g:.2g}")) for g in grid)
                wg = tuple(int(r.get(f"Workgroup_Size_{c}", 0) or 0) for c in "XYZ")
                key = (short(nm), grid, wg, r.get("LDS_Block_Size", r.get("Group_Segment_Size", "")))
                tot[key] += d
                cnt[key] += 1
    s = a.steps
    print(f"all kernels: {everything / s / 1e6:.3f} ms/step over {s} steps (warm-up included if traced)")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:a.top]:
        nm, grid, wg, lds = k
        blocks = tuple(g // max(w, 1) for g, w in zip(grid, wg))
        print(f"{v / s / 1e6:8.3f} ms/step  x{cnt[k] / s:5.1f}  avg {v / cnt[k] / 1e6:7.3f} ms  "
              f"blocks {blocks} wg {wg} lds {lds}  {nm}")


if __name__ == "__main__":
    main()
