#!/usr/bin/env python3
"""Idle time between kernels in a rocprofv3 --kernel-trace CSV, per training step.

Steps are delimited by the last kernel of torch's Adam (the step's final op): the last
`--steps` + 1 Adam ends bound the timed steps when the bench ran with --view-only-steps 0
--no-inference.  Reports per step: wall (first kernel start -> Adam end), busy (union of kernel
intervals), idle, and the largest gaps with the kernels on either side.

    python tools/trace_gaps.py <dir with *kernel_trace.csv> --steps 20
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def load(path):
    files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True) if os.path.isdir(path) else [path]
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--marker", default="adam", help="substring (lower-case) of the step's last kernel")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    rows = load(a.trace)
    ends = [i for i, r in enumerate(rows) if a.marker in r[2].lower()]
    # the LAST marker kernel of each step: a step may launch several Adam kernels back to back
    last = [i for j, i in enumerate(ends) if j + 1 == len(ends) or ends[j + 1] != i + 1]
    bounds = last[-(a.steps + 1):]
    tot_wall = tot_busy = 0.0
    pair_gap = defaultdict(float)
    pair_n = defaultdict(int)
    for s, (i0, i1) in enumerate(zip(bounds[:-1], bounds[1:])):
        seg = rows[i0 + 1:i1 + 1]
        t_start, t_end = rows[i0][1], seg[-1][1]
        busy, cur_s, cur_e = 0, None, None
        prev_end, prev_name = t_start, rows[i0][2]
        for st, en, nm in seg:
            gap = st - prev_end
            if gap > 0:
                k = (prev_name[:60], nm[:60])
                pair_gap[k] += gap
                pair_n[k] += 1
            if cur_e is None or st > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = st, en
            else:
                cur_e = max(cur_e, en)
            if en >= prev_end:
                prev_end, prev_name = en, nm
        busy += cur_e - cur_s
        wall = t_end - t_start
        tot_wall += wall
        tot_busy += busy
        print(f"step {s:2d}: wall {wall / 1e6:8.3f} ms  busy {busy / 1e6:8.3f}  idle {(wall - busy) / 1e6:7.3f}  kernels {len(seg)}")
    n = max(len(bounds) - 1, 1)
    print(f"mean: wall {tot_wall / n / 1e6:.3f} ms  busy {tot_busy / n / 1e6:.3f}  idle {(tot_wall - tot_busy) / n / 1e6:.3f} ms/step")
    print("largest idle (summed over the steps, per kernel pair prev -> next):")
    for k, v in sorted(pair_gap.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"  {v / n / 1e6:8.3f} ms/step  x{pair_n[k] / n:5.1f}  {k[0]}  ->  {k[1]}")


if __name__ == "__main__":
    main()
