"""Per-kernel averages of rocprofv3 --pmc counter CSVs:  python tools/pmc_summary.py DIR [pattern]"""
import collections
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"(gat_\w+|seg_\w+|gemm_\w+|lstm_\w+)(<[^>]*>)?")
agg = collections.defaultdict(list)
for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        m = pat.search(r["Kernel_Name"])
        if m:
            agg[(m.group(0), r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:45s} {c:20s} n={len(v):3d} avg={sum(v) / len(v):.4g}")
