"""Turn rocprofv3 PMC counter CSVs (FETCH_SIZE pass + WRITE_SIZE pass) into HBM traffic per
launch for the kernels bench.py reports, written to profiles/pmc_traffic.json.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE (KB) reports exactly half
of the bytes of wide (16 B/lane) coalesced reads, so hbm_read = 2 * FETCH_SIZE * 1024;
WRITE_SIZE (KB) is exact for 16-B stores.  Narrower accesses are uncalibrated, so the result
is an upper-bound-ish estimate for kernels that mix 4-B gathers in (documented in DESIGN.md).

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR [--out profiles/pmc_traffic.json]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

KERNELS = {"gat_agg_fwd": "gat_agg_fwd_kernel", "gat_agg_bwd_dst": "gat_agg_bwd_dst_kernel",
           "gat_agg_bwd_src": "gat_agg_bwd_src_kernel", "gemm": "gemm_f32_kernel",
           "set2set_seg_fwd": "seg_fwd_kernel"}


def read_counter(d, counter):
    per = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                for key, pat in KERNELS.items():
                    if pat in name:
                        per[key].append(float(row["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    fetch = read_counter(a.fetch_dir, "FETCH_SIZE")
    write = read_counter(a.write_dir, "WRITE_SIZE")
    out = {}
    for key in KERNELS:
        if not fetch.get(key) or not write.get(key):
            continue
        f_kb = sum(fetch[key]) / len(fetch[key])
        w_kb = sum(write[key]) / len(write[key])
        out[key] = {"launches": len(fetch[key]), "fetch_size_kb": round(f_kb, 1),
                    "write_size_kb": round(w_kb, 1),
                    "hbm_bytes_per_launch": int(2 * f_kb * 1024 + w_kb * 1024),
                    "correction": "read = 2 x FETCH_SIZE (gfx950 16-B/lane reads), write = WRITE_SIZE"}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
