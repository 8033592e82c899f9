"""Turn rocprofv3 PMC counter CSVs (FETCH_SIZE pass + WRITE_SIZE pass) into HBM traffic per
launch of the C-ABI entry points bench.py reports, written to profiles/pmc_traffic.json.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE (KB) reports exactly half
of the bytes of wide (16 B/lane) coalesced reads, so hbm_read = 2 * FETCH_SIZE * 1024;
WRITE_SIZE (KB) is exact for 16-B stores.  The aggregation kernels read their streams with
16-B buffer loads; their small 4-B index / logit reads are uncalibrated (documented in
DESIGN.md).  One entry-point launch = one launch of each of its kernels, so its traffic is the
sum of the per-kernel averages.  The result is stored under the WORKLOAD key bench.py computes
("<workload>/mols_per_step=<n>[/proj_bf16]"), so a bench line only ever reports traffic that was
profiled on its own workload.

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR --workload KEY [--out profiles/pmc_traffic.json]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ENTRIES = {  # C-ABI entry point -> its kernels (name substrings; "[big]": the big-window
    # instantiation, template argument BIG = true, launched beside the molecule-window one)
    "gat_agg_fwd": ["gat_softmax_kernel", "gat_agg_fwd_lds_kernel", "gat_agg_fwd_lds_kernel[big]",
                    "gat_agg_fwd_gather_kernel",
                    # round 5: the destination-wave forward (and its split-softmax launch)
                    "gat_agg_fwd_dst_kernel", "gat_softmax_dst4_kernel", "gat_softmax_dst_kernel"],
    "gat_agg_bwd": ["gat_agg_bwd_lds_kernel", "gat_agg_bwd_lds_kernel[big]", "gat_agg_bwd_dst_kernel",
                    "gat_agg_bwd_src_kernel", "gat_mean_bwd_src_kernel", "gat_mean_bwd_softmax_kernel",
                    "gat_mean_bwd_gel_kernel",
                    # round 5: the flatten layer's one-pass source-atom backward
                    "gat_flat_bwd_src1_kernel"],
    "set2set_seg_fwd": ["seg_fwd_kernel"],
    # round 5: the small-K GAT projection (layer 1)
    "gemm_smallk": ["gemm_smallk_kernel"],
}
# kernels launched exactly once per entry-point call, whichever path the call takes (a call of
# mvml_gat_agg_bwd launches the molecule-window kernel, or — head-mean layer by source atom —
# gat_mean_bwd_src_kernel instead): the per-launch traffic is the entry's kernels' total over
# the number of calls, so layers on different kernel paths average correctly
ANCHORS = {"gat_agg_fwd": ["gat_agg_fwd_lds_kernel", "gat_agg_fwd_dst_kernel"],
           "gat_agg_bwd": ["gat_agg_bwd_lds_kernel", "gat_mean_bwd_src_kernel", "gat_flat_bwd_src1_kernel"],
           "set2set_seg_fwd": ["seg_fwd_kernel"],
           "gemm_smallk": ["gemm_smallk_kernel"]}


def _pattern(name, pat):
    """Does kernel `name` (demangled) belong to pattern `pat`?"""
    big = pat.endswith("[big]")
    base = pat[:-5] if big else pat
    if base not in name:
        return False
    if "lds_kernel" in base:
        return ("true>" in name) == big
    return True


def read_counter(d, counter):
    per = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                for entry, pats in ENTRIES.items():
                    for pat in pats:
                        if _pattern(name, pat):
                            per[(entry, pat)].append(float(row["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    fetch = read_counter(a.fetch_dir, "FETCH_SIZE")
    write = read_counter(a.write_dir, "WRITE_SIZE")
    out = {}
    for entry, pats in ENTRIES.items():
        calls_f = sum(len(fetch.get((entry, p), [])) for p in ANCHORS[entry])
        calls_w = sum(len(write.get((entry, p), [])) for p in ANCHORS[entry])
        if not calls_f or not calls_w:
            continue
        f_kb = sum(sum(fetch[(entry, p)]) for p in pats if fetch.get((entry, p))) / calls_f
        w_kb = sum(sum(write[(entry, p)]) for p in pats if write.get((entry, p))) / calls_w
        if not f_kb:
            continue
        out[entry] = {"kernels": {p: {"launches": len(fetch.get((entry, p), [])),
                                      "fetch_size_kb": round(sum(fetch[(entry, p)]) / len(fetch[(entry, p)]), 1)
                                      if fetch.get((entry, p)) else None,
                                      "write_size_kb": round(sum(write[(entry, p)]) / len(write[(entry, p)]), 1)
                                      if write.get((entry, p)) else None} for p in pats},
                      "hbm_bytes_per_launch": int(2 * f_kb * 1024 + w_kb * 1024),
                      "calls": calls_f,
                      "correction": "read = 2 x FETCH_SIZE (gfx950 16-B/lane reads), write = WRITE_SIZE; "
                                    "averaged over both GAT layers"}
    try:
        with open(a.out) as f:
            allw = json.load(f)
    except (OSError, ValueError):
        allw = {}
    allw[a.workload] = out
    with open(a.out, "w") as f:
        json.dump(allw, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
