"""Per-kernel GEMM counter report from rocprofv3 --pmc passes and a --kernel-trace --stats run of
the same command (tools/pmc_gemm.sh; the passes run separately, see MI355X_MICROARCH.md §PMC).

    python tools/pmc_gemm_report.py gpurun_out/pmc_g1 gpurun_out/pmc_g2 gpurun_out/pmc_g3 \
        --stats gpurun_out/prof_gk/run_kernel_stats.csv > profiles/r05_pmc_gemm_config3.txt

Units (MI355X_MICROARCH.md §PMC): GRBM_GUI_ACTIVE is summed over the 8 XCDs; SQ_WAVE_CYCLES,
SQ_WAIT_* and SQ_ACTIVE_INST_* count quad-cycles summed over waves; SQ_VALU_MFMA_BUSY_CYCLES
counts SIMD cycles summed over the 1024 SIMDs.  So
    mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024)
is the fraction of SIMD-cycles with the matrix pipe busy during the launch, and the wave-cycle
split (issue / parked on s_waitcnt or barrier / issue-stalled) adds up to ~1.
"""
import argparse
import collections
import csv
import os
import re


def short(name):
    m = re.search(r"(gemm_\w+_kernel<[^>]*>)", name)
    return m.group(1) if m else name[:60]


def load(dirs):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        with open(os.path.join(d, "run_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                if "gemm_" not in r["Kernel_Name"]:
                    continue
                per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def load_stats(path):
    out = {}
    if not path:
        return out
    with open(path) as f:
        for r in csv.DictReader(f):
            if "gemm_" in r["Name"]:
                out[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3,
                                         float(r["Percentage"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--stats")
    ap.add_argument("--min-calls", type=int, default=10)
    a = ap.parse_args()
    per = load(a.dirs)
    stats = load_stats(a.stats)

    def avg(c, k):
        v = c.get(k)
        return sum(v) / len(v) if v else float("nan")

    print("kernel <AK, BKM, EPI, FAST, NP, BPS, ROWS, EX>  (x3w/x3s/f32 as in csrc/gemm_f32.hip;")
    print("  planes <APS, ROWS, EX, CELL, BK, ABL> as in csrc/gemm_planes.hip); clk_GHz = GRBM_GUI_ACTIVE / 8 / duration")
    hdr = ("calls", "avg_us", "step%", "mfma_busy", "issue", "parked", "stalled", "lds_stall",
           "lds_conf", "valu/mfma", "clk_GHz")
    print(f"{'kernel':58s} " + " ".join(f"{h:>9s}" for h in hdr))
    rows = []
    for k, c in per.items():
        n = len(c.get("GRBM_GUI_ACTIVE", []))
        if n < a.min_calls and k not in stats:
            continue
        cyc = avg(c, "GRBM_GUI_ACTIVE") / 8
        wave = avg(c, "SQ_WAVE_CYCLES")
        st = stats.get(k, (n, float("nan"), float("nan")))
        rows.append((st[2] if st[2] == st[2] else -1, k, (
            st[0], st[1], st[2],
            avg(c, "SQ_VALU_MFMA_BUSY_CYCLES") / (cyc * 1024),
            avg(c, "SQ_ACTIVE_INST_ANY") / wave,
            avg(c, "SQ_WAIT_ANY") / wave,
            avg(c, "SQ_WAIT_INST_ANY") / wave,
            avg(c, "SQ_WAIT_INST_LDS") / wave,
            avg(c, "SQ_LDS_BANK_CONFLICT") / avg(c, "SQ_LDS_IDX_ACTIVE"),
            avg(c, "SQ_INSTS_VALU") / avg(c, "SQ_INSTS_MFMA"),
            cyc / (st[1] * 1e3) if st[1] == st[1] else float("nan"))))
    for _, k, v in sorted(rows, reverse=True):
        if v[0] < a.min_calls:
            continue
        print(f"{k:58s} " + " ".join(f"{x:9.3f}" if isinstance(x, float) else f"{x:9d}" for x in v))


if __name__ == "__main__":
    main()
