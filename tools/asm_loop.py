"""Instruction mix of the innermost loops of one kernel in a hipcc -S listing.
    python tools/asm_loop.py FILE.s KERNEL_SUBSTRING [--dump OUT]"""
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    s = open(path).read().split("\n")
    starts = [i for i, l in enumerate(s) if l.startswith("_Z") and pat in l and ": ;" in l + " ;" and not l.startswith("\t")]
    if not starts:
        sys.exit("kernel not found")
    i0 = starts[0]
    print(s[i0])
    i1 = next(i for i in range(i0 + 1, len(s)) if s[i].startswith(".Lfunc_end"))
    body = s[i0:i1]
    labels = {l.strip().rstrip(":"): k for k, l in enumerate(body) if re.match(r"^\.LBB\S+:", l.strip())}
    for k, l in enumerate(body):
        m = re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < k:
            a = labels[m.group(1)]
            seg = [x.strip() for x in body[a:k + 1] if x.strip() and not x.strip().startswith((".", ";"))]
            cnt = {}
            for x in seg:
                op = x.split()[0]
                key = ("mfma" if "mfma" in op else "ds_read" if op.startswith("ds_read") else
                       "ds_write" if op.startswith("ds_write") else
                       "vmem" if op.startswith(("global_", "buffer_")) else
                       "waitcnt" if op == "s_waitcnt" else "barrier" if op == "s_barrier" else
                       "salu" if op.startswith("s_") else "valu")
                cnt[key] = cnt.get(key, 0) + 1
            print(f"loop lines {a}-{k}: {len(seg)} instrs {cnt}")
            if dump:
                open(dump, "w").write("\n".join(body[a:k + 1]))
    for l in s[i1:i1 + 400]:
        if re.search(r"NumVgprs|NumAgprs|ScratchSize|Occupancy|NumSgprs|TotalNumVgpr", l):
            print(l.strip())


if __name__ == "__main__":
    main()
