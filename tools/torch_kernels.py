"""Torch (at::native) and HIP-runtime kernels inside one training step of a rocprofv3 kernel
trace (between two consecutive mvml_adam_flat launches), with the framework kernel before each:
    python tools/torch_kernels.py gpurun_out/TAG_prof/run_kernel_trace.csv [step_index]"""
import csv
import sys


def main(path, k=3):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adam_flat" in r["Kernel_Name"]]
    a, b = idx[k], idx[k + 1]
    seq = rows[a + 1:b + 1]
    tot, n = 0.0, 0
    for j, r in enumerate(seq):
        name = r["Kernel_Name"]
        if "at::native" not in name and "rocclr" not in name:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        n += 1
        prev = next((x["Kernel_Name"] for x in reversed(seq[:j]) if "at::native" not in x["Kernel_Name"]
                     and "rocclr" not in x["Kernel_Name"]), "")
        short = name[name.find("native::") + 8:] if "native::" in name else name
        prev = prev.replace("void ", "").replace("mvml::", "").replace("(anonymous namespace)::", "")
        print(f"{d:8.1f} us grid {r['Grid_Size_X']:>9}  {short[:50]:50s} after {prev[:60]}")
    step = (int(seq[-1]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e6
    print(f"{n} launches, {tot / 1e3:.3f} ms of a {step:.2f} ms step")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3)
