"""Practical HBM yardsticks on the box, to read the kernels' roofline fractions against: what
plain streaming achieves with the runtime's and torch's own kernels (no mvml code), 4 GiB
operands, HIP events, GB/s and fraction of the 8 TB/s nominal peak.

  read    x.sum() over fp32 (torch reduction: reads only), and mvml_absmax_f32's flat pass
          (grid-stride float4 loads, one atomic per workgroup: the simplest read stream here)
  write   hipMemsetAsync (tensor.zero_) and torch.fill_(1.0) (stores only)
  copy    hipMemcpyAsync device-to-device (y.copy_(x)): read + write
  scale   y = x * 2 (torch elementwise: read + write)

    python tools/hbm_ceiling.py [--gib 4] [--reps 10]
"""
import argparse

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mvml-mpi_amd")]
from mvml_gat.functional import absmax  # noqa: E402

PEAK = 8000.0  # GB/s, MI355X HBM3E nominal


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    n = int(a.gib * (1 << 30)) // 4
    x = torch.randn(n, device="cuda")
    y = torch.empty_like(x)
    nb = n * 4
    amx = torch.zeros(1, dtype=torch.int32, device="cuda")
    tests = [("read  (x.sum)", lambda: x.sum(), nb),
             ("read  (mvml absmax flat)", lambda: absmax(x, 1, n, n, amx, 0), nb),
             ("read  (mvml absmax, strided)", lambda: absmax(x, n // 2048, 1024, 2048, amx, 0), nb // 2),
             ("write (hipMemset, zero_)", lambda: y.zero_(), nb),
             ("write (torch fill_ 1.0)", lambda: y.fill_(1.0), nb),
             ("copy  (hipMemcpy D2D)", lambda: y.copy_(x), 2 * nb),
             ("scale (y = 2 x)", lambda: torch.mul(x, 2.0, out=y), 2 * nb)]
    for name, fn, bytes_ in tests:
        ms = timed(fn, a.reps)
        gbs = bytes_ / ms / 1e6
        print(f"{name:28s} {ms:8.3f} ms  {gbs:7.0f} GB/s  {gbs / PEAK:.3f} of peak", flush=True)


if __name__ == "__main__":
    main()
