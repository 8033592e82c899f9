"""Layer-1 projection on the config-3 shape (M = atoms of a 65,536-molecule batch, N = 1544 Wcat
rows, K = 76): the small-K memory kernel (option smallk 1 = non-temporal stores, the default;
2 = plain stores; 3 / 4 = 8 / 128 row blocks per wave instead of 32; 5 / 6 = timing ablations
without the MFMAs / without the C stores — wrong results; 10 = B fragments in registers, the
first build) against the 256x256 tile (smallk 0),
interleaved in one process; HIP events on torch's current stream.  Default X: 0/1 values like
the atom features (the kernel skips the products of A's zero low plane); --random: Gaussian.
Algorithmic bytes: read X, its row maxima and the il4 weight image once, write Y once.

    python tools/smallk_bench.py [--m 1753156] [--n 1544] [--k 76] [--iters 10]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mvml-mpi_amd"), ROOT]
import torch  # noqa: E402

from mvml_gat._lib import call, lib, option, ptr, stream_ptr, ws_ptr_size  # noqa: E402
from mvml_gat.functional import _row_pitch, absmax, absmax_rows, slot  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1753156)
    ap.add_argument("--n", type=int, default=1544)
    ap.add_argument("--k", type=int, default=76)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--kinds", default="1,10,2,5,6,0")
    ap.add_argument("--random", action="store_true")
    a = ap.parse_args()
    M, N, K = a.m, a.n, a.k
    dev = "cuda"
    st = stream_ptr()
    # 0 / 1 values like the atom features (--random: Gaussian rows, no zero low plane)
    X = torch.randn(M, K, device=dev) if a.random else (torch.rand(M, K, device=dev) < 0.15).float()
    W = torch.randn(N, K, device=dev) * 0.05
    ldc = _row_pitch(N)
    Y = torch.empty(M, ldc, device=dev)
    bmx = torch.zeros(1, dtype=torch.int32, device=dev)
    absmax(W, N, K, K, bmx, 0)
    rows = absmax_rows(X, M, K, K)
    img = torch.empty_like(W)
    call("mvml_split_f16x2_il4", N, K, ptr(W), K, slot(bmx, 0), ptr(img), st)
    wp, wn = ws_ptr_size(lib().mvml_gemm_workspace_size(M, N, K), dev)
    nbytes = 4 * (M * N + M * K + M + N * K)
    kinds = [int(x) for x in a.kinds.split(",")]

    def run(kind):
        with option("smallk", kind):
            call("mvml_gemm_f16x2_rows", M, N, K, ptr(X), K, ptr(W), K, 0, ptr(img), ptr(rows), slot(bmx, 0),
                 None, 0.0, 0, ptr(Y), ldc, wp, wn, st)

    outs = {}
    for kd in kinds:
        run(kd)
        torch.cuda.synchronize()
        outs[kd] = Y[:, :N].clone()
    ref = outs[0 if 0 in outs else kinds[-1]].double()
    times = {kd: [] for kd in kinds}
    for _ in range(a.iters):
        for kd in kinds:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            run(kd)
            e.record()
            torch.cuda.synchronize()
            times[kd].append(s.elapsed_time(e))
    print(f"M={M} N={N} K={K} ldc={ldc}: algorithmic {nbytes / 1e9:.2f} GB per launch")
    for kd in kinds:
        t = sorted(times[kd])[len(times[kd]) // 2]
        d = float(((outs[kd].double() - ref).abs().amax(1) / ref.abs().amax(1).clamp_min(1e-30)).max())
        print(f"smallk={kd}: median {t:.3f} ms  min {min(times[kd]):.3f}  {nbytes / t / 1e6:.0f} GB/s "
              f"({nbytes / t / 1e6 / 8000:.3f} of 8 TB/s)  max row rel diff vs smallk={kinds[-1]}: {d:.2e}")


if __name__ == "__main__":
    main()
