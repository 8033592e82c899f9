"""The LDS-DMA split-fp16 tile (mvml_gemm_f16x2_planes) against the register-staged 256x256
tile (mvml_gemm_f16x2_rows, B from its il4 image) on the row-scaled products of a config-3
training step: time per launch, fp32-equivalent TF/s and the fraction of 833 TF/s (the fp16
MFMA peak / 3), and each result's error against float64 on sampled rows.

    python tools/planes_bench.py [shape indices, e.g. 0,1] [--iters 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mvml-mpi_amd"), ROOT]
import torch  # noqa: E402

from mvml_gat.functional import (absmax, absmax_rows, gemm, gemm_planes, slot, split_il4,  # noqa: E402
                                 split_il8)

N_ATOMS, B = 1754373, 65536
SHAPES = [  # name, M, N, K
    ("L2 fwd  X Wcat^T", N_ATOMS, 1928, 768),
    ("L2 dX   gY Wcat", N_ATOMS, 768, 1928),
    ("LSTM gates l0", B, 1536, 1152),
    ("LSTM gates l1", B, 1536, 768),
    ("LSTM dx l0", B, 1152, 1536),
    ("odd     K=76 N=1544", 100003, 1544, 76),
]
PEAK = 2500.0 / 3


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shapes", nargs="?", default=None)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    shapes = SHAPES if a.shapes is None else [SHAPES[int(i)] for i in a.shapes.split(",")]
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    for name, M, N, K in shapes:
        # rows spread over 2^-8 .. 2^8 (the per-row scales matter), B plain
        A = torch.randn((M, K), device=dev, generator=g) * torch.exp2(
            torch.randint(-8, 9, (M, 1), device=dev, generator=g).float())
        Bm = torch.randn((N, K), device=dev, generator=g)
        mx = torch.zeros(2, dtype=torch.int32, device=dev)
        absmax(Bm, N, K, K, mx, 1)
        rows = absmax_rows(A, M, K, K)
        il4 = split_il4(Bm, N, K, K, slot(mx, 1))
        il8 = split_il8(Bm, N, K, K, amax_ptr=slot(mx, 1))
        kp = il8.shape[1]
        flops = 2.0 * M * N * K
        C0 = torch.empty((M, N), device=dev)
        C1 = torch.empty((M, N), device=dev)
        C2 = torch.empty((M, N), device=dev)
        t_old = timed(lambda: gemm(A, Bm, M, N, K, 0, 0, K, K, C0, N, amax=(None, slot(mx, 1)), arows=rows,
                                   bil4=il4), a.iters)
        t_new = timed(lambda: gemm_planes(A, M, N, K, K, il8, kp, C1, N, slot(mx, 1), arows=rows), a.iters)
        aimg = split_il8(A, M, K, K, rows_max=rows)
        t_split = timed(lambda: split_il8(A, M, K, K, rows_max=rows, out=aimg), a.iters)
        t_img = timed(lambda: gemm_planes(aimg, M, N, K, kp, il8, kp, C2, N, slot(mx, 1), arows=rows,
                                          a_image=True), a.iters)
        # float64 on sampled rows: each row's error relative to its own max
        idx = torch.cat([torch.arange(0, min(M, 300), device=dev),
                         torch.randint(0, M, (300,), device=dev, generator=g),
                         torch.arange(max(0, M - 300), M, device=dev)])
        ref = A[idx].double() @ Bm.double().T
        den = ref.abs().amax(dim=1, keepdim=True).clamp_min(1e-300)

        def err(Cx):
            return ((Cx[idx].double() - ref).abs() / den).max().item()

        def tf(ms):
            return flops / (ms * 1e-3) / 1e12

        print(f"{name:20s} M={M:8d} N={N:5d} K={K:5d} | rows(il4) {t_old:7.3f} ms {tf(t_old):6.1f} TF/s "
              f"({tf(t_old) / PEAK:.3f}) err {err(C0):.2e} | planes {t_new:7.3f} ms {tf(t_new):6.1f} "
              f"({tf(t_new) / PEAK:.3f}) err {err(C1):.2e} | A image {t_img:7.3f} ms ({tf(t_img) / PEAK:.3f}) "
              f"err {err(C2):.2e} + split {t_split:6.3f} ms | planes vs rows max diff "
              f"{((C1 - C0).abs().max() / C0.abs().max()).item():.2e}", flush=True)
        del A, Bm, C0, C1, C2, aimg, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
