"""Projection GEMM with and without the logits epilogue (mvml_gat_proj_fwd vs mvml_gemm_f32)
on the bench shapes (65,536 KEGG-like molecules)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mvml-mpi_amd"), ROOT]
import torch  # noqa: E402

from mvml_gat import _lib  # noqa: E402
from mvml_gat._lib import call, ptr  # noqa: E402
from mvml_gat.functional import _GEMM_ENTRY, gemm  # noqa: E402


def timeit(fn, it=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    N = 1754373
    L = _lib.lib()
    st = _lib.stream_ptr()
    for H, F, K, mean in ((4, 192, 76, 0), (4, 384, 768, 1)):
        C = L.mvml_gat_proj_cols(H, F, mean)
        ldy = (C + 3) // 4 * 4
        X = torch.randn(N, K, device="cuda")
        W = torch.randn(C, K, device="cuda") * 0.05
        Y = torch.empty(N, ldy, device="cuda")
        attn = torch.randn(2 * H * F, device="cuda")
        elr = torch.empty(N, 2 * H, device="cuda")
        wsz = L.mvml_gat_proj_fwd_workspace_size(N, H, F)
        ws = torch.empty(wsz, dtype=torch.uint8, device="cuda")
        fl = 2 * N * C * K
        for algo in ("f32", "x3", "f16x2"):
            t0 = timeit(lambda: gemm(X, W, N, C, K, 0, 0, K, K, Y, ldy, algo=algo))
            t1 = timeit(lambda: call("mvml_gat_proj_fwd", N, ptr(X), K, K, ptr(W), K, ptr(attn), H, F,
                                     mean, _GEMM_ENTRY[algo][1], ptr(Y), ldy, ptr(elr), None, None, None, 0,
                                     ptr(ws), wsz, st))
            print(f"H{H} F{F} K{K} {algo}: gemm {t0:8.3f} ms ({fl / t0 / 1e9:6.1f} TF/s)   proj_fwd "
                  f"{t1:8.3f} ms ({fl / t1 / 1e9:6.1f} TF/s)")


if __name__ == "__main__":
    main()
