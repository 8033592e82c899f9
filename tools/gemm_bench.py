"""Microbenchmark of mvml_gemm_f32 on the GEMM shapes of one GNNModule training step, with
torch.matmul (hipBLASLt / rocBLAS fp32) on the same shapes as a yardstick.  Prints TF/s."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mvml-mpi_amd"), ROOT]
import torch  # noqa: E402
from mvml_gat._lib import option  # noqa: E402
from mvml_gat.functional import gemm  # noqa: E402

N_ATOMS, B = 1754373, 65536
SHAPES = [  # name, M, N, K, a_kmajor, b_kmajor
    ("L2 fwd  X*Wcat^T", N_ATOMS, 1928, 768, 0, 0),
    ("L2 dX   gY*Wcat", N_ATOMS, 768, 1928, 0, 1),
    ("L2 dW   gY^T*X", 1928, 768, N_ATOMS, 1, 1),
    ("L1 fwd  K=74", N_ATOMS, 1544, 74, 0, 0),
    ("LSTM gates x*Wih^T", B, 1536, 768, 0, 0),
    ("LSTM dx g*Wih", B, 768, 1536, 0, 1),
    ("LSTM dW g^T*x", 1536, 768, B, 1, 1),
    ("LSTM dW batched l0", 1536, 768, 5 * B, 1, 1),
    ("LSTM dW batched hh", 1536, 384, 5 * B, 1, 1),
    ("LSTM dW batched l1", 1536, 384, 6 * B, 1, 1),
    ("L1 dW   gY^T*X N=76", 1552, 76, N_ATOMS, 1, 1),
    ("L1 fwd  K=76", N_ATOMS, 1544, 76, 0, 0),
    ("LSTM dxh l>0 merged", B, 768, 1536, 0, 1),
    ("LSTM dxh l0 merged", B, 1152, 1536, 0, 1),
    ("BiLSTM step fwd 1024", 1024, 1536, 384, 0, 0),
    ("BiLSTM step fwd 2730", 2730, 1536, 384, 0, 0),
    ("BiLSTM step fwd 8192", 8192, 1536, 384, 0, 0),
    ("BiLSTM step bwd 1024", 1024, 384, 1536, 0, 1),
    ("BiLSTM step bwd 2730", 2730, 384, 1536, 0, 1),
    ("BiLSTM step bwd 8192", 8192, 384, 1536, 0, 1),
]


def tf(fn, flops, it=30):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / it
    return ms, flops / (ms * 1e-3) / 1e12


def main():
    dev = "cuda"
    torch.manual_seed(0)
    algos = sys.argv[1].split(",") if len(sys.argv) > 1 else ["x3-128", "x3-256"]
    shapes = SHAPES
    if len(sys.argv) > 2:  # e.g. "0,4": indices into SHAPES
        shapes = [SHAPES[int(i)] for i in sys.argv[2].split(",")]
    for name, M, N, K, ak, bk in shapes:
        A = torch.randn((K, M) if ak else (M, K), device=dev)
        Bm = torch.randn((K, N) if bk else (N, K), device=dev)
        C = torch.empty((M, N), device=dev)
        flops = 2 * M * N * K
        cols = []
        for algo in algos:
            if algo.startswith(("f16x2r", "f16x2i")):  # per-row A maxima (r) / B il4 image (i)
                rws, il = algo.startswith(("f16x2r", "f16x2ri")), "i" in algo.split("-")[0][5:]
                if ak:
                    cols.append(f"{algo}      n/a")
                    continue
                from mvml_gat.functional import absmax, absmax_rows, slot, split_il4
                mx = torch.zeros(2, dtype=torch.int32, device=dev)
                absmax(A, M, K, K, mx, 0)
                absmax(Bm, Bm.shape[0], Bm.shape[1], Bm.shape[1], mx, 1)
                rows = absmax_rows(A, M, K, K) if rws else None
                img = split_il4(Bm, Bm.shape[0], Bm.shape[1], Bm.shape[1], slot(mx, 1)) if il else None
                with option("gemm_tile", int(algo.split("-")[1]) if "-" in algo else 0):
                    ms, t = tf(lambda: gemm(A, Bm, M, N, K, 0, bk, K, N if bk else K, C, N,
                                            amax=(None if rws else slot(mx, 0), slot(mx, 1)), arows=rows,
                                            bil4=img), flops)
            elif algo == "torch":
                At = A.t() if ak else A
                Bt = Bm if bk else Bm.t()
                ms, t = tf(lambda: torch.matmul(At, Bt, out=C), flops)
            else:
                a = algo.split("-")[0]
                with option("gemm_tile", int(algo.split("-")[1]) if "-" in algo else 0):
                    ms, t = tf(lambda: gemm(A, Bm, M, N, K, ak, bk, M if ak else K, N if bk else K, C, N,
                                            algo=a), flops)
            cols.append(f"{algo} {ms:8.3f} ms {t:6.1f} TF/s")
        print(f"{name:22s} M={M:8d} N={N:5d} K={K:8d}  " + " | ".join(cols), flush=True)
        del A, Bm, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
