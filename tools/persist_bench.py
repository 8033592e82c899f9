"""A/B of the persistent tile loop (option gemm_persist = P workgroups looping over tiles) on the
per-row split-fp16 products of the GAT projection (layer 1: K = 76, memory-bound; layer 2)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mvml-mpi_amd"), ROOT]
import torch  # noqa: E402
from mvml_gat._lib import option  # noqa: E402
from mvml_gat.functional import absmax, absmax_rows, gemm, slot, split_il4  # noqa: E402
from gemm_bench import tf  # noqa: E402

N_ATOMS = 1754373
for name, M, N, K in (("L1 fwd K=76", N_ATOMS, 1544, 76), ("L2 fwd", N_ATOMS, 1928, 768)):
    A = torch.randn((M, K), device="cuda")
    B = torch.randn((N, K), device="cuda")
    C = torch.empty((M, N), device="cuda")
    mx = torch.zeros(2, dtype=torch.int32, device="cuda")
    absmax(B, N, K, K, mx, 1)
    rows = absmax_rows(A, M, K, K)
    img = split_il4(B, N, K, K, slot(mx, 1))
    cols = []
    for p in (0, 256, 512, 1024):
        with option("gemm_persist", p):
            ms, t = tf(lambda: gemm(A, B, M, N, K, 0, 0, K, K, C, N, amax=(None, slot(mx, 1)), arows=rows,
                                    bil4=img), 2 * M * N * K)
        cols.append(f"persist {p}: {ms:7.3f} ms {t:6.1f} TF/s")
    print(f"{name:14s} " + " | ".join(cols), flush=True)
    del A, B, C
    torch.cuda.empty_cache()
