"""Yardstick for the split-fp16 GEMM: hipBLASLt (torch.matmul) fp16 / bf16 with fp32 accumulation
on the step's big shapes, at K and at K' = 3K (the pre-split formulation [A_h | A_h | A_l] x
[B_h ; B_l ; B_h] of the same fp32-accurate product).  Random data (DVFS: zeros clock higher).
Prints TF/s of the library GEMM itself and the fp32-equivalent rate of the 3K form."""
import torch

N_ATOMS, B = 1754373, 65536
SHAPES = [("L2 fwd", N_ATOMS, 1928, 768), ("L2 dX", N_ATOMS, 768, 1928),
          ("L2 dW", 1928, 768, N_ATOMS), ("LSTM gates", B, 1536, 768)]


def timed(fn, it=8):
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
    torch.manual_seed(0)
    for name, M, N, K in SHAPES:
        for dt in (torch.float16, torch.bfloat16):
            for kmul in (1, 3):
                Kx = K * kmul
                A = torch.randn(M, Kx, device="cuda", dtype=dt)
                Bm = torch.randn(Kx, N, device="cuda", dtype=dt)
                C = torch.empty(M, N, device="cuda", dtype=dt)  # fp32 accumulate, 16-bit output
                if name == "L2 dW":  # K = atoms: A^T-shaped operands as in the step
                    A = torch.randn(Kx, M, device="cuda", dtype=dt).t()
                ms = timed(lambda: torch.matmul(A, Bm, out=C))
                fl = 2 * M * N * Kx
                print(f"{name:10s} {str(dt):15s} K={Kx:8d} {ms:8.3f} ms {fl / ms / 1e9:8.1f} TF/s"
                      + (f"  fp32-equiv {2 * M * N * K / ms / 1e9:6.1f} TF/s" if kmul == 3 else ""), flush=True)
                del A, Bm, C
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
