"""Where a small-K product goes wrong: per shape, the max row error and the pattern of bad
entries (row % 16, column % 64, column slab)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mvml-mpi_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from test_gpu_smallk import SHAPES, _inputs, _run  # noqa: E402

for shape in SHAPES + [(64, 64, 32), (16, 16, 32), (16, 16, 64), (16, 16, 76), (16, 64, 16), (32, 16, 48)]:
    M, N, K = shape
    A, B = _inputs(M, N, K, 3 + K)
    A = A.abs() if False else A
    ref = A.double() @ B.double().t()
    for il4 in (True, False):
        C = _run(A, B, M, N, K, il4=il4).double().cpu()
        den = ref.abs().max(1).values.clamp_min(1e-300).unsqueeze(1)
        e = (C - ref).abs() / den
        bad = e > 1e-5
        msg = f"{shape} il4={il4}: max {float(e.max()):.2e} bad {int(bad.sum())}/{bad.numel()}"
        if bad.any():
            r, c = bad.nonzero(as_tuple=True)
            msg += (f" rows%16 {sorted(set((r % 16).tolist()))[:16]} cols%64 {sorted(set((c % 64).tolist()))[:20]}"
                    f" slabs {sorted(set((c // 64).tolist()))[:10]} first {(int(r[0]), int(c[0]))}"
                    f" got {float(C[r[0], c[0]]):.4e} want {float(ref[r[0], c[0]]):.4e}")
        print(msg, flush=True)
