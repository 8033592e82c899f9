"""GraphNorm forward / backward (mvml_graphnorm_fwd / _bwd, model.py:93's PyG GraphNorm over the
Set2Set readout) at the bench's shape: 65,536 molecule rows x 768 columns in 1024 groups of 64.
ms per launch with HIP events and GB/s of the algorithmic bytes (forward: x read, y written;
backward: x and g_y read, g_x written, plus the [3][G][D] double partials and their reduction).

    python tools/graphnorm_bench.py [--B 65536] [--D 768] [--group 64] [--reps 20]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mvml-mpi_amd")]
from mvml_gat import _lib  # noqa: E402
from mvml_gat._lib import call, ptr, stream_ptr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--D", type=int, default=768)
    ap.add_argument("--group", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    B, D = a.B, a.D
    dev = "cuda"
    offs = torch.arange(0, B + a.group, a.group, dtype=torch.int64).clamp_(max=B).unique().to(dev)
    G = offs.numel() - 1
    gen = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn((B, D), device=dev, generator=gen)
    gy = torch.randn((B, D), device=dev, generator=gen)
    w, b, ms = (torch.randn(D, device=dev, generator=gen) for _ in range(3))
    y, gx = torch.empty_like(x), torch.empty_like(x)
    gw, gb, gms = (torch.empty(D, device=dev) for _ in range(3))
    L = _lib.lib()
    wp, wn = _lib.ws_ptr_size(L.mvml_graphnorm_bwd_workspace_size(G, D), dev)
    st = stream_ptr()

    def fwd():
        call("mvml_graphnorm_fwd", G, D, ptr(offs), ptr(x), ptr(w), ptr(b), ptr(ms), 1e-5, ptr(y), st)

    def bwd():
        call("mvml_graphnorm_bwd", G, D, ptr(offs), ptr(x), ptr(w), ptr(ms), 1e-5, ptr(gy), ptr(gx),
             ptr(gw), ptr(gb), ptr(gms), wp, wn, st)

    for name, fn, nbytes in (("fwd", fwd, 2 * B * D * 4),
                             ("bwd", bwd, 3 * B * D * 4 + 2 * 3 * G * D * 8)):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms_ = e0.elapsed_time(e1) / a.reps
        print(f"graphnorm {name}: B={B} D={D} G={G} {ms_ * 1e3:.1f} us/launch, "
              f"{nbytes / ms_ / 1e6:.0f} GB/s of {nbytes / 1e6:.0f} MB", flush=True)


if __name__ == "__main__":
    main()
