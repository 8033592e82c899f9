"""Fusion Conv2d(12, 12, 3) + ReLU kernels (mvml_conv3_fwd / _bwd, model.py:27, 69) at the bench's
65,536 molecules: ms per launch with HIP events.   python tools/conv_bench.py [--B 65536] [--reps 10]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mvml-mpi_amd")]
from mvml_gat import _lib  # noqa: E402
from mvml_gat._lib import call, ptr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    B, C, W = a.B, 12, 384
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    att = torch.randn((B, C, 3, W), device=dev, generator=g)
    w = torch.randn((C, C, 3, 3), device=dev, generator=g) * 0.1
    b = torch.randn((C,), device=dev, generator=g) * 0.1
    out = torch.empty((B, C, W - 2), device=dev)
    g_out = torch.randn((B, C, W - 2), device=dev, generator=g)
    g_in = torch.empty_like(att)
    gw, gb = torch.empty_like(w), torch.empty_like(b)
    L = _lib.lib()
    nws = L.mvml_conv3_bwd_workspace_size(B)
    ws = torch.empty(max(int(nws), 256), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def fwd():
        call("mvml_conv3_fwd", B, C, C, W, ptr(att), ptr(w), ptr(b), ptr(out), st)

    def bwd():
        call("mvml_conv3_bwd", B, C, C, W, ptr(att), ptr(w), ptr(out), ptr(g_out), ptr(g_in), ptr(gw),
             ptr(gb), ptr(ws), nws, st)

    for name, fn in (("conv3_fwd", fwd), ("conv3_bwd", bwd)):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.reps
        byts = 4 * B * (C * 3 * W + C * (W - 2)) if name == "conv3_fwd" else 4 * B * (2 * C * 3 * W + 2 * C * (W - 2))
        print(f"{name}: {ms:.3f} ms  {byts / ms / 1e6:.0f} GB/s (algorithmic bytes)")


if __name__ == "__main__":
    main()
