"""Fusion-head attention + Conv2d(12, 12, 3) + ReLU (model.py:62-69) at the bench's 65,536
molecules: the fused kernels (mvml_attn_conv_fwd / _bwd, the attention cube on chip) against the
separate launches they replace (mvml_token_attn_fold_fwd + mvml_conv3_fwd, mvml_conv3_bwd +
mvml_token_attn_fold_bwd), ms per launch with HIP events and GB/s of each one's algorithmic bytes.

    python tools/attn_conv_bench.py [--B 65536] [--reps 10] [--only fused|separate]
"""
import argparse
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mvml-mpi_amd")]
from mvml_gat import _lib  # noqa: E402
from mvml_gat._lib import call, ptr  # noqa: E402
from mvml_gat.fusion import attn_conv_bytes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", choices=["fused", "separate"], default=None)
    a = ap.parse_args()
    B, H, D = a.B, 12, 384
    HD = H * D
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    PV = torch.randn((3 * B, 2 * HD), device=dev, generator=g)
    Xn = torch.randn((3 * B, D), device=dev, generator=g)
    w = torch.randn((H, H, 3, 3), device=dev, generator=g) * 0.1
    b = torch.randn((H,), device=dev, generator=g) * 0.1
    P = torch.empty((B, H, 3, 3), device=dev)
    out = torch.empty((B, H, D - 2), device=dev)
    g_out = torch.randn((B, H, D - 2), device=dev, generator=g)
    gPV, gk = torch.empty_like(PV), torch.empty_like(Xn)
    gw, gb = torch.empty_like(w), torch.empty_like(b)
    amx = torch.zeros(1, dtype=torch.int32, device=dev)
    L = _lib.lib()
    nws = max(L.mvml_attn_conv_bwd_workspace_size(B), L.mvml_conv3_bwd_workspace_size(B))
    ws = torch.empty(max(int(nws), 256), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    sc = 1.0 / math.sqrt(D)
    att = gatt = None
    if a.only != "fused":
        att = torch.empty((B, H, 3, D), device=dev)
        gatt = torch.empty_like(att)

    def fused_fwd():
        call("mvml_attn_conv_fwd", B, H, D, ptr(PV), 2 * HD, ptr(Xn), D, sc, ptr(w), ptr(b), ptr(P),
             ptr(out), 0.0, 0, st)

    def fused_bwd():
        call("mvml_attn_conv_bwd", B, H, D, ptr(PV), 2 * HD, ptr(Xn), D, sc, ptr(P), ptr(w), ptr(out),
             ptr(g_out), 1.0, ptr(gPV), 2 * HD, ptr(gk), D, ptr(amx), None, ptr(gw), ptr(gb), ptr(ws), nws, st)

    def sep_fwd():
        call("mvml_token_attn_fold_fwd", B, H, D, ptr(PV), 2 * HD, ptr(Xn), D, sc, ptr(att), ptr(P), st)
        call("mvml_conv3_fwd", B, H, H, D, ptr(att), ptr(w), ptr(b), ptr(out), st)

    def sep_bwd():
        call("mvml_conv3_bwd", B, H, H, D, ptr(att), ptr(w), ptr(out), ptr(g_out), ptr(gatt), ptr(gw),
             ptr(gb), ptr(ws), nws, st)
        call("mvml_token_attn_fold_bwd", B, H, D, ptr(PV), 2 * HD, ptr(Xn), D, sc, ptr(P), ptr(gatt),
             ptr(gPV), 2 * HD, ptr(gk), D, ptr(amx), st)

    cube = 4 * B * H * 3 * D  # the attention cube: written + read (fwd), read + written + read (bwd)
    runs = []
    if a.only != "separate":
        runs += [("fused fwd", fused_fwd, attn_conv_bytes(B, H, D, False)),
                 ("fused bwd", fused_bwd, attn_conv_bytes(B, H, D, True))]
    if a.only != "fused":
        runs += [("separate fwd", sep_fwd, attn_conv_bytes(B, H, D, False) + 2 * cube),
                 ("separate bwd", sep_bwd, attn_conv_bytes(B, H, D, True) + 3 * cube)]
    for name, fn, byts in runs:
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.reps
        print(f"{name:13s}: {ms:7.3f} ms  {byts / 1e9:6.2f} GB algorithmic  {byts / ms / 1e6:6.0f} GB/s",
              flush=True)


if __name__ == "__main__":
    main()
