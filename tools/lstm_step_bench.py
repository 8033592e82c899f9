"""Microbenchmark of one wide-batch BiLSTM step (mvml_bilstm_wide_step_fwd / _bwd, both
directions in one launch) as a function of the live row count M, H = 384 (MVP's blstm_dim).
Prints the average launch time and the recurrent product's TF/s."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mvml-mpi_amd"), ROOT]
import torch  # noqa: E402
from mvml_gat._lib import call, lib, option, ptr, stream_ptr  # noqa: E402
from mvml_gat.functional import slot  # noqa: E402


def timed(fn, it=50):
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
    dev = torch.device("cuda", 0)
    H, G = 384, 1536
    MS = [int(m) for m in sys.argv[1].split(",")] if len(sys.argv) > 1 else [256, 1024, 2048, 2730, 4096, 8192]
    torch.manual_seed(0)
    W = [torch.randn(G, H, device=dev) * 0.05 for _ in range(2)]
    WT = [w.t().contiguous() for w in W]
    bias = [torch.randn(G, device=dev) * 0.1 for _ in range(4)]
    amx = torch.full((3,), 0x3F800000, dtype=torch.int32, device=dev)
    amx[1:] = torch.tensor([0.25], device=dev).view(torch.int32)
    st = stream_ptr(dev)
    for M in MS:
        h = torch.rand(M, 2 * H, device=dev) - 0.5
        gx = [torch.randn(M, G, device=dev) for _ in range(2)]
        cp = [torch.randn(M, H, device=dev) for _ in range(2)]
        c = [torch.empty(M, H, device=dev) for _ in range(2)]
        out = torch.empty(M, 2 * H, device=dev)
        act = [torch.empty(M, G, device=dev) for _ in range(2)]

        def fwd():
            call("mvml_bilstm_wide_step_fwd", M, M, H, H, ptr(h[:, :H]), ptr(h[:, H:]), 2 * H, ptr(W[0]),
                 ptr(W[1]), H, ptr(gx[0]), ptr(gx[1]), G, ptr(bias[0]), ptr(bias[1]), ptr(bias[2]),
                 ptr(bias[3]), ptr(cp[0]), ptr(cp[1]), ptr(c[0]), ptr(c[1]), ptr(out[:, :H]),
                 ptr(out[:, H:]), 2 * H, ptr(act[0]), ptr(act[1]), slot(amx, 0), slot(amx, 1),
                 slot(amx, 2), st)
        torch.sigmoid_(act[0])
        gn = [torch.randn(M, G, device=dev) * 0.1 for _ in range(2)]
        gout = torch.randn(M, 2 * H, device=dev)
        carry = [torch.randn(M, H, device=dev) for _ in range(4)]
        gg = [torch.empty(M, G, device=dev) for _ in range(2)]
        amg = torch.tensor([1.0, 1.0], device=dev).view(torch.int32)
        nws = int(lib().mvml_bilstm_wide_step_bwd_workspace_size(M, H))
        ws = torch.empty(nws, dtype=torch.uint8, device=dev)

        def bwd(R=M):
            call("mvml_bilstm_wide_step_bwd", M, M, R, R, H, ptr(gn[0]), ptr(gn[1]), ptr(WT[0]),
                 ptr(WT[1]), G, ptr(gout[:, :H]), ptr(gout[:, H:]), 2 * H, ptr(act[0]), ptr(act[0]),
                 ptr(c[0]), ptr(c[1]), ptr(cp[0]), ptr(cp[1]), ptr(carry[0]), ptr(carry[1]),
                 ptr(carry[2]), ptr(carry[3]), ptr(gg[0]), ptr(gg[1]), slot(amg, 0), slot(amg, 1),
                 slot(amx, 1), slot(amx, 2), ptr(ws), nws, st)
        fl = 2 * 2 * M * G * H
        outs = {}
        for tile in (256, 128):
            with option("lstm_tile", tile):
                tf_ = timed(fwd)
                tb = timed(bwd)
                tb0 = timed(lambda: bwd(0))
                fwd()
                bwd()
                torch.cuda.synchronize()
                outs[tile] = [t.clone() for t in (c[0], c[1], out, act[0], act[1], gg[0], gg[1], carry[2])]
            print(f"M={M:5d} tile {tile}  fwd {tf_ * 1e3:7.1f} us ({fl / tf_ / 1e9:6.1f} TF/s)  bwd {tb * 1e3:7.1f} us "
                  f"({fl / tb / 1e9:6.1f} TF/s; cell-only {tb0 * 1e3:6.1f} us)", flush=True)
        dif = max(float(((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item())
                  for a, b in zip(outs[128], outs[256]))
        print(f"M={M:5d} max rel diff 128 vs 256 tile: {dif:.2e}", flush=True)


if __name__ == "__main__":
    main()
