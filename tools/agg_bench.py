"""Microbenchmark of the fused GAT aggregation kernels, per layer, on the bench workload
(65,536 KEGG-like molecules): time per launch and algorithmic GB/s (formulas in
mvml_gat.functional.agg_fwd_bytes / agg_bwd_bytes), plus the Set2Set segment pass."""
import argparse
import contextlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mvml-mpi_amd"), ROOT]
import torch  # noqa: E402

from mvml_gat import _lib, synth  # noqa: E402
from mvml_gat._lib import call, ptr  # noqa: E402
from mvml_gat.functional import agg_bwd_bytes, agg_fwd_bytes  # noqa: E402


def timeit(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def bench_layer(a, g, N, E, st, L, H, F, mode, name):
    """One layer's aggregation forward (and backward) on seeded inputs; returns (out, attn, gY)."""
    torch.manual_seed(0)
    C = L.mvml_gat_proj_cols(H, F, int(mode == 1))
    ldy = (C + 63) // 64 * 64  # the product's 256-B row pitch
    Y = torch.randn((N, ldy), device="cuda") * 0.3
    bias = torch.randn(H * F, device="cuda") * 0.1
    elr = torch.randn((N, 2 * H), device="cuda")
    oc = F if mode == 1 else H * F
    out = torch.empty((N, oc), device="cuda")
    attn = torch.empty((E, H), device="cuda")
    # the output maxima the GNN path asks for (max |out| and per-row |max|)
    omx = torch.zeros(1, dtype=torch.int32, device="cuda")
    orow = torch.empty(N, dtype=torch.int32, device="cuda")
    f = lambda: call("mvml_gat_agg_fwd", N, ptr(g.node_groups), g.num_node_groups,
                     ptr(g.in_rowptr), ptr(g.in_src), ptr(Y), ldy, H, F, ptr(elr), ptr(bias), 0.2,
                     mode, ptr(out), ptr(attn), ptr(omx), ptr(orow), st)
    if a.no_fwd:
        f()
        ms = float("nan")
    else:
        ms = timeit(f)
    by = agg_fwd_bytes(N, E, H, F, oc, C - H * F)
    print(f"  agg_fwd {name:16s} {ms:7.3f} ms  {by / 1e9:6.2f} GB  {by / ms / 1e6:7.1f} GB/s", flush=True)
    if a.no_bwd:
        return out, attn, None
    g_out = torch.randn_like(out)
    ldg = (C + 2 * H + 63) // 64 * 64
    gY = torch.empty((N, ldg), device="cuda")
    wsz = L.mvml_gat_agg_bwd_workspace_size(E, H)
    ws = torch.empty(wsz, dtype=torch.uint8, device="cuda")
    gmx = torch.zeros(1, dtype=torch.int32, device="cuda")  # max |gY| (split-fp16 scale)
    grow = torch.empty(N, dtype=torch.int32, device="cuda") if mode == 1 else None  # layer 2 only
    b = lambda: call("mvml_gat_agg_bwd", N, ptr(g.node_groups), g.num_node_groups,
                     ptr(g.in_rowptr), ptr(g.in_src), ptr(g.out_rowptr), ptr(g.out_dst),
                     ptr(g.out_inslot), ptr(Y), ldy, ptr(elr), ptr(attn), ptr(out), ptr(g_out), H, F,
                     0.2, mode, ptr(gY), ldg, ptr(gmx), ptr(grow), ptr(ws), wsz, st)
    ms = timeit(b)
    by = agg_bwd_bytes(N, E, H, F, oc, mode)
    print(f"  agg_bwd {name:16s} {ms:7.3f} ms  {by / 1e9:6.2f} GB  {by / ms / 1e6:7.1f} GB/s", flush=True)
    return out, attn, gY[:, :C + 2 * H]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mols", type=int, default=65536)
    ap.add_argument("--config", default="3")
    ap.add_argument("--layers", default="01", help="which layers: 0 = L1 flatten+ELU, 1 = L2 mean, "
                    "2 = L1 flatten without ELU (the ELU-link backward)")
    ap.add_argument("--no-bwd", action="store_true")
    ap.add_argument("--no-fwd", action="store_true", help="time only the backward (forward runs once)")
    ap.add_argument("--ab", default="", help="option sets to compare on one box, e.g. "
                    "'dst_fwd=0,flat_src=0;dst_fwd=1,flat_src=2' (outputs checked equal across sets)")
    a = ap.parse_args()
    sets = [dict(kv.split("=") for kv in s.split(",") if kv) for s in a.ab.split(";")] if a.ab else [{}]
    sb = getattr(synth, f"config{a.config}")(a.mols)
    g = sb.to_graph().to("cuda")
    N, E = g.num_nodes(), g.num_edges()
    L = _lib.lib()
    st = _lib.stream_ptr()
    print(f"config{a.config}: {a.mols} molecules, N={N}, E={E}")
    # "2": layer 1 as the GNN runs it on large batches with the ELU link (mode 2: the next
    # layer's GEMM applied ELU', so the backward reads no `out`)
    layers = ((4, 192, 0, "L1 flatten+ELU"), (4, 384, 1, "L2 mean"), (4, 192, 2, "L1 flatten (link)"))
    for (H, F, mode, name) in [layers[int(i)] for i in a.layers]:
        ref = None
        for opts in sets:
            with contextlib.ExitStack() as es:
                for k, v in opts.items():
                    es.enter_context(_lib.option(k, int(v)))
                tag = ",".join(f"{k}={v}" for k, v in opts.items())
                res = bench_layer(a, g, N, E, st, L, H, F, mode, f"{name} [{tag}]")
            if ref is None:
                ref = res
            else:
                d = [(x - y).abs().max().item() if x is not None else 0.0 for x, y in zip(res, ref)]
                print(f"    [{tag}] max|diff| vs first set: out {d[0]:.3e} attn {d[1]:.3e} gY {d[2]:.3e}")
            del res
    D = 384
    X = torch.randn((N, D), device="cuda")
    B = g.batch_size
    qs = torch.randn((B, 2 * D), device="cuda")
    lse = torch.empty(B, device="cuda")
    f = lambda: call("mvml_set2set_seg_fwd", B, D, ptr(g.node_offsets), ptr(X), ptr(qs), 2 * D, ptr(lse), st)
    ms = timeit(f)
    by = 4 * (N * D + B * 3 * D)
    print(f"  set2set seg_fwd        {ms:7.3f} ms  {by / 1e9:6.2f} GB  {by / ms / 1e6:7.1f} GB/s")


if __name__ == "__main__":
    main()
