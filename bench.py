#!/usr/bin/env python3
"""bench.py — molecules/sec of MVML-MPI's molecular-graph view (GNNModule, model.py:77-95)
forward + backward on MI355X, plus the aggregation kernel's fraction of the HBM roofline.

Step = one data-parallel training step of the graph view over a resident synthetic batch:
GNNModule forward (GAT 74->4x192 flatten+ELU -> 4x384 mean, Set2Set 6 iters x 3-layer LSTM,
GraphNorm per 64-molecule group, Linear+ReLU+Dropout), backward from a fixed upstream gradient
(what the multi-view fusion would send back), one flat RCCL all-reduce of the gradients when
N > 1, and the reference's Adam step (main.py:88, lr 1e-3, wd 1e-4).
Workload = BASELINE config 3 (KEGG-like molecule sizes, GraphNorm groups of 64 = config.py:21
batch size); each rank owns --mols-per-gpu molecules (weak scaling, no data-path collective).

    python bench.py [--gpus N --steps K --warmup W]     (N>1: launched by torch.distributed.run)

Prints ONE JSON line on rank 0 (the driver's contract); a per-kernel breakdown goes to stderr.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mvml-mpi_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "molecules/sec GAT-view fwd+bwd at 1/2/4/8 GPU; % HBM peak on aggregation"
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
FP32_MFMA_PEAK_TFS = 157.3  # f32-input MFMA = f32 vector peak (same table)
BF16_MFMA_PEAK_TFS = 2500.0  # dense bf16 MFMA peak (same table; the 5 PF figure is 2:1 sparse)
TIMED = ["mvml_gat_agg_fwd", "mvml_gat_agg_bwd", "mvml_gemm_f32", "mvml_gemm_f32x3", "mvml_gemm_bf16", "mvml_gat_proj_fwd", "mvml_set2set_seg_fwd",
         "mvml_set2set_seg_bwd", "mvml_lstm_cell_fwd", "mvml_lstm_cell_bwd", "mvml_set2set_gx",
         "mvml_graphnorm_fwd", "mvml_graphnorm_bwd", "mvml_colsum_f32", "mvml_gat_fold_weights",
         "mvml_gat_unfold_grads", "mvml_relu_bwd", "mvml_layernorm_fwd", "mvml_layernorm_bwd",
         "mvml_token_attn_fwd", "mvml_token_attn_bwd", "mvml_conv3_fwd", "mvml_conv3_bwd",
         "mvml_bce_logits"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mols-per-gpu", type=int, default=65536)
    ap.add_argument("--group-size", type=int, default=64)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timer", action="store_true")
    ap.add_argument("--with-fusion", action="store_true",
                    help="config 3 with its consumer: the MVP fusion head (SURVEY 8f-1) + BCE loss "
                         "on the GAT view's output (the SMILES / fingerprint views, out of scope, "
                         "are synthetic fixed embeddings)")
    ap.add_argument("--workload", choices=["config3", "config5"], default="config3",
                    help="config5 = BASELINE config 5 skewed-size stress (150-400 atoms + hubs of "
                         "in-degree 32-128; --mols-per-gpu defaults to 8192 there)")
    ap.add_argument("--proj-bf16", action="store_true",
                    help="BASELINE config 4: the GAT projection GEMMs (fc / res_fc, forward and "
                         "backward) on bf16 operands with fp32 accumulation (mvml_gemm_bf16); "
                         "everything else stays fp32")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def kernel_report(summary, elapsed_ms_per_step, steps):
    """Per entry point: calls/step, avg ms, share of the step, achieved GB/s or TFLOP/s."""
    rows = {}
    for name, ev in summary.items():
        if not ev:
            continue
        tot = sum(ms for ms, _ in ev)
        byts = sum((t or {}).get("bytes", 0) for _, t in ev)
        flops = sum((t or {}).get("flops", 0) for _, t in ev)
        rows[name] = dict(calls=len(ev) / steps, avg_ms=tot / len(ev), ms_per_step=tot / steps,
                          share=tot / steps / elapsed_ms_per_step,
                          gbs=(byts / (tot * 1e-3) / 1e9) if byts else None,
                          tfs=(flops / (tot * 1e-3) / 1e12) if flops else None)
    return rows


def roofline_entry(ev, kind):
    tot_ms = sum(ms for ms, _ in ev)
    if kind == "hbm":
        byts = sum(t["bytes"] for _, t in ev)
        ach = byts / (tot_ms * 1e-3) / 1e9
        return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "avg_launch_ms": round(tot_ms / len(ev), 4),
                "bytes_per_launch": int(byts / len(ev))}
    flops = sum(t["flops"] for _, t in ev)
    ach = flops / (tot_ms * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": round(ach, 2), "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
            "frac": round(ach / FP32_MFMA_PEAK_TFS, 4), "avg_launch_ms": round(tot_ms / len(ev), 4)}


def load_traffic(kernel):
    """HBM traffic per launch from the committed rocprofv3 PMC summary (profiles/), if any."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(kernel, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(seconds, group_size):
    """The CPU restatement of the reference path (oracle/, DGL semantics in plain PyTorch,
    fp32) timed on this host's cores on a bounded sample of the same workload."""
    from mvml_gat import synth
    from oracle.gnn_ref import GNNModuleRef
    from oracle.graph_ref import batch_ref
    n_mols = 4 * group_size
    sb = synth.config3(n_mols, seed=7)
    gd = batch_ref(sb.num_nodes, sb.src_local, sb.dst_local, sb.num_edges)
    gd["group_offsets"] = list(range(0, n_mols, group_size)) + [n_mols]
    torch.manual_seed(0)
    ref = GNNModuleRef(74, [192, 384], 0.5, 6, 3).train()
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-4)
    X = torch.as_tensor(sb.feats)
    up = torch.randn(n_mols, 384) * 1e-3

    def step():
        opt.zero_grad()
        ref(gd, X).backward(up)
        opt.step()

    step()
    t0, n = time.perf_counter(), 0
    while n < 2 or time.perf_counter() - t0 < seconds:
        step()
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n * n_mols / dt, 2), "unit": "molecules/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"{n} steps x {n_mols} KEGG-like molecules ({int(sb.num_nodes.sum())} atoms), "
                      f"fwd+bwd+Adam, oracle/gnn_ref.py GNNModuleRef in fp32 (DGL-semantics CPU "
                      f"restatement, not DGL)"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    import mvml_gat
    from mvml_gat import _lib, synth
    from mvml_gat.dist import FlatGradAllReduce
    mvml_gat.lib()

    t_gen = time.perf_counter()
    if args.workload == "config5":
        n5 = args.mols_per_gpu if args.mols_per_gpu != 65536 else 8192
        sb = synth.config5(n5, seed=1 + 1000 * args.seed + rank)
    else:
        sb = synth.config3(args.mols_per_gpu, seed=1000 * args.seed + rank)
    g = sb.to_graph(group_size=args.group_size).to(dev)
    feats = g.ndata["h"]
    N, E, B = g.num_nodes(), g.num_edges(), g.batch_size
    log(f"[rank {rank}] data: {B} molecules, {N} atoms, {E} edges ({time.perf_counter() - t_gen:.1f}s)")

    torch.manual_seed(args.seed)
    model = mvml_gat.GNNModule(74, [192, 384], 0.5, 6, 3,
                               proj_dtype=torch.bfloat16 if args.proj_bf16 else None).to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-4)
    reducer = FlatGradAllReduce(model.parameters(), average=True)
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    upstream = torch.randn((B, 384), device=dev, generator=gen) * 1e-3
    if args.with_fusion:
        fusion = mvml_gat.MVFusion(384, 12, 11, 0.5).to(dev).train()
        params = list(model.parameters()) + list(fusion.parameters())
        opt = torch.optim.Adam(params, lr=1e-3, weight_decay=1e-4)
        reducer = FlatGradAllReduce(params, average=True)
        smiles_x = torch.randn((B, 384), device=dev, generator=gen)
        fp_x = torch.randn((B, 384), device=dev, generator=gen)
        labels = (torch.rand((B, 11), device=dev, generator=gen) > 0.8).float()

    def step():
        opt.zero_grad(set_to_none=False)
        out = model(g, feats)
        if args.with_fusion:
            mvml_gat.bce_with_logits(fusion(smiles_x, out, fp_x), labels).backward()
        else:
            out.backward(upstream)
        reducer()
        opt.step()

    for _ in range(args.warmup):
        step()
    if not args.no_kernel_timer:
        _lib.timer.enable(TIMED)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    _lib.timer.disable()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms_per_step = elapsed * 1e3 / args.steps
    value = world * B * args.steps / elapsed

    roofline, extra = None, {}
    if not args.no_kernel_timer:
        summ = _lib.timer.summary()
        rows = kernel_report(summ, ms_per_step, args.steps)
        if rank == 0:
            for name, r in sorted(rows.items(), key=lambda kv: -kv[1]["ms_per_step"]):
                perf = (f"{r['gbs']:8.1f} GB/s" if r["gbs"] else "") + (f"{r['tfs']:7.2f} TF/s" if r["tfs"] else "")
                log(f"  {name:26s} {r['calls']:6.1f}/step avg {r['avg_ms']:8.3f} ms "
                    f"{r['ms_per_step']:8.2f} ms/step ({100 * r['share']:5.1f}%) {perf}")
        if summ.get("mvml_gat_agg_fwd"):
            roofline = roofline_entry(summ["mvml_gat_agg_fwd"], "hbm")
            roofline["kernel"] = "mvml_gat_agg_fwd (both GAT layers; fused edge-softmax + u_mul_e-sum)"
            roofline["traffic"] = load_traffic("gat_agg_fwd")
        if summ.get("mvml_gat_agg_bwd"):
            extra["roofline_agg_bwd"] = roofline_entry(summ["mvml_gat_agg_bwd"], "hbm")
            extra["roofline_agg_bwd"]["traffic"] = load_traffic("gat_agg_bwd")
        proj_ev = summ.get("mvml_gat_proj_fwd", [])
        gemm_ev = summ.get("mvml_gemm_f32", []) + summ.get("mvml_gemm_f32x3", []) + ([] if args.proj_bf16 else proj_ev)
        bf_ev = summ.get("mvml_gemm_bf16", []) + (proj_ev if args.proj_bf16 else [])
        if bf_ev:
            extra["roofline_gemm_bf16"] = roofline_entry(bf_ev, "mfma")
            extra["roofline_gemm_bf16"].update(
                peak=BF16_MFMA_PEAK_TFS, note="GAT projection GEMMs on bf16 operands (config 4)",
                frac=round(extra["roofline_gemm_bf16"]["achieved"] / BF16_MFMA_PEAK_TFS, 4))
        if gemm_ev:
            extra["roofline_gemm"] = roofline_entry(gemm_ev, "mfma")
            if summ.get("mvml_gemm_f32x3"):
                # split-bf16: 6 bf16 MFMA per fp32 multiply-add -> fp32-equivalent peak 2.5 PF / 6
                extra["roofline_gemm"].update(
                    peak=BF16_MFMA_PEAK_TFS / 6, note="fp32-accurate split-bf16 (x3) on bf16 MFMA; "
                    "achieved is fp32-equivalent TFLOP/s, peak = dense bf16 MFMA peak / 6")
                extra["roofline_gemm"]["frac"] = round(extra["roofline_gemm"]["achieved"] / (BF16_MFMA_PEAK_TFS / 6), 4)
        extra["kernel_ms_per_step"] = {k: round(v["ms_per_step"], 3) for k, v in rows.items()}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds, args.group_size)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "molecules/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16 projection, f32 elsewhere" if args.proj_bf16 else "f32",
            "data": "synthetic (seeded KEGG-like drug-like molecules, random-init weights)",
            "config": {"workload": ("BASELINE config 5 (150-400-atom molecules with 1-4 hubs of in-degree "
                                    "32-128): " if args.workload == "config5" else "BASELINE config 3: ") +
                                   "GNNModule (GAT [192,384] x4 heads, Set2Set 6x3, "
                                   "GraphNorm, fc) fwd+bwd+Adam over KEGG-like molecules"
                                   + (" + MVP fusion head (12-head 3-token attention, Conv2d, MLP) "
                                      "+ BCEWithLogits" if args.with_fusion else
                                      " (fixed upstream gradient at the view output)"),
                       "mols_per_gpu": B, "atoms_per_gpu": N, "edges_per_gpu": E,
                       "graphnorm_group": args.group_size, "parallelism": f"dp{world}",
                       "projection": "bf16 operands, fp32 accumulate (config 4)" if args.proj_bf16
                       else "fp32-accurate split-bf16 x3"},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
