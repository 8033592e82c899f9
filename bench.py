#!/usr/bin/env python3
"""bench.py — molecules/sec of MVML-MPI's molecular-graph view (GNNModule, model.py:77-95)
forward + backward + the multi-view fusion head on MI355X, plus the aggregation kernel's
fraction of the HBM roofline.

Workload (default) = BASELINE config 3 as written: ONE global set of 1,000,000 synthetic
KEGG-like molecules (mvml_gat.synth.Config3Set), sharded over the ranks in whole 64-molecule
GraphNorm groups (the reference's mini-batches, config.py:21 / main.py:79-81 / model.py:93)
balanced by edges (mvml_gat.dist.shard_groups), resident in HBM and streamed through steps of
--mols-per-step molecules per GPU.  Step = one data-parallel training step of model.py:51-72
restricted to the graph view: device collation of the step's molecules (dataset.py:52-54:
dgl.batch + CSR + node-group plan, mvml_build_csr) -> GNNModule forward -> MVFusion (shared LayerNorm, 12-head 3-token
attention, Conv2d, MLP) -> BCEWithLogits (main.py:91) -> backward -> one flat RCCL all-reduce of
the gradients (N > 1) -> Adam (main.py:88).  The SMILES and fingerprint view embeddings that
the fusion also consumes are fixed synthetic tensors (their views are not this workload).
After the timed steps: a view-only figure (fixed upstream gradient, the round-1 headline) and
one inference pass over the rank's whole shard whose (B_shard, 384) embeddings are all-gathered
into the full 1M x 384 matrix (north_star's final embedding gather).

    python bench.py [--gpus N --steps K --warmup W]

--gpus N without WORLD_SIZE in the environment starts N ranks itself (torch.distributed.run as
a child process, before any GPU call); rank 0 prints the ONE JSON line (the driver's contract),
a per-kernel breakdown goes to stderr.  --workload config5 = the skewed-size stress (per-rank
sets, weak scaling).  --dry-run = CPU/gloo rehearsal of the launcher, sharding, all-reduce and
gather plumbing with a trivial stand-in model (never a measurement: no HIP code runs).
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
SMALLK_MAX_K = 96  # mvml_gemm_f16x2_rows products at K <= this run gemm_smallk_kernel (option smallk)
TIMED = ["mvml_gat_agg_fwd", "mvml_gat_agg_bwd", "mvml_gemm_f32", "mvml_gemm_f32x3", "mvml_gemm_bf16", "mvml_gat_proj_fwd", "mvml_set2set_seg_fwd",
         "mvml_set2set_seg_bwd", "mvml_lstm_cell_fwd", "mvml_lstm_cell_bwd", "mvml_set2set_gx",
         "mvml_graphnorm_fwd", "mvml_graphnorm_bwd", "mvml_colsum_f32", "mvml_gat_fold_weights",
         "mvml_gat_unfold_grads", "mvml_relu_bwd", "mvml_layernorm_fwd", "mvml_layernorm_bwd",
         "mvml_token_attn_fwd", "mvml_token_attn_bwd", "mvml_token_attn_fold_fwd",
         "mvml_token_attn_fold_bwd", "mvml_gemm_f32x3_batched", "mvml_conv3_fwd", "mvml_conv3_bwd",
         "mvml_bce_logits", "mvml_gat_attn_grad", "mvml_bilstm_seq_fwd", "mvml_bilstm_seq_bwd", "mvml_bilstm_wide_fwd", "mvml_bilstm_wide_bwd",
         "mvml_lstm_gates_cell_fwd", "mvml_gemm_f16x2", "mvml_gemm_f16x2_amax", "mvml_gemm_f16x2_amax_colsum",
         "mvml_absmax_f32",
         "mvml_gemm_f16x2_bsplit", "mvml_attn_conv_fwd", "mvml_attn_conv_bwd",
         "mvml_bilstm_wide_step_fwd", "mvml_bilstm_wide_step_bwd", "mvml_bilstm_pack_rows",
         "mvml_bilstm_gather_rows", "mvml_bilstm_token_grad", "mvml_bilstm_select_last",
         "mvml_bilstm_token_grad_packed", "mvml_bilstm_packed_tokens", "mvml_gemm_f16x2_rows",
         "mvml_absmax_rows_f32", "mvml_segment_max_bits",
         "mvml_gemm_f16x2_ex", "mvml_gemm_f16x2_batched",
         "mvml_split_f16x2_il4", "mvml_build_csr", "mvml_build_node_groups"]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=["config3", "config5", "mvp"], default="config3",
                    help="mvp = BASELINE config 4: the whole MVP model (SMILES BiLSTM + graph view + "
                         "fingerprint MLP + fusion) DP training step on shards of the config-3 set")
    ap.add_argument("--total-mols", type=int, default=1_000_000,
                    help="config 3: size of the ONE global molecule set sharded over the ranks")
    ap.add_argument("--mols-per-step", type=int, default=None,
                    help="molecules per GPU per step (whole GraphNorm groups); default 65536 for "
                         "config3, 8192 for config5 / mvp")
    ap.add_argument("--group-size", type=int, default=64)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--view-only-steps", type=int, default=3,
                    help="extra steps timed without the fusion head (fixed upstream gradient)")
    ap.add_argument("--no-inference", action="store_true",
                    help="skip the inference pass + embedding all-gather over the whole shard")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timer", action="store_true")
    ap.add_argument("--proj-bf16", action="store_true",
                    help="BASELINE config 4: the GAT projection GEMMs (fc / res_fc, forward and "
                         "backward) on bf16 operands with fp32 accumulation (mvml_gemm_bf16)")
    ap.add_argument("--no-view-overlap", action="store_true",
                    help="mvp workload: run the SMILES view after the graph view on one stream "
                         "(default: on a side stream beside it, mvml_gat.mvp.OVERLAP_VIEWS)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo plumbing rehearsal with a stand-in model (no measurement)")
    return ap.parse_args(argv)


def mols_per_step(args):
    """The per-GPU step size the workload runs with (explicit, or the workload's default)."""
    if args.mols_per_step is not None:
        return args.mols_per_step
    return 65536 if args.workload == "config3" else 8192


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ----------------------------------------------------------------------------- reporting
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


def gemm_shape_report(ev, steps):
    """MVML_GEMM_SHAPES=1: the GEMM time per (M, N, K, A K-major, B K-major), to stderr."""
    by = {}
    for ms, t in ev:
        k = (t or {}).get("shape")
        c, tot, fl = by.get(k, (0, 0.0, 0))
        by[k] = (c + 1, tot + ms, fl + (t or {}).get("flops", 0))
    for k, (c, tot, fl) in sorted(by.items(), key=lambda x: -x[1][1]):
        log(f"  gemm {str(k):40s} {c / steps:5.1f}/step {tot / steps:8.3f} ms/step "
            f"{fl / (tot * 1e-3) / 1e12:7.1f} TF/s")


def full_batch_bytes(ev):
    """Algorithmic bytes per launch on a FULL step batch: per layer tag the largest launch (the
    set's short last batch, if timed, is smaller), averaged over the layers — the batch the PMC
    traffic in profiles/pmc_traffic.json was collected on."""
    by = {}
    for _, t in ev:
        by[t.get("layer")] = max(by.get(t.get("layer"), 0), t["bytes"])
    return sum(by.values()) / len(by)


def roofline_entry(ev, kind, traffic_full=None):
    """traffic_full: PMC HBM bytes per launch on a full step batch (or None).  The line reports
    the traffic SCALED to the timed launches' batch mix (traffic_full x bytes_per_launch /
    full-batch bytes), so traffic / bytes_per_launch compares like with like; the full-batch
    pair is reported beside it."""
    tot_ms = sum(ms for ms, _ in ev)
    if kind == "hbm":
        byts = sum(t["bytes"] for _, t in ev)
        ach = byts / (tot_ms * 1e-3) / 1e9
        avg = byts / len(ev)
        full = full_batch_bytes(ev)
        r = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(ach / HBM_PEAK_GBS, 4), "avg_launch_ms": round(tot_ms / len(ev), 4),
             "bytes_per_launch": int(avg), "traffic": None}
        if traffic_full:
            r.update(traffic=int(traffic_full * avg / full), full_batch_bytes_per_launch=int(full),
                     full_batch_traffic_per_launch=int(traffic_full),
                     traffic_over_algorithmic=round(traffic_full / full, 4))
        return r
    flops = sum(t["flops"] for _, t in ev)
    ach = flops / (tot_ms * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": round(ach, 2), "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
            "frac": round(ach / FP32_MFMA_PEAK_TFS, 4), "avg_launch_ms": round(tot_ms / len(ev), 4)}


def load_traffic(workload_key, entry):
    """HBM traffic per launch of `entry` from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json), ONLY if it was profiled on this exact workload; else None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    return d.get(workload_key, {}).get(entry, {}).get("hbm_bytes_per_launch")


ALLOC_KEYS = ("num_alloc_retries", "num_device_alloc", "num_device_free", "num_sync_all_streams",
              "num_ooms")


def alloc_stats(args):
    """Caching-allocator counters (device mallocs / frees / retries) and the reserved bytes: a
    step that misses the cache pays hipMalloc, and a retry frees every cached block (a device
    synchronisation) — both show as time outside every kernel."""
    if args.dry_run:
        return {}
    s = torch.cuda.memory_stats()
    out = {k: int(s.get(k, 0)) for k in ALLOC_KEYS}
    out["reserved_bytes"] = int(s.get("reserved_bytes.all.current", 0))
    out["peak_allocated_bytes"] = int(s.get("allocated_bytes.all.peak", 0))
    return out


# ----------------------------------------------------------------------------- CPU baseline
def usable_cores():
    """CPUs this process may actually run on: the affinity mask, capped by a cgroup v2 quota
    (on the GPU box os.cpu_count() reports the whole machine, not this job's share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds, group_size, with_fusion):
    """The CPU restatement of the reference path (oracle/: DGL / PyG semantics in plain PyTorch,
    fp32 — NOT DGL, which cannot be installed here) timed on this host's cores on a bounded
    sample of the same workload (BASELINE.md plan: all usable cores, 3 warm-ups, median of >= 10
    timed steps over whole 64-molecule groups)."""
    from mvml_gat import synth
    from oracle.fusion_ref import MVFusionRef, bce_logits_ref
    from oracle.gnn_ref import GNNModuleRef
    from oracle.graph_ref import batch_ref
    cores = usable_cores()
    torch.set_num_threads(cores)
    n_mols = 4 * group_size
    sb = synth.Config3Set(n_mols, seed=7).molecules(0, n_mols)
    gd = batch_ref(sb.num_nodes, sb.src_local, sb.dst_local, sb.num_edges)
    gd["group_offsets"] = list(range(0, n_mols, group_size)) + [n_mols]
    torch.manual_seed(0)
    ref = GNNModuleRef(74, [192, 384], 0.5, 6, 3).train()
    params = list(ref.parameters())
    fus = None
    if with_fusion:
        fus = MVFusionRef(384, 12, 11, 0.5).train()
        params += list(fus.parameters())
    opt = torch.optim.Adam(params, lr=1e-3, weight_decay=1e-4)
    X = torch.as_tensor(sb.feats)
    g = torch.Generator().manual_seed(1)
    up = torch.randn(n_mols, 384, generator=g) * 1e-3
    sx, fx = torch.randn(n_mols, 384, generator=g), torch.randn(n_mols, 384, generator=g)
    labels = (torch.rand(n_mols, 11, generator=g) > 0.8).float()

    def step():
        opt.zero_grad()
        out = ref(gd, X)
        if fus is not None:
            bce_logits_ref(fus(sx, out, fx), labels).backward()
        else:
            out.backward(up)
        opt.step()

    for _ in range(3):
        step()
    times = []
    t_end = time.perf_counter() + seconds
    while len(times) < 10 or time.perf_counter() < t_end:
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
        if len(times) >= 200:
            break
    med = float(np.median(times))
    return {"value": round(n_mols / med, 2), "unit": "molecules/s", "cores": cores,
            "kind": "port", "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
            "sample": f"median of {len(times)} steps (3 warm-ups) x {n_mols} KEGG-like molecules "
                      f"({int(sb.num_nodes.sum())} atoms, {n_mols // group_size} GraphNorm groups of "
                      f"{group_size}), fwd+bwd{' + MVFusion + BCE' if with_fusion else ''} + Adam, "
                      "oracle/gnn_ref.py + oracle/fusion_ref.py in fp32 (DGL-semantics CPU "
                      "restatement, not DGL)"}


# ----------------------------------------------------------------------------- data
class Batch:
    """One step's resident inputs: the device-built graph + features, and the fusion head's
    other two view embeddings / labels (seeded by the batch's first global molecule index, so
    they do not depend on how the set was sharded).  mvp: the SMILES token batch (synthetic
    characters, ~1.8 per atom like KEGG's 50 characters for 28 atoms) and real 2513-value
    fingerprints (the restated fingerprints of the 420 KEGG test-split molecules,
    fingerprints.kegg_pool(), cycled by global molecule index) instead of the two fixed view
    embeddings."""

    def __init__(self, sb, first_mol, group_size, dev, with_fusion, mvp=False):
        self.g = sb.to_graph(group_size=group_size).to(dev)
        self.feats = self.g.ndata["h"]
        self.B, self.N, self.E = self.g.batch_size, self.g.num_nodes(), self.g.num_edges()
        if with_fusion:
            gen = torch.Generator(device=dev).manual_seed(1234 + first_mol)
            self.smiles_x = torch.randn((self.B, 384), device=dev, generator=gen)
            self.fp_x = torch.randn((self.B, 384), device=dev, generator=gen)
            self.labels = (torch.rand((self.B, 11), device=dev, generator=gen) > 0.8).float()
        if mvp:
            rng = np.random.default_rng([first_mol, 77])
            lens = np.clip(np.rint(1.8 * sb.num_nodes * rng.uniform(0.8, 1.2, self.B)), 5, 462).astype(np.int64)
            T = int(lens.max())
            tok = rng.integers(2, 39, size=(self.B, T)).astype(np.float32)
            tok[np.arange(T)[None, :] >= lens[:, None]] = 0.0
            self.smiles = {"smiles": torch.from_numpy(tok).to(dev), "seq_len": lens.tolist()}
            pool = _fp_pool()
            self.fp = torch.from_numpy(pool[(first_mol + np.arange(self.B)) % len(pool)]).to(dev)


_POOL = []


def _fp_pool():
    if not _POOL:
        from mvml_gat.fingerprints import kegg_pool
        _POOL.append(kegg_pool())
    return _POOL[0]


def build_batches(args, rank, world, dev, with_fusion):
    from mvml_gat import dist as mdist
    from mvml_gat import synth
    gs = args.group_size
    if args.workload == "mvp":
        gset = synth.Config3Set(args.total_mols, seed=args.seed)
        g0, g1 = mdist.shard_groups(gset.group_costs(gs), world, rank)
        lo, hi = g0 * gs, min(g1 * gs, args.total_mols)
        per = max(gs, mols_per_step(args) // gs * gs)
        hi = min(hi, lo + 16 * per)  # at most 16 resident steps per rank
        return ([Batch(gset.molecules(m, min(hi, m + per)), m, gs, dev, True, mvp=True)
                 for m in range(lo, hi, per)], (lo, hi))
    if args.workload == "config3":
        gset = synth.Config3Set(args.total_mols, seed=args.seed)
        g0, g1 = mdist.shard_groups(gset.group_costs(gs), world, rank)
        lo, hi = g0 * gs, min(g1 * gs, args.total_mols)
        per = max(gs, mols_per_step(args) // gs * gs)
        out = []
        for m in range(lo, hi, per):
            sb = gset.molecules(m, min(hi, m + per))
            out.append(Batch(sb, m, gs, dev, with_fusion))
        return out, (lo, hi)
    n5 = mols_per_step(args)
    sb = synth.config5(n5, seed=1 + 1000 * args.seed + rank)
    return [Batch(sb, rank * n5, gs, dev, with_fusion)], (rank * n5, (rank + 1) * n5)


# ----------------------------------------------------------------------------- dry-run stand-in
class _PlumbingStandIn(torch.nn.Module):
    """--dry-run only: a trivial CPU model with the view's call signature (segment mean of the
    atom features -> Linear), so the launcher / sharding / all-reduce / all-gather plumbing can
    be rehearsed on gloo without a GPU.  Never used for any reported number."""

    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(74, 384)
        self.head = torch.nn.Linear(3 * 384, 11)

    def view(self, g, feats):
        B = g.batch_size
        gid = torch.repeat_interleave(torch.arange(B), torch.as_tensor(g._bnn))
        s = torch.zeros(B, 74).index_add(0, gid, feats)
        return self.lin(s / torch.as_tensor(g._bnn).clamp(min=1).unsqueeze(1).float())

    def forward(self, g, feats):
        return self.view(g, feats)

    def fuse(self, sx, gx, fx):
        return self.head(torch.cat([sx, gx, fx], 1))


# ----------------------------------------------------------------------------- worker
def run(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        # MVML_BENCH_ONE_DEVICE=1 + MVML_BENCH_BACKEND=gloo: a rehearsal of the N-rank path on a
        # one-GPU box (every rank on cuda:0; RCCL refuses two ranks per device) — the driver's
        # N-GPU runs use neither (one rank per GPU over RCCL)
        one_dev = os.environ.get("MVML_BENCH_ONE_DEVICE") == "1"
        torch.cuda.set_device(0 if one_dev else local_rank)
        dev = torch.device("cuda", 0 if one_dev else local_rank)
        if world > 1:
            backend = os.environ.get("MVML_BENCH_BACKEND", "nccl")
            if backend == "nccl":
                dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
            else:
                dist.init_process_group(backend, rank=rank, world_size=world)

    from mvml_gat.dist import EmbeddingAllGather, FlatGradAllReduce
    from mvml_gat import functional as F
    if not args.dry_run:
        import mvml_gat
        from mvml_gat import _lib
        mvml_gat.lib()

    def sync():
        if not args.dry_run:
            torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    t_gen = time.perf_counter()
    if args.dry_run:
        from mvml_gat import dist as mdist
        from mvml_gat import synth
        gs = args.group_size
        gset = synth.Config3Set(args.total_mols, seed=args.seed)
        g0, g1 = mdist.shard_groups(gset.group_costs(gs), world, rank)
        lo, hi = g0 * gs, min(g1 * gs, args.total_mols)
        batches = []
        for m in range(lo, hi, mols_per_step(args)):
            sb = gset.molecules(m, min(hi, m + mols_per_step(args)))
            b = Batch.__new__(Batch)
            b.g = sb.to_graph(group_size=gs)
            b.feats = torch.as_tensor(sb.feats)
            b.B, b.N, b.E = b.g.batch_size, b.g.num_nodes(), b.g.num_edges()
            gen = torch.Generator().manual_seed(1234 + m)
            b.smiles_x, b.fp_x = torch.randn((b.B, 384), generator=gen), torch.randn((b.B, 384), generator=gen)
            b.labels = (torch.rand((b.B, 11), generator=gen) > 0.8).float()
            batches.append(b)
        shard = (lo, hi)
    else:
        batches, shard = build_batches(args, rank, world, dev, with_fusion=True)
    n_local = sum(b.B for b in batches)
    log(f"[rank {rank}] shard molecules [{shard[0]}, {shard[1]}): {len(batches)} batches, "
        f"{n_local} molecules, {sum(b.N for b in batches)} atoms, {sum(b.E for b in batches)} edges "
        f"({time.perf_counter() - t_gen:.1f}s)")

    torch.manual_seed(args.seed)
    mvp = args.workload == "mvp"
    if args.dry_run:
        model = _PlumbingStandIn()
        fusion = None
        params = list(model.parameters())
    elif mvp:
        import mvml_gat.mvp as mvp_mod
        from mvml_gat.mvp import MVP
        mvp_mod.OVERLAP_VIEWS = not args.no_view_overlap
        # main.py:85-87 with config.py defaults: hidden [192, 384], rnn 128 / 384 x 2, fp 512,
        # 12 fusion heads, dropout 0.5
        full = MVP(11, 74, [192, 384], 6, 3, 128, 384, 2, 512, 12, 0.5,
                   proj_dtype=torch.bfloat16 if args.proj_bf16 else None).to(dev).train()
        model, fusion = full.gnn, None
        # every parameter, as main.py:88 passes model.parameters(): the never-used LayerNorms
        # (model.py:42, 120) keep grad None through the reducer, so Adam skips them
        params = list(full.parameters())
    else:
        model = mvml_gat.GNNModule(74, [192, 384], 0.5, 6, 3,
                                   proj_dtype=torch.bfloat16 if args.proj_bf16 else None).to(dev).train()
        fusion = mvml_gat.MVFusion(384, 12, 11, 0.5).to(dev).train()
        params = list(model.parameters()) + list(fusion.parameters())
    # main.py:88's Adam (lr 1e-3, weight decay 1e-4): by default mvml_gat.FlatAdam — the gradient
    # gather, the ONE all-reduce of [gradients | presence flags] and the update as HIP kernels
    # over flat buffers, no host synchronisation (MVML_BENCH_ADAM=fused / foreach: torch's Adam
    # behind FlatGradAllReduce, which reads the reduced presence flags back every step)
    adam_kind = "torch" if args.dry_run else os.environ.get("MVML_BENCH_ADAM", "flat")
    if adam_kind == "flat":
        from mvml_gat.optim import FlatAdam
        opt = FlatAdam(params, lr=1e-3, weight_decay=1e-4, average=True)
        reducer = lambda: None  # noqa: E731  (the all-reduce is inside FlatAdam.step)
    else:
        opt = torch.optim.Adam(params, lr=1e-3, weight_decay=1e-4,
                               **({"fused": True} if adam_kind == "fused" else {}))
        reducer = FlatGradAllReduce(params, average=True)

    one = torch.ones((), device=dev)  # dL/dL, made once (backward() would fill one every step)

    def step(b, fused=True):
        opt.zero_grad(set_to_none=False)
        if not args.dry_run:
            # the collation (dgl.batch + CSR + node-group plan) on the device, every step, as the
            # reference's DataLoader collates every batch (dataset.py:52-54)
            b.g.recollate()
        if mvp and fused:
            mvml_gat.bce_with_logits(full(b.smiles, b.g, b.feats, b.fp), b.labels).backward(one)
            mvp_mod.join_side_stream(dev)
            reducer()
            opt.step()
            return
        out = model(b.g, b.feats)
        if args.dry_run:
            torch.nn.functional.binary_cross_entropy_with_logits(
                model.fuse(b.smiles_x, out, b.fp_x), b.labels).backward()
        elif fused:
            mvml_gat.bce_with_logits(fusion(b.smiles_x, out, b.fp_x), b.labels).backward(one)
        else:
            out.backward(b.upstream)
        reducer()
        opt.step()

    nb = len(batches)
    # the first warm-up step runs the batch with the most edges, so the caching allocator sizes
    # its blocks for the largest step once (no device malloc inside the timed region)
    big = max(range(nb), key=lambda j: (batches[j].E, batches[j].N))
    for i in range(args.warmup):
        step(batches[big] if i == 0 else batches[i % nb])
    timer_on = not args.no_kernel_timer and not args.dry_run
    if timer_on:
        _lib.timer.enable(TIMED)
    if adam_kind == "flat":
        opt.allreduce_events = []  # the timed steps' all-reduces only
    barrier()
    sync()
    mem0 = alloc_stats(args)
    step_ev = []
    t0 = time.perf_counter()
    mols = 0
    for i in range(args.steps):
        b = batches[(args.warmup + i) % nb]
        if not args.dry_run:
            step_ev.append(torch.cuda.Event(enable_timing=True))
            step_ev[-1].record()
        step(b)
        mols += b.B
    if not args.dry_run:
        step_ev.append(torch.cuda.Event(enable_timing=True))
        step_ev[-1].record()
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    mem1 = alloc_stats(args)
    if timer_on:
        _lib.timer.disable()
    step_ms = [round(a.elapsed_time(b), 3) for a, b in zip(step_ev[:-1], step_ev[1:])]

    def reduce_max(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.item()

    def reduce_sum(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.item()

    elapsed = reduce_max(elapsed)
    total_mols = reduce_sum(mols)
    ms_per_step = elapsed * 1e3 / max(args.steps, 1)
    value = total_mols / elapsed if elapsed > 0 else 0.0

    roofline, extra = None, {}
    if adam_kind == "flat" and world > 1:
        # HIP events around each timed step's one all-reduce of [gradients | presence flags]
        ar = opt.allreduce_ms()
        extra["allreduce_ms"] = {"rank0": round(ar, 4), "max_over_ranks": round(reduce_max(ar), 4),
                                 "bytes": int(opt.gbuf.numel() * 4),
                                 "what": "mean per-step duration of the gradient all-reduce (HIP events on "
                                         "the step's stream), this rank and the slowest rank"}
    extra["optimizer"] = ("FlatAdam (mvml_grad_gather + one all-reduce + mvml_adam_flat)" if adam_kind == "flat"
                          else f"torch.optim.Adam ({adam_kind}) + FlatGradAllReduce")
    mps = mols_per_step(args)  # the per-step molecule count the workload actually used
    wkey = f"{args.workload}/mols_per_step={mps}" + ("/proj_bf16" if args.proj_bf16 else "")
    if timer_on:
        summ = _lib.timer.summary()
        rows = kernel_report(summ, ms_per_step, args.steps)
        if os.environ.get("MVML_GEMM_SHAPES") and rank == 0:
            gemm_shape_report(summ.get("mvml_gemm_f32x3", []) + summ.get("mvml_gemm_f32x3_batched", [])
                              + summ.get("mvml_gemm_f16x2", []) + summ.get("mvml_gemm_f16x2_amax", [])
                              + summ.get("mvml_gemm_f16x2_amax_colsum", [])
                              + summ.get("mvml_gemm_f16x2_rows", [])
                              + summ.get("mvml_gemm_f16x2_bsplit", [])
                              + summ.get("mvml_gemm_f16x2_ex", []) + summ.get("mvml_gemm_f16x2_batched", [])
                              + summ.get("mvml_gemm_f16x2_planes", [])
                              + summ.get("mvml_lstm_gates_cell_fwd", [])
                              + summ.get("mvml_gat_proj_fwd", []), args.steps)
        if rank == 0:
            for name, r in sorted(rows.items(), key=lambda kv: -kv[1]["ms_per_step"]):
                perf = (f"{r['gbs']:8.1f} GB/s" if r["gbs"] else "") + (f"{r['tfs']:7.2f} TF/s" if r["tfs"] else "")
                log(f"  {name:26s} {r['calls']:6.1f}/step avg {r['avg_ms']:8.3f} ms "
                    f"{r['ms_per_step']:8.2f} ms/step ({100 * r['share']:5.1f}%) {perf}")
        if summ.get("mvml_gat_agg_fwd"):
            roofline = roofline_entry(summ["mvml_gat_agg_fwd"], "hbm", load_traffic(wkey, "gat_agg_fwd"))
            roofline["kernel"] = "mvml_gat_agg_fwd (both GAT layers; edge-softmax fused into the u_mul_e-sum aggregation)"
            roofline["traffic_profile"] = wkey if roofline["traffic"] else None
        if summ.get("mvml_gat_agg_bwd"):
            extra["roofline_agg_bwd"] = roofline_entry(summ["mvml_gat_agg_bwd"], "hbm",
                                                       load_traffic(wkey, "gat_agg_bwd"))
        proj_ev = summ.get("mvml_gat_proj_fwd", [])
        # the GAT projection at small K (K <= 96: layer 1's, on the wave-per-64-column memory
        # kernel gemm_smallk_kernel) is an HBM roofline of its own, not MFMA work
        rows_ev = summ.get("mvml_gemm_f16x2_rows", [])
        # (the path the library actually took, not the shape: mvml_gemm_rows_smallk)
        sk_ev = [e for e in rows_ev if (e[1] or {}).get("role") == "gat_proj" and e[1].get("path") == "smallk"]
        rows_ev = [e for e in rows_ev if e not in sk_ev]
        if sk_ev:
            extra["roofline_proj_l1"] = roofline_entry(sk_ev, "hbm", load_traffic(wkey, "gemm_smallk"))
            extra["roofline_proj_l1"]["kernel"] = (
                "mvml_gemm_f16x2_rows at K <= 96 (layer-1 projection X[N, 76] Wcat[1544, 76]^T, "
                "gemm_smallk_kernel); bytes = A, B and C once")
        # layer 1's weight gradient (N = 76 columns: gY^T X over every atom, split-K) streams the
        # N x 1544 gradient rows once at 36 flop per byte: an HBM roofline of its own too
        # (mvml_gemm_f16x2_amax_colsum: the same product with the bias column sums from its reads)
        amax_ev = summ.get("mvml_gemm_f16x2_amax", []) + summ.get("mvml_gemm_f16x2_amax_colsum", [])
        dw_ev = [e for e in amax_ev if (e[1] or {}).get("role") == "gat_dw" and e[1]["shape"][1] <= 96]
        amax_ev = [e for e in amax_ev if e not in dw_ev]
        if dw_ev:
            extra["roofline_dw_l1"] = roofline_entry(dw_ev, "hbm", load_traffic(wkey, "gemm_dw_l1"))
            extra["roofline_dw_l1"]["kernel"] = (
                "mvml_gemm_f16x2_amax_colsum for the layer-1 weight gradient gY[N, 1544]^T X[N, 76] and "
                "the bias column sums from the same reads (split-K gemm_f32_kernel + splitk_reduce_kernel "
                "+ the row sums' final pass); bytes = gY's 1544 columns, X and dW once")
        gemm_ev = (summ.get("mvml_gemm_f32", []) + summ.get("mvml_gemm_f32x3", [])
                   + summ.get("mvml_gemm_f16x2", []) + amax_ev
                   + summ.get("mvml_gemm_f16x2_bsplit", []) + rows_ev
                   + summ.get("mvml_gemm_f32x3_batched", []) + summ.get("mvml_lstm_gates_cell_fwd", [])
                   + summ.get("mvml_gemm_f16x2_ex", []) + summ.get("mvml_gemm_f16x2_batched", [])
                   + summ.get("mvml_gemm_f16x2_planes", [])
                   + ([] if args.proj_bf16 else proj_ev))
        bf_ev = summ.get("mvml_gemm_bf16", []) + (proj_ev if args.proj_bf16 else [])
        if bf_ev:
            extra["roofline_gemm_bf16"] = roofline_entry(bf_ev, "mfma")
            extra["roofline_gemm_bf16"].update(
                peak=BF16_MFMA_PEAK_TFS, note="GAT projection GEMMs on bf16 operands (config 4)",
                frac=round(extra["roofline_gemm_bf16"]["achieved"] / BF16_MFMA_PEAK_TFS, 4))
        if gemm_ev:
            extra["roofline_gemm"] = roofline_entry(gemm_ev, "mfma")
            if (summ.get("mvml_gemm_f16x2") or summ.get("mvml_gemm_f16x2_amax")
                    or summ.get("mvml_gemm_f16x2_amax_colsum") or summ.get("mvml_gemm_f16x2_bsplit")
                    or summ.get("mvml_gemm_f16x2_rows") or summ.get("mvml_gemm_f16x2_ex")):
                # scaled split-fp16: 3 fp16 MFMA per fp32 multiply-add -> fp32-equivalent peak
                # 2.5 PF / 3 (the skinny products that fall back to split-bf16 count against it too)
                extra["roofline_gemm"].update(
                    peak=BF16_MFMA_PEAK_TFS / 3, note="fp32-accurate scaled split-fp16 on fp16 MFMA "
                    "(3 MFMA per fp32 product); achieved is fp32-equivalent TFLOP/s, peak = dense "
                    "fp16 MFMA peak / 3; operand |max| passes (mvml_absmax_f32) timed separately")
                extra["roofline_gemm"]["frac"] = round(extra["roofline_gemm"]["achieved"] / (BF16_MFMA_PEAK_TFS / 3), 4)
            elif summ.get("mvml_gemm_f32x3"):
                # split-bf16: 6 bf16 MFMA per fp32 multiply-add -> fp32-equivalent peak 2.5 PF / 6
                extra["roofline_gemm"].update(
                    peak=BF16_MFMA_PEAK_TFS / 6, note="fp32-accurate split-bf16 (x3) on bf16 MFMA; "
                    "achieved is fp32-equivalent TFLOP/s, peak = dense bf16 MFMA peak / 6")
                extra["roofline_gemm"]["frac"] = round(extra["roofline_gemm"]["achieved"] / (BF16_MFMA_PEAK_TFS / 6), 4)
        extra["kernel_ms_per_step"] = {k: round(v["ms_per_step"], 3) for k, v in rows.items()}
        if "mvml_build_csr" in rows:
            # device collation per step batch (inside the timed step): CSR build + node-group plan
            extra["batching_ms_per_batch"] = round(sum(rows[k]["ms_per_step"] for k in
                                                       ("mvml_build_csr", "mvml_build_node_groups")
                                                       if k in rows), 4)
        # time per step outside every timed entry point: torch-side kernels (Adam, zero_grad,
        # pads / copies), launch gaps and allocator stalls (config 3: one stream, so the
        # entry-point times do not overlap)
        extra["untimed_ms_per_step"] = round(ms_per_step - sum(v["ms_per_step"] for v in rows.values()), 3)
    if step_ms:
        extra["step_ms"] = {"min": min(step_ms), "median": float(np.median(step_ms)),
                            "max": max(step_ms), "each": step_ms}
    if mem0:
        extra["allocator"] = {k: mem1[k] - mem0[k] for k in ALLOC_KEYS}
        extra["allocator"].update(reserved_gb=round(mem1["reserved_bytes"] / 2 ** 30, 2),
                                  peak_allocated_gb=round(mem1["peak_allocated_bytes"] / 2 ** 30, 2))

    # ---- view-only figure (the graph view alone, fixed upstream gradient at its output)
    if args.view_only_steps > 0 and not args.dry_run:
        for b in batches:
            gen = torch.Generator(device=dev).manual_seed(99 + b.B)
            b.upstream = torch.randn((b.B, 384), device=dev, generator=gen) * 1e-3
        step(batches[0], fused=False)
        barrier()
        sync()
        t1 = time.perf_counter()
        vm = 0
        for i in range(args.view_only_steps):
            b = batches[i % nb]
            step(b, fused=False)
            vm += b.B
        sync()
        barrier()
        ve = reduce_max(time.perf_counter() - t1)
        extra["view_only"] = {"value": round(reduce_sum(vm) / ve, 2), "unit": "molecules/s",
                              "ms_per_step": round(ve * 1e3 / args.view_only_steps, 3),
                              "steps": args.view_only_steps,
                              "what": "GNNModule fwd+bwd from a fixed upstream gradient + all-reduce + Adam"}
        for b in batches:
            b.upstream = None

    # ---- inference over the whole shard + the final embedding all-gather
    if not args.no_inference:
        model.eval()
        gather = EmbeddingAllGather()
        with torch.no_grad():
            model(batches[0].g, batches[0].feats)  # warm
            barrier()
            sync()
            t1 = time.perf_counter()
            emb = torch.cat([model(b.g, b.feats) for b in batches], 0)
            sync()
            t2 = time.perf_counter()
            barrier()
            full = gather(emb)
            sync()
            t3 = time.perf_counter()
        fwd_s, gat_s = reduce_max(t2 - t1), reduce_max(t3 - t2)
        extra["inference"] = {
            "molecules": int(full.shape[0]), "value": round(full.shape[0] / fwd_s, 2),
            "unit": "molecules/s", "forward_ms": round(fwd_s * 1e3, 2),
            "allgather_ms": round(gat_s * 1e3, 2), "allgather_bytes": int(full.numel() * 4),
            "checksum": float(full.double().sum().item()),
            "what": "GNNModule eval forward over every molecule of the shard, then one all-gather "
                    "of the (B_shard, 384) embeddings into the full matrix on every rank"}
        model.train()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.dry_run and not mvp:
        cpu = cpu_baseline(args.cpu_seconds, args.group_size, with_fusion=True)

    if rank == 0:
        gsz = args.group_size
        if args.workload == "config3":
            wl = (f"BASELINE config 3: one global set of {args.total_mols} KEGG-like molecules, "
                  f"sharded in whole {gsz}-molecule GraphNorm groups, streamed through "
                  f"{mols_per_step(args)}-molecule steps per GPU; view + fusion: GNNModule (GAT "
                  "[192,384] x4 heads, Set2Set 6x3, GraphNorm, fc) -> MVFusion (12-head 3-token "
                  "attention, Conv2d, MLP) -> BCEWithLogits, fwd+bwd+Adam")
        elif args.workload == "mvp":
            wl = (f"BASELINE config 4: the whole MVP model (model.py:13-75; RNNModule BiLSTM 2x384 "
                  f"over synthetic SMILES tokens, GNNModule, FPNModule 2513->512->384 over real "
                  f"fingerprint vectors (the restated fingerprints of the 420 KEGG test-split molecules, "
                  f"cycled), fusion head) -> BCEWithLogits -> backward -> one flat all-reduce of "
                  f"the {sum(p.numel() for p in params)} gradients -> Adam, on shards of the "
                  f"{args.total_mols}-molecule config-3 set")
        else:
            wl = ("BASELINE config 5 (150-400-atom molecules with 1-4 hubs of in-degree 32-128, "
                  "per-rank sets): GNNModule -> MVFusion -> BCEWithLogits, fwd+bwd+Adam")
        line = {
            "metric": METRIC if not args.dry_run else "DRY RUN (plumbing rehearsal, not a measurement)",
            "value": round(value, 2), "unit": "molecules/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16 projection, f32 elsewhere" if args.proj_bf16 else "f32",
            "data": "synthetic (seeded KEGG-like drug-like molecules, random-init weights; the "
                    "SMILES / fingerprint view embeddings fed to the fusion are fixed random tensors)",
            "config": {"workload": wl, "global_mols": args.total_mols if args.workload == "config3" else None,
                       "mols_per_step_per_gpu": batches[0].B, "batches_on_rank0": nb,
                       "atoms_per_step_rank0": batches[0].N, "edges_per_step_rank0": batches[0].E,
                       "graphnorm_group": gsz, "parallelism": f"dp{world}",
                       "projection": "bf16 operands, fp32 accumulate (config 4)" if args.proj_bf16
                       else {"x3": "fp32-accurate split-bf16 x3", "f16x2": "fp32-accurate scaled split-fp16",
                             "f32": "f32 MFMA"}.get(F.GEMM_ALGO, F.GEMM_ALGO)},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launcher: N ranks as child processes (no GPU call has happened in this process)
        from mvml_gat.dist import launch_local_ranks
        sys.exit(launch_local_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:]))
    run(args)


if __name__ == "__main__":
    main()
