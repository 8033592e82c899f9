"""world_size-2 gloo test of the data-parallel decomposition used by bench.py: each rank owns
whole GraphNorm groups, runs forward/backward independently, then ONE flat all-reduce of the
gradients reproduces the single-process gradient of the full batch."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mvml_gat.dist import FlatGradAllReduce, shard_groups


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(seed=0):
    from _util import batch_of_sizes, model_pair
    sizes = [9, 12, 7, 15, 10, 8, 11, 6, 13, 5]  # 5 groups of 2 molecules
    sb = batch_of_sizes(sizes, seed=seed)
    _, ref = model_pair(hidden=(8, 12), seed=seed, n_iters=2, n_layers=2)
    ref = ref.double().eval()
    return sb, ref


def _subbatch(sb, lo, hi):
    from _util import graph_dict
    from mvml_gat.synth import SynthBatch
    e0, e1 = int(sb.num_edges[:lo].sum()), int(sb.num_edges[:hi].sum())
    n0, n1 = int(sb.num_nodes[:lo].sum()), int(sb.num_nodes[:hi].sum())
    s = SynthBatch(sb.num_nodes[lo:hi], sb.num_edges[lo:hi], sb.src_local[e0:e1],
                   sb.dst_local[e0:e1], sb.feats[n0:n1])
    return graph_dict(s, group_size=2), torch.as_tensor(s.feats, dtype=torch.float64)


def _loss(model, gd, X, row0=0):
    y = model(gd, X)
    w = torch.arange(row0 * y.shape[1], row0 * y.shape[1] + y.numel(), dtype=y.dtype).view_as(y).sin()
    return (y * w).sum()


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sb, ref = _setup()
    costs = [int(sb.num_edges[2 * i:2 * i + 2].sum()) for i in range(5)]
    g0, g1 = shard_groups(costs, world, rank)
    gd, X = _subbatch(sb, 2 * g0, 2 * g1)
    _loss(ref, gd, X, 2 * g0).backward()
    FlatGradAllReduce(ref.parameters())()
    if rank == 0:
        out.put({n: p.grad.numpy().copy() for n, p in ref.named_parameters()})
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_flat_allreduce_matches_single_process():
    sb, ref = _setup()
    gd, X = _subbatch(sb, 0, 10)
    _loss(ref, gd, X).backward()
    want = {n: p.grad.clone() for n, p in ref.named_parameters()}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for n, g in want.items():
        assert torch.allclose(torch.as_tensor(got[n]), g, rtol=1e-10, atol=1e-12), (n, (torch.as_tensor(got[n]) - g).abs().max().item(), g.abs().max().item())


def test_shard_groups_balanced_and_covering():
    costs = np.r_[np.full(10, 100), np.full(10, 1000)]
    cuts = [shard_groups(costs, 4, r) for r in range(4)]
    assert cuts[0][0] == 0 and cuts[-1][1] == 20
    assert all(cuts[i][1] == cuts[i + 1][0] for i in range(3))
    loads = [costs[a:b].sum() for a, b in cuts]
    assert max(loads) <= 1.5 * (costs.sum() / 4)


def _gather_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mvml_gat.dist import EmbeddingAllGather
    sb, ref = _setup()
    costs = [int(sb.num_edges[2 * i:2 * i + 2].sum()) for i in range(5)]
    g0, g1 = shard_groups(costs, world, rank)
    gd, X = _subbatch(sb, 2 * g0, 2 * g1)
    with torch.no_grad():
        emb = ref(gd, X) if g1 > g0 else torch.zeros((0, 12), dtype=torch.float64)
        full = EmbeddingAllGather()(emb)
    out.put((rank, full.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_embedding_allgather_matches_single_process():
    """north_star's final embedding gather: per-rank (B_shard, D) embeddings of whole GraphNorm
    groups, all-gathered, equal the single-process embeddings of the whole batch, in order."""
    sb, ref = _setup()
    gd, X = _subbatch(sb, 0, 10)
    with torch.no_grad():
        want = ref(gd, X).numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(2):
        assert got[r].shape == want.shape
        np.testing.assert_allclose(got[r], want, rtol=1e-12, atol=1e-14)


def test_config3_set_shards_are_slices_of_the_global_set():
    """Config3Set.molecules(lo, hi) is independent of which range asks (chunk-seeded), so a
    rank's shard is exactly its slice of the single-process 1M-molecule set."""
    from mvml_gat.synth import Config3Set, slice_batch
    s = Config3Set(300, seed=5, chunk=128)
    full = s.molecules(0, 300)
    assert full.batch_size == 300 and int(full.num_nodes.sum()) == full.feats.shape[0]
    for lo, hi in ((0, 64), (64, 200), (192, 300), (127, 129)):
        part = s.molecules(lo, hi)
        ref = slice_batch(full, lo, hi)
        for k in ("num_nodes", "num_edges", "src_local", "dst_local", "feats"):
            np.testing.assert_array_equal(getattr(part, k), getattr(ref, k), err_msg=k)
    costs = s.group_costs(64)
    assert len(costs) == 5 and costs.sum() >= full.num_edges.sum()


def _run_bench(*args):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--dry-run", *args],
                       capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_launcher_two_ranks_dry_run():
    """`bench.py --gpus 2` with no WORLD_SIZE starts 2 ranks itself; one JSON line comes back
    with n_gpus 2; sharding + all-gather reproduce the single-rank embeddings exactly, and the
    DP training steps (flat all-reduce) run."""
    common = ["--total-mols", "1024", "--mols-per-step", "256"]
    one = _run_bench("--gpus", "1", "--steps", "0", "--warmup", "0", *common)
    two = _run_bench("--gpus", "2", "--steps", "0", "--warmup", "0", *common)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["inference"]["molecules"] == one["inference"]["molecules"] == 1024
    assert two["inference"]["checksum"] == one["inference"]["checksum"]
    trained = _run_bench("--gpus", "2", "--steps", "2", "--warmup", "1", *common)
    assert trained["n_gpus"] == 2 and trained["value"] > 0 and trained["config"]["parallelism"] == "dp2"


def _mvp_setup():
    """A small MVPRef (float64, eval: no dropout) and a 4-molecule batch in 2 GraphNorm groups."""
    from _util import batch_of_sizes, graph_dict
    from oracle.fusion_ref import MVPRef
    torch.manual_seed(3)
    ref = MVPRef(num_classes=3, in_feats=74, hidden_feats=(8, 12), num_step_set2set=2,
                 num_layer_set2set=2, rnn_embed_dim=6, blstm_dim=5, blstm_layers=1, fp_2_dim=7,
                 num_heads=2, dropout=0.5).double().eval()
    sb = batch_of_sizes([9, 12, 7, 15], seed=4)
    g = torch.Generator().manual_seed(5)
    lens = [7, 4, 9, 6]
    tok = torch.randint(1, 39, (4, 9), generator=g).double()
    for i, L in enumerate(lens):
        tok[i, L:] = 0
    fp = (torch.rand(4, 2513, generator=g) < 0.2).double()
    y = (torch.rand(4, 3, generator=g) < 0.4).double()
    return ref, sb, tok, lens, fp, y


def _mvp_batch(sb, tok, lens, fp, y, lo, hi):
    gd, X = _subbatch(sb, lo, hi)
    return ({"smiles": tok[lo:hi], "seq_len": lens[lo:hi]}, gd, X, fp[lo:hi], y[lo:hi])


def _mvp_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mvml_gat.mvp import train_step
    from oracle.fusion_ref import bce_logits_ref
    ref, sb, tok, lens, fp, y = _mvp_setup()
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-4)
    red = FlatGradAllReduce(ref.parameters(), average=True)
    for _ in range(2):
        train_step(ref, opt, _mvp_batch(sb, tok, lens, fp, y, 2 * rank, 2 * rank + 2), red,
                   loss_fn=bce_logits_ref)
    if rank == 0:
        out.put(({n: p.detach().numpy().copy() for n, p in ref.named_parameters()},
                 [n for n, p in ref.named_parameters() if p.grad is None]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_mvp_train_step_keeps_reference_adam_semantics():
    """two gloo ranks of mvp.train_step (each half of the batch, one flat
    all-reduce, Adam lr 1e-3 wd 1e-4 as main.py:88) equal the single-process steps; the
    parameters that never get a gradient in the reference (MVP.norm_layer, RNNModule.norm_layer,
    model.py:42, 120) keep grad None and are NOT moved by Adam's weight decay."""
    from mvml_gat.mvp import train_step
    from oracle.fusion_ref import bce_logits_ref
    ref, sb, tok, lens, fp, y = _mvp_setup()
    init = {n: p.detach().clone() for n, p in ref.named_parameters()}
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-4)
    for _ in range(2):
        train_step(ref, opt, _mvp_batch(sb, tok, lens, fp, y, 0, 4), loss_fn=bce_logits_ref)
    want = {n: p.detach().clone() for n, p in ref.named_parameters()}
    unused = {n for n, p in ref.named_parameters() if p.grad is None}
    assert unused == {"norm_layer.weight", "norm_layer.bias", "rnn.norm_layer.weight",
                      "rnn.norm_layer.bias"}, unused
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mvp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, got_unused = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert set(got_unused) == unused
    for n in unused:
        assert torch.equal(torch.as_tensor(got[n]), init[n]), n
    for n, w in want.items():
        d = (torch.as_tensor(got[n]) - w).abs().max().item()
        assert d <= 1e-12 * max(1.0, w.abs().max().item()), (n, d)


def _pattern_worker(rank, world, port, out):
    """Step 1: no rank uses parameter b.  Step 2: only rank 1 does — rank 0's LOCAL pattern is
    the same in both steps, so only the reduced flags tell it that b now has a gradient."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a = torch.nn.Parameter(torch.ones(3, dtype=torch.float64))
    b = torch.nn.Parameter(torch.ones(2, dtype=torch.float64))
    red = FlatGradAllReduce([a, b])
    seen = []
    for step in range(2):
        a.grad = b.grad = None
        loss = (a * (rank + 1)).sum()
        if step == 1 and rank == 1:
            loss = loss + (b * 3).sum()
        loss.backward()
        red()
        seen.append(None if b.grad is None else b.grad.tolist())
    out.put((rank, seen, a.grad.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_flat_allreduce_follows_other_ranks_presence_changes():
    """the presence flags must follow the GLOBAL pattern every step (a cache keyed
    on the local pattern left b None on rank 0 while rank 1 stepped it)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pattern_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r, (seen, ag)) for r, seen, ag in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(2):
        seen, ag = got[r]
        assert seen[0] is None, (r, seen)          # nobody used b: stays None (Adam skips it)
        assert seen[1] == [3.0, 3.0], (r, seen)    # rank 1's gradient, summed, on BOTH ranks
        assert ag == [3.0, 3.0, 3.0]               # 1 + 2
