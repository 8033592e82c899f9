"""Shared helpers for the parity tests: seeded molecule batches and weight-tied model pairs."""
import numpy as np
import torch

from mvml_gat import synth
from mvml_gat.nn import GNNModule
from oracle.gnn_ref import GNNModuleRef


def batch_of_sizes(sizes, seed=0, rings=2, hubs=False, n_hubs=1, partners=100):
    """Chain + ring molecules of the given sizes; hubs: n_hubs atoms per molecule bonded to
    `partners` random other atoms each (in / out degree partners + 3)."""
    rng = np.random.default_rng(seed)
    sizes = np.asarray(sizes, dtype=np.int64)
    hub_fn = None
    if hubs:
        def hub_fn(M, n, bonds, nb, deg):
            k = min(n - 1, partners)
            out = np.full((M, bonds.shape[1] + n_hubs * k, 2), -1, dtype=np.int32)
            nb2 = nb.copy()
            for i in range(M):
                row = bonds[i][bonds[i, :, 0] >= 0]
                out[i, :len(row)] = row
                pos = len(row)
                for h in rng.choice(n, size=min(n_hubs, n), replace=False):
                    pt = rng.choice(np.setdiff1d(np.arange(n), [h]), size=k, replace=False)
                    out[i, pos:pos + k, 0] = h
                    out[i, pos:pos + k, 1] = pt
                    deg[i, h] += k
                    deg[i, pt] += 1
                    pos += k
                nb2[i] = pos
            return out, nb2, deg
    return synth._gen_sizes(rng, sizes, lambda M, n: np.minimum(np.full(M, rings), max(n // 5, 0)),
                            hubs=hub_fn)


def graph_dict(sb, group_size=None):
    """Oracle-side view of a SynthBatch (numpy arrays)."""
    from oracle.graph_ref import batch_ref
    b = batch_ref(sb.num_nodes, sb.src_local, sb.dst_local, sb.num_edges)
    B = len(sb.num_nodes)
    gs = group_size or max(B, 1)
    b["group_offsets"] = list(range(0, B, gs)) + [B]
    return b


def randomize_(module, seed=0, scale=0.1):
    """Give zero-initialised parameters (biases, GraphNorm) non-trivial values."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in module.named_parameters():
            if name.endswith("bias") or "norm" in name:
                p.add_(scale * torch.randn(p.shape, generator=g))


def model_pair(in_feats=74, hidden=(192, 384), dropout=0.5, seed=0, n_iters=6, n_layers=3):
    torch.manual_seed(seed)
    prod = GNNModule(in_feats, list(hidden), dropout, n_iters, n_layers)
    randomize_(prod, seed)
    ref = GNNModuleRef(in_feats, list(hidden), dropout, n_iters, n_layers)
    missing = ref.load_state_dict(prod.state_dict(), strict=True)
    return prod, ref
