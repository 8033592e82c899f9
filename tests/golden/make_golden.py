"""Generate the committed golden fixtures (tests/golden/*.npz) from the CPU oracle.

These are regression vectors of the oracle restatement (float64), NOT outputs of the reference:
the reference's third-party kernels (dgl / dgllife / PyG) are not installable here and the
reference ships no fixtures (SURVEY.md §8c — parity unpinned).  They pin the oracle against
drift and give the GPU tests a fixed target that does not depend on re-running the oracle.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mvml-mpi_amd")]

from oracle.gnn_ref import GNNModuleRef  # noqa: E402
from oracle.graph_ref import batch_ref, bigraph_edges, csr_ref  # noqa: E402

MOLS = [  # (num_atoms, bonds) — small hand-made molecules incl. a ring, a branch and an ion
    (6, [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 0)]),           # benzene-like ring
    (4, [(0, 1), (1, 2), (1, 3)]),                                    # branched
    (1, []),                                                          # single atom (ion)
    (5, [(0, 1), (1, 2), (2, 3), (3, 4), (4, 1)]),                    # tail + 4-ring
    (3, [(0, 1), (1, 2)]),
]


# (file, GraphNorm group size).  gnn_small: ONE group over the whole 5-molecule batch, exactly
# model.py:93 (GraphNorm with batch=None normalises over the mini-batch).  gnn_small_groups:
# groups of 3 + 2 molecules, the multi-group batching of mvml_gat; a 2-molecule group makes
# GraphNorm ill-conditioned (x - mean cancels), so fp32 errors are amplified ~10x there.
FIXTURES = (("gnn_small.npz", 5), ("gnn_small_groups.npz", 3))


def build(group_size=3, seed=7):
    n = [m[0] for m in MOLS]
    edges = [bigraph_edges(a, b) for a, b in MOLS]
    src_l = np.concatenate([e[0] for e in edges])
    dst_l = np.concatenate([e[1] for e in edges])
    ne = [len(e[0]) for e in edges]
    g = batch_ref(n, src_l, dst_l, ne)
    B = len(MOLS)
    g["group_offsets"] = list(range(0, B, group_size)) + [B]
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((sum(n), 74)) * 0.5
    torch.manual_seed(seed)
    ref = GNNModuleRef(74, [16, 24], 0.5, 3, 2).double().eval()
    gen = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in ref.named_parameters():
            if name.endswith("bias") or "norm" in name:
                p.add_(0.1 * torch.randn(p.shape, generator=gen, dtype=p.dtype))
    Xt = torch.as_tensor(X).requires_grad_()
    out = ref(g, Xt)
    gout = torch.as_tensor(rng.standard_normal(out.shape))
    out.backward(gout)
    d = {"num_nodes": np.asarray(n, np.int64), "num_edges": np.asarray(ne, np.int64),
         "src_local": src_l, "dst_local": dst_l, "group_size": np.int64(group_size), "X": X,
         "out": out.detach().numpy(), "g_out": gout.numpy(), "g_X": Xt.grad.numpy()}
    for k, v in g.items():
        if k in ("src", "dst", "node_offsets", "edge_offsets"):
            d["batch_" + k] = np.asarray(v)
    c = csr_ref(g["src"], g["dst"], sum(n))
    for k in ("in_rowptr", "in_src", "in_eid", "out_rowptr", "out_dst", "out_inslot"):
        d["csr_" + k] = c[k]
    for name, p in ref.named_parameters():
        d["param:" + name] = p.detach().numpy()
        d["grad:" + name] = p.grad.numpy()
    return d


if __name__ == "__main__":
    for name, gs in FIXTURES:
        d = build(group_size=gs)
        path = os.path.join(HERE, name)
        np.savez_compressed(path, **d)
        print(f"wrote {path} ({os.path.getsize(path)} bytes, {len(d)} arrays)")
