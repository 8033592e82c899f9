"""mvml_gat — MI355X-native molecular-graph (GAT) view of MVML-MPI.

Drop-in for the reference's graph view (model.py:77-95) on the HIP path:

    from mvml_gat import GNNModule, batch
    bg = batch(graphs).to("cuda")                 # dgl.batch + device-side CSR build
    emb = GNNModule(74, [192, 384], 0.5, 6, 3).cuda()(bg, bg.ndata["h"])   # (B, 384)

All arithmetic of the training step runs in hand-written HIP kernels (libmvml_gat.so, C ABI in
include/mvml_gat.h); main.py:88's optimizer is ``FlatAdam(model.parameters(), lr=...,
weight_decay=...)`` (Adam on the device, one gradient all-reduce).  There is no CPU fallback: ops raise if the library is missing or the
tensors are not on the GPU.
"""
from ._lib import MvmlError, lib
from .batching import BatchedMolGraph, MolGraph, batch, bigraph_from_bonds, from_arrays, graph
from .fusion import FPNModule, MVFusion, bce_with_logits
from .smiles import RNNModule, collate_smiles, tokens_struct
from .nn import GAT, GATConv, GATLayer, GNNModule, GraphNorm, Set2Set
from .optim import FlatAdam

__all__ = ["GNNModule", "MVFusion", "FPNModule", "RNNModule", "tokens_struct", "collate_smiles", "bce_with_logits", "GAT", "GATLayer", "GATConv", "Set2Set", "GraphNorm", "BatchedMolGraph",
           "MolGraph", "batch", "graph", "bigraph_from_bonds", "from_arrays", "lib", "MvmlError", "FlatAdam"]
__version__ = "0.1.0"
