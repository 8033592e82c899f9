"""The whole MVP model (/root/reference/model.py:13-75) on the HIP path: the three view encoders
and the multi-view attention fusion, with the reference's constructor signature and
state_dict keys (``gnn.*``, ``rnn.*``, ``fp_mlp.*``, ``norm_layer_module.*``, ``conv.*``,
``linear_{q,k,v}.weight``, ``norm_layer.*``, ``mlp.*``), so a reference ``net_i.pkl``
``model_state_dict`` loads unchanged.

    MVP(num_classes, in_feats, hidden_feats, num_step_set2set, num_layer_set2set, rnn_embed_dim,
        blstm_dim, blstm_layers, fp_2_dim, num_heads, dropout, device)
    logits = model(smiles, graphs, atom_feats, fp_t)          # model.py:51-73

``smiles`` is dataset.py's ``{"smiles": [B, T], "seq_len": [...]}``, ``graphs`` a
BatchedMolGraph on the GPU with ``atom_feats`` its (N, 74) features, ``fp_t`` the (B, 2513)
fingerprints.  Every product runs on libmvml_gat.so (no CPU fallback); ``train_step`` is one
step of main.py:24-36 (BCEWithLogitsLoss, Adam) with BASELINE config 4's data-parallel flat
gradient all-reduce between backward and the optimizer step.
"""
import torch
import torch.nn as nn

from .fusion import FPNModule, MVFusion, bce_with_logits
from .nn import GNNModule
from .smiles import RNNModule, tokens_struct


# run the SMILES view on a side stream beside the graph view (MVP.forward)
OVERLAP_VIEWS = True
_SIDE = {}


def _side_stream(dev):
    """One side stream per device, created once (its workspace and allocator blocks persist)."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=dev)
    return _SIDE[key]


class MVP(MVFusion):
    def __init__(self, num_classes, in_feats=64, hidden_feats=None, num_step_set2set=6,
                 num_layer_set2set=3, rnn_embed_dim=64, blstm_dim=128, blstm_layers=2, fp_2_dim=128,
                 num_heads=4, dropout=0.2, device='cpu', proj_dtype=None):
        if hidden_feats is None:
            hidden_feats = [64, 64]
        super().__init__(hidden_feats[-1], num_heads, num_classes, dropout)
        self.device = device
        self.vocab = tokens_struct()
        self.gnn = GNNModule(in_feats, hidden_feats, dropout, num_step_set2set, num_layer_set2set,
                             proj_dtype=proj_dtype)
        self.rnn = RNNModule(self.vocab, rnn_embed_dim, blstm_dim, blstm_layers,
                             self.final_hidden_feats, dropout, bidirectional=True, device=device)
        self.fp_mlp = FPNModule(fp_2_dim, self.final_hidden_feats)
        self.sigmoid = nn.Sigmoid()

    def forward(self, smiles, graphs, atom_feats, fp_t):
        # The SMILES and graph views are independent until the fusion (model.py:53-55): the
        # BiLSTM recurrence (hundreds of short, latency-bound launches per step) runs on a side
        # stream while the graph view's HBM / MFMA-bound kernels run on the current one, so the
        # view kernels fill the CUs the recurrence leaves idle.  Autograd runs each op's backward
        # on its forward stream, so the two backward passes overlap the same way; the fusion
        # waits for both.  Same kernels, same arithmetic: results are bitwise those of running
        # the views one after the other.
        dev = atom_feats.device
        if dev.type != "cuda" or not OVERLAP_VIEWS:
            smiles_x = self.rnn(smiles)
            graph_x = self.gnn(graphs, atom_feats)
        else:
            cur = torch.cuda.current_stream(dev)
            side = _side_stream(dev)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                smiles_x = self.rnn(smiles)
            graph_x = self.gnn(graphs, atom_feats)
            cur.wait_stream(side)
            smiles_x.record_stream(cur)
        fp_x = self.fp_mlp(fp_t)
        # the shared LayerNorm (model.py:54-56), Q/K/V, attention, Conv2d and MLP
        return MVFusion.forward(self, smiles_x, graph_x, fp_x)

    def predict(self, smiles, graphs, atom_feats, fp_t):
        return self.sigmoid(self.forward(smiles, graphs, atom_feats, fp_t))


def join_side_stream(dev):
    """Make the current stream wait for the SMILES view's side stream.  After backward the
    side stream has accumulated that view's parameter gradients; the reducer and the optimizer
    read them on the current stream.  Autograd's end-of-backward leaf-stream sync already
    orders this, and this explicit wait (one event) keeps the order from depending on it."""
    dev = torch.device(dev)
    if dev.type != "cuda" or not OVERLAP_VIEWS:
        return
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key in _SIDE:
        torch.cuda.current_stream(dev).wait_stream(_SIDE[key])


def train_step(model, optimizer, batch, reducer=None, loss_fn=bce_with_logits):
    """main.py:24-36 for one batch: forward, BCEWithLogitsLoss (main.py:91), backward, the
    data-parallel flat gradient all-reduce (reducer, BASELINE config 4), optimizer step.
    batch = (smiles, graphs, atom_feats, fp_t, labels); returns the loss tensor.  Gradients are
    zeroed in place like the reference's optimizer.zero_grad() under its pinned torch 1.12.1
    (set_to_none=False, main.py:34); parameters that never receive a gradient (the unused
    LayerNorms, model.py:42, 120) keep grad None — the reducer preserves that — so Adam's
    weight decay leaves them alone.  loss_fn: the HIP BCEWithLogits by default (the CPU tests
    pass the oracle's)."""
    smiles, graphs, atom_feats, fp_t, labels = batch
    optimizer.zero_grad(set_to_none=False)
    loss = loss_fn(model(smiles, graphs, atom_feats, fp_t), labels)
    loss.backward()
    join_side_stream(atom_feats.device)
    if reducer is not None:
        reducer()
    optimizer.step()
    return loss
