"""Oracle: the multi-view attention fusion head of MVP — TEST INFRASTRUCTURE ONLY.

CPU restatement in plain PyTorch (float64 for parity, float32 for a CPU baseline) of
model.py:28-48 (layers) and model.py:57-71 (forward), with the loss of main.py:91:

    v_s, v_g, v_f = LayerNorm(384)(smiles_x), LayerNorm(384)(graph_x), LayerNorm(384)(fp_x)
    X = stack([v_s, v_g, v_f], dim=1)                          (B, 3, 384)   model.py:57-60
    q/k/v = Linear(384, 384*nh, bias=False)(X) -> (B, nh, 3, 384)            model.py:65-67
    att = softmax(q k^T / sqrt(384)) v                         (B, nh, 3, 384) model.py:68-70
    out = Dropout(ReLU(Conv2d(nh, nh, 3)(att))).view(B, -1)    (B, nh*382)    model.py:27, 71
    logits = Linear(1024, C)(Dropout(ReLU(Linear(nh*382, 1024)(out))))      model.py:40-45, 72
    loss = BCEWithLogitsLoss()(logits, labels)                                main.py:91

`norm_layer` (LayerNorm(nh*382), model.py:39) is constructed by the reference but never used
in its forward; it is kept here (and in the product module) only for state_dict parity.
Parity status: unpinned against the real reference (no torch 1.12 / reference run here); the
restatement is pinned by hand-derivable known answers in tests/test_oracle_kat.py.
"""
import math

import torch
import torch.nn as nn


class MVFusionRef(nn.Module):
    def __init__(self, dim=384, num_heads=12, num_classes=11, dropout=0.5):
        super().__init__()
        self.dim, self.num_heads = dim, num_heads
        self.norm_layer_module = nn.LayerNorm(dim)
        self.conv = nn.Sequential(nn.Conv2d(num_heads, num_heads, kernel_size=3), nn.ReLU(),
                                  nn.Dropout(dropout))
        self.linear_q = nn.Linear(dim, dim * num_heads, bias=False)
        self.linear_k = nn.Linear(dim, dim * num_heads, bias=False)
        self.linear_v = nn.Linear(dim, dim * num_heads, bias=False)
        self._norm_fact = 1 / math.sqrt(dim)
        self.norm_layer = nn.LayerNorm((dim - 2) * num_heads)
        self.mlp = nn.Sequential(nn.Linear((dim - 2) * num_heads, 1024), nn.ReLU(), nn.Dropout(dropout),
                                 nn.Linear(1024, num_classes))

    def forward(self, smiles_x, graph_x, fp_x, conv_branch=None, mlp_branch=None):
        """conv_branch (B, nh, 1, dim-2) / mlp_branch (B, 1024): optional given sides of the two
        ReLUs (gnn_ref.relu_branch), for evaluating the float64 oracle on the fp32 product's side
        of each kink (the parity tests); None = plain ReLU."""
        B = graph_x.shape[0]
        ln = self.norm_layer_module
        x = torch.cat([ln(smiles_x).view(B, 1, -1), ln(graph_x).view(B, 1, -1),
                       ln(fp_x).view(B, 1, -1)], dim=1)
        nh, dk = self.num_heads, self.dim
        q = self.linear_q(x).reshape(B, 3, nh, dk).transpose(1, 2)
        k = self.linear_k(x).reshape(B, 3, nh, dk).transpose(1, 2)
        v = self.linear_v(x).reshape(B, 3, nh, dk).transpose(1, 2)
        dist = torch.softmax(torch.matmul(q, k.transpose(2, 3)) * self._norm_fact, dim=-1)
        att = torch.matmul(dist, v)
        if conv_branch is None and mlp_branch is None:
            out = self.conv(att).view(B, -1)
            return self.mlp(out)
        from .gnn_ref import relu_branch
        c = self.conv[0](att)
        c = relu_branch(c, conv_branch.view_as(c)) if conv_branch is not None else torch.relu(c)
        out = self.conv[2](c).view(B, -1)
        h = self.mlp[0](out)
        h = relu_branch(h, mlp_branch) if mlp_branch is not None else torch.relu(h)
        return self.mlp[3](self.mlp[2](h))


def bce_logits_ref(logits, labels):
    """main.py:91: torch.nn.BCEWithLogitsLoss() (mean reduction)."""
    return nn.functional.binary_cross_entropy_with_logits(logits, labels)


class FPNModuleRef(nn.Module):
    """model.py:138-155 restated (reference order: fc1 -> Dropout -> ReLU -> fc2)."""

    def __init__(self, fp_2_dim=128, out_feats=384, dropout=0.2):
        super().__init__()
        self.fc1 = nn.Linear(2513, fp_2_dim)
        self.act_func = nn.ReLU()
        self.fc2 = nn.Linear(fp_2_dim, out_feats)
        self.dropout = nn.Dropout(p=dropout)

    def forward(self, fp):
        return self.fc2(self.act_func(self.dropout(self.fc1(fp))))


class MVPRef(MVFusionRef):
    """model.py:13-75 restated: MVP = RNNModule + GNNModule + FPNModule views -> the fusion head
    above, with the reference's state_dict keys (gnn.*, rnn.*, fp_mlp.*, fusion keys).
    forward(smiles_batch, graph_dict, atom_feats, fp_t, branches=None) -> logits (B, C)."""

    def __init__(self, num_classes=11, in_feats=74, hidden_feats=(192, 384), num_step_set2set=6,
                 num_layer_set2set=3, rnn_embed_dim=128, blstm_dim=384, blstm_layers=2,
                 fp_2_dim=512, num_heads=12, dropout=0.5):
        from .gnn_ref import GNNModuleRef
        from .smiles_ref import RNNModuleRef
        hidden_feats = list(hidden_feats)
        super().__init__(hidden_feats[-1], num_heads, num_classes, dropout)
        self.gnn = GNNModuleRef(in_feats, hidden_feats, dropout, num_step_set2set, num_layer_set2set)
        self.rnn = RNNModuleRef(39, rnn_embed_dim, blstm_dim, blstm_layers, hidden_feats[-1], dropout)
        self.fp_mlp = FPNModuleRef(fp_2_dim, hidden_feats[-1], dropout)

    def forward(self, smiles, graph, atom_feats, fp_t, branches=None, conv_branch=None,
                mlp_branch=None):
        return MVFusionRef.forward(self, self.rnn(smiles), self.gnn(graph, atom_feats, branches),
                                   self.fp_mlp(fp_t), conv_branch, mlp_branch)
