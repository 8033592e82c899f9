"""Oracle: GAT -> Set2Set -> GraphNorm -> Linear restated in plain PyTorch on CPU.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py; parity unpinned against DGL/PyG).
Every function runs in whatever dtype its inputs carry (float64 for parity, float32 for
the CPU baseline) and on whatever device they live on (the CPU normally; the bench-size
parity tests run the same float64 torch ops on the GPU — still the checker, never the
product path), and is differentiable with torch autograd, which supplies the oracle
backward (a15).

Restated semantics (pinned third-party versions from README.md:10-19):

* ``gatconv_ref``   dgl 0.9.1 GATConv.forward with residual=True (res_fc = Linear without
  bias because in_feats != H*F), explicit bias, feat/attn dropout 0:
  Z = fc(X).view(N,H,F); el = (Z*attn_l).sum(-1); er = (Z*attn_r).sum(-1);
  e = leaky_relu(el[src] + er[dst], 0.2); a = edge_softmax(e) over in-edges of each dst
  (max-subtracted; DGL treats the max as a constant); rst[v] = sum_e a_e * Z[src_e];
  rst += res_fc(X).view(N,H,F); rst += bias.view(H,F).
* ``gat_ref``       dgllife 0.3.0 GAT(in_feats, hidden_feats) defaults (model.py:81):
  num_heads 4 per layer, layers 0..L-2 agg 'flatten' + ELU, last layer agg 'mean',
  no activation.
* ``set2set_ref``   dgl 0.9.1 Set2Set(input_dim, n_iters=6, n_layers=3) (model.py:82-84, 92):
  q* = 0; h = c = 0; repeat n_iters: q, (h, c) = LSTM(q*[None], (h, c));
  e_n = <x_n, q[g(n)]>; alpha = softmax_nodes(e); r = sum_nodes(alpha * x); q* = [q, r].
* ``graphnorm_ref`` torch_geometric 2.2.0 GraphNorm(in_channels, eps=1e-5) called with
  batch=None (model.py:93): per normalisation group (the whole mini-batch in the
  reference) mean = mean(x); out = x - mean*mean_scale; var = mean(out**2);
  y = weight * out / sqrt(var + eps) + bias.
* ``GNNModuleRef``  model.py:77-95 with identical parameter names, so a state_dict saved
  from the reference's GNNModule (prefix ``gnn.`` stripped) loads into it unchanged.
"""
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


def _as_long(a, device=None):
    if isinstance(a, torch.Tensor):
        return a.to(device=device, dtype=torch.long)
    return torch.as_tensor(np.asarray(a), dtype=torch.long, device=device)


def edge_softmax_ref(score, dst, num_nodes):
    """dgl edge_softmax(norm_by='dst'): score (E,H) -> attention (E,H)."""
    H = score.shape[1]
    idx = dst.view(-1, 1).expand(-1, H)
    smax = torch.full((num_nodes, H), -math.inf, dtype=score.dtype, device=score.device)
    smax = smax.scatter_reduce(0, idx, score.detach(), reduce="amax", include_self=True)
    ex = torch.exp(score - smax[dst])
    ssum = torch.zeros((num_nodes, H), dtype=score.dtype, device=score.device).index_add(0, dst, ex)
    return ex / ssum[dst]


def leaky_relu_branch(x, slope, positive):
    """LeakyReLU whose branch is GIVEN per element (positive: bool, same shape): equal to
    leaky_relu(x) wherever sign(x) agrees with `positive`, and its gradient is 1 / slope by
    `positive`.  Used by the parity tests to evaluate the float64 oracle on the SAME side of the
    kink at 0 as the fp32 path under test: at |x| ~ 1e-8 the side is decided by fp32 rounding
    of el + er, and the two one-sided derivatives differ by 0.8 (a subgradient choice, not an
    error of either implementation)."""
    return torch.where(positive, x, x * slope)


def relu_branch(x, positive):
    """ReLU whose side is GIVEN per element (the product's own fp32 side, read off its post-ReLU
    output > 0): equal to relu(x) wherever sign(x) agrees; used like leaky_relu_branch."""
    return torch.where(positive, x, torch.zeros_like(x))


def gatconv_ref(src, dst, X, fc_w, res_w, attn_l, attn_r, bias, num_heads, out_feats,
                negative_slope=0.2, return_attention=False, branch=None):
    src = _as_long(src, X.device)
    dst = _as_long(dst, X.device)
    n = X.shape[0]
    H, Fo = num_heads, out_feats
    Z = (X @ fc_w.t()).view(n, H, Fo)
    el = (Z * attn_l).sum(-1)
    er = (Z * attn_r).sum(-1)
    if branch is None:
        e = F.leaky_relu(el[src] + er[dst], negative_slope)
    else:
        e = leaky_relu_branch(el[src] + er[dst], negative_slope, branch)
    a = edge_softmax_ref(e, dst, n)
    rst = torch.zeros((n, H, Fo), dtype=X.dtype, device=X.device).index_add(0, dst, a.unsqueeze(-1) * Z[src])
    rst = rst + (X @ res_w.t()).view(n, H, Fo)
    rst = rst + bias.view(1, H, Fo)
    if return_attention:
        return rst, a
    return rst


def _bf16_round(x):
    """x rounded to bf16 (round-to-nearest-even, via fp32 as the product sees its fp32 operands),
    carried in x's dtype."""
    return x.to(torch.float32).to(torch.bfloat16).to(x.dtype)


class _ProjBF16(torch.autograd.Function):
    """Y = bf16(X) bf16(Wcat)^T, with the backward's two products on bf16-rounded operands too:
    dX = bf16(gY) bf16(Wcat), dWcat = bf16(gY)^T bf16(X) — exactly the rounding points of the
    bf16 projection (mvml_gemm_bf16 on X, Wcat and gY; mvml_gat.functional GATLayerFunction with
    algo 'bf16'), every other operation in the input dtype (float64: the bf16-EMULATED oracle)."""

    @staticmethod
    def forward(ctx, X, Wcat):
        ctx.save_for_backward(X, Wcat)
        return _bf16_round(X) @ _bf16_round(Wcat).t()

    @staticmethod
    def backward(ctx, gY):
        X, Wcat = ctx.saved_tensors
        g = _bf16_round(gY)
        return g @ _bf16_round(Wcat), g.t() @ _bf16_round(X)


def gat_layer_bf16_ref(src, dst, X, p, num_heads, out_feats, agg_mode, activation, branch=None):
    """The bf16-projection path's GATConv in ITS association (mvml_gat_fold_weights): one
    product Y = X Wcat^T with Wcat = [fc.weight ; res_fc.weight (head mean in the 'mean' layer) ;
    A_l ; A_r], A_l[h] = sum_f attn_l[h, f] fc.weight[h F + f] (el = X A_l^T is (Z * attn_l).sum
    re-associated), so el / er and the residual see the same bf16 rounding as Z; then dgl's
    edge softmax and u_mul_e sum exactly as gatconv_ref.  Same function as gat_layer_ref up to
    the re-association and the bf16 rounding of _ProjBF16."""
    src = _as_long(src, X.device)
    dst = _as_long(dst, X.device)
    n = X.shape[0]
    H, Fo = num_heads, out_feats
    fc_w, res_w = p["fc.weight"], p["res_fc.weight"]
    mean = agg_mode == "mean"
    Wfc = fc_w.view(H, Fo, -1)
    A_l = (p["attn_l"].view(H, Fo, 1) * Wfc).sum(1)
    A_r = (p["attn_r"].view(H, Fo, 1) * Wfc).sum(1)
    R_w = res_w.view(H, Fo, -1).mean(0) if mean else res_w
    Wcat = torch.cat([fc_w, R_w, A_l, A_r], 0)
    Y = _ProjBF16.apply(X, Wcat)
    HF = H * Fo
    RC = Fo if mean else HF
    Z = Y[:, :HF].view(n, H, Fo)
    R = Y[:, HF:HF + RC]
    el, er = Y[:, HF + RC:HF + RC + H], Y[:, HF + RC + H:HF + RC + 2 * H]
    s = el[src] + er[dst]
    e = F.leaky_relu(s, 0.2) if branch is None else leaky_relu_branch(s, 0.2, branch)
    a = edge_softmax_ref(e, dst, n)
    agg = torch.zeros((n, H, Fo), dtype=X.dtype, device=X.device).index_add(0, dst, a.unsqueeze(-1) * Z[src])
    bias = p["bias"].view(H, Fo)
    if mean:
        out = agg.mean(1) + R + bias.mean(0)
    else:
        out = (agg + R.view(n, H, Fo) + bias).flatten(1)
    if activation is not None:
        out = activation(out)
    return out


def gat_layer_ref(src, dst, X, p, num_heads, out_feats, agg_mode, activation, branch=None,
                  proj=None):
    """dgllife GATLayer.forward: gat_conv -> flatten(1) | mean(1) -> activation.  proj='bf16':
    the bf16-emulated projection (gat_layer_bf16_ref)."""
    if proj == "bf16":
        return gat_layer_bf16_ref(src, dst, X, p, num_heads, out_feats, agg_mode, activation, branch)
    rst = gatconv_ref(src, dst, X, p["fc.weight"], p["res_fc.weight"], p["attn_l"],
                      p["attn_r"], p["bias"], num_heads, out_feats, branch=branch)
    out = rst.flatten(1) if agg_mode == "flatten" else rst.mean(1)
    if activation is not None:
        out = activation(out)
    return out


def gat_ref(src, dst, X, layer_params, hidden_feats, num_heads=None, branches=None, proj=None):
    L = len(hidden_feats)
    num_heads = num_heads or [4] * L
    h = X
    for i in range(L):
        last = i == L - 1
        h = gat_layer_ref(src, dst, h, layer_params[i], num_heads[i], hidden_feats[i],
                          "mean" if last else "flatten", None if last else F.elu,
                          branch=None if branches is None else branches[i], proj=proj)
    return h


def set2set_ref(node_offsets, X, lstm, n_iters):
    node_offsets = np.asarray(node_offsets, dtype=np.int64)
    B = len(node_offsets) - 1
    D = X.shape[1]
    dev = X.device
    counts = torch.as_tensor(np.diff(node_offsets), dtype=torch.long, device=dev)
    gid = torch.repeat_interleave(torch.arange(B, device=dev), counts)
    nl = lstm.num_layers
    h = (X.new_zeros((nl, B, D)), X.new_zeros((nl, B, D)))
    q_star = X.new_zeros((B, 2 * D))
    for _ in range(n_iters):
        q, h = lstm(q_star.unsqueeze(0), h)
        q = q.view(B, D)
        e = (X * q[gid]).sum(-1)
        emax = torch.full((B,), -math.inf, dtype=X.dtype, device=dev).scatter_reduce(
            0, gid, e.detach(), reduce="amax", include_self=True)
        ex = torch.exp(e - emax[gid])
        esum = torch.zeros(B, dtype=X.dtype, device=dev).index_add(0, gid, ex)
        alpha = ex / esum[gid]
        readout = torch.zeros((B, D), dtype=X.dtype, device=dev).index_add(0, gid, X * alpha.unsqueeze(-1))
        q_star = torch.cat([q, readout], dim=-1)
    return q_star


def graphnorm_ref(x, weight, bias, mean_scale, eps=1e-5, group_offsets=None):
    if group_offsets is None:
        group_offsets = [0, x.shape[0]]
    outs = []
    for g0, g1 in zip(group_offsets[:-1], group_offsets[1:]):
        xs = x[int(g0):int(g1)]
        mean = xs.mean(0, keepdim=True)
        out = xs - mean * mean_scale
        var = (out * out).mean(0, keepdim=True)
        std = (var + eps).sqrt()
        outs.append(weight * out / std + bias)
    return torch.cat(outs, 0)


class _GATConvParams(nn.Module):
    """Parameter layout of dgl 0.9.1 GATConv (registration order: attn_l, attn_r, bias,
    fc, res_fc)."""

    def __init__(self, in_feats, out_feats, num_heads):
        super().__init__()
        self.fc = nn.Linear(in_feats, out_feats * num_heads, bias=False)
        self.attn_l = nn.Parameter(torch.empty(1, num_heads, out_feats))
        self.attn_r = nn.Parameter(torch.empty(1, num_heads, out_feats))
        self.bias = nn.Parameter(torch.empty(num_heads * out_feats))
        self.res_fc = nn.Linear(in_feats, out_feats * num_heads, bias=False)
        gain = nn.init.calculate_gain("relu")
        nn.init.xavier_normal_(self.fc.weight, gain=gain)
        nn.init.xavier_normal_(self.attn_l, gain=gain)
        nn.init.xavier_normal_(self.attn_r, gain=gain)
        nn.init.constant_(self.bias, 0)
        nn.init.xavier_normal_(self.res_fc.weight, gain=gain)


class _GATLayerParams(nn.Module):
    def __init__(self, in_feats, out_feats, num_heads):
        super().__init__()
        self.gat_conv = _GATConvParams(in_feats, out_feats, num_heads)


class _GATParams(nn.Module):
    def __init__(self, in_feats, hidden_feats, num_heads=4):
        super().__init__()
        self.gnn_layers = nn.ModuleList()
        for i, hf in enumerate(hidden_feats):
            self.gnn_layers.append(_GATLayerParams(in_feats, hf, num_heads))
            in_feats = hf * num_heads if i < len(hidden_feats) - 1 else hf


class _Set2SetParams(nn.Module):
    def __init__(self, input_dim, n_iters, n_layers):
        super().__init__()
        self.input_dim, self.n_iters, self.n_layers = input_dim, n_iters, n_layers
        self.lstm = nn.LSTM(2 * input_dim, input_dim, n_layers)


class _GraphNormParams(nn.Module):
    def __init__(self, in_channels, eps=1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(in_channels))
        self.bias = nn.Parameter(torch.zeros(in_channels))
        self.mean_scale = nn.Parameter(torch.ones(in_channels))


class GNNModuleRef(nn.Module):
    """model.py:77-95 restated.  forward(graph_dict, atom_feats) -> (B, hidden_feats[-1]).

    ``graph`` is a dict with numpy ``src``, ``dst``, ``node_offsets`` and optional
    ``group_offsets`` (GraphNorm groups, in molecules; default: the whole batch,
    which is what model.py:93 does with batch=None).
    """

    def __init__(self, in_feats=74, hidden_feats=None, dropout=0.5, num_step_set2set=6,
                 num_layer_set2set=3, proj=None):
        super().__init__()
        self.proj = proj  # None: exact; 'bf16': the bf16-emulated GAT projections
        hidden_feats = list(hidden_feats or [192, 384])
        self.hidden_feats = hidden_feats
        self.conv = _GATParams(in_feats, hidden_feats)
        self.readout = _Set2SetParams(hidden_feats[-1], num_step_set2set, num_layer_set2set)
        self.norm = _GraphNormParams(hidden_feats[-1] * 2)
        self.fc = nn.Sequential(nn.Linear(hidden_feats[-1] * 2, hidden_feats[-1]), nn.ReLU(),
                                nn.Dropout(p=dropout))

    def layer_params(self):
        out = []
        for layer in self.conv.gnn_layers:
            c = layer.gat_conv
            out.append({"fc.weight": c.fc.weight, "res_fc.weight": c.res_fc.weight,
                        "attn_l": c.attn_l, "attn_r": c.attn_r, "bias": c.bias})
        return out

    def forward(self, graph, atom_feats, branches=None, fc_branch=None):
        """branches: optional per-GAT-layer bool (E, H) LeakyReLU sides (leaky_relu_branch);
        fc_branch: optional bool (B, out) side of the fc ReLU (relu_branch)."""
        node_x = gat_ref(graph["src"], graph["dst"], atom_feats, self.layer_params(),
                         self.hidden_feats, branches=branches, proj=self.proj)
        graph_x = set2set_ref(graph["node_offsets"], node_x, self.readout.lstm,
                              self.readout.n_iters)
        out = graphnorm_ref(graph_x, self.norm.weight, self.norm.bias, self.norm.mean_scale,
                            self.norm.eps, graph.get("group_offsets"))
        if fc_branch is None:
            return self.fc(out)
        return self.fc[2](relu_branch(self.fc[0](out), fc_branch))
