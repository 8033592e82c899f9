"""nn.Modules with the reference's constructor signatures and state_dict layout.

Drop-in replacements, on the MI355X HIP path, for
  * dgl 0.9.1 ``GATConv`` and dgllife 0.3.0 ``GATLayer`` / ``GAT`` (model.py:6, 81, 91),
  * dgl 0.9.1 ``Set2Set`` (model.py:7, 82-84, 92),
  * torch_geometric 2.2.0 ``GraphNorm`` (model.py:10, 85, 93),
  * ``GNNModule`` itself (model.py:77-95).
Parameter names/shapes/registration order follow the reference so a ``net_i.pkl``
``model_state_dict`` (keys under ``gnn.``) loads unchanged.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import functional as Fn
from .batching import BatchedMolGraph


class GATConv(nn.Module):
    """dgl.nn.pytorch.GATConv (0.9.1) parameters for the configuration dgllife uses here:
    residual=True (res_fc is a bias-free Linear when in_feats != heads*out_feats), explicit
    bias, feat/attn dropout 0.  forward() returns rst (N, H, F) like DGL (activation None)."""

    def __init__(self, in_feats, out_feats, num_heads, feat_drop=0.0, attn_drop=0.0,
                 negative_slope=0.2, residual=False, activation=None,
                 allow_zero_in_degree=False, bias=True):
        super().__init__()
        if feat_drop or attn_drop:
            raise NotImplementedError("GATConv: feat_drop/attn_drop > 0 are not on the fused path")
        if not residual or not bias or in_feats == out_feats * num_heads:
            raise NotImplementedError(
                "GATConv: only residual=True with a projecting res_fc and bias=True (the "
                "dgllife GAT defaults used by model.py:81) are implemented")
        self._num_heads = num_heads
        self._in_feats = in_feats
        self._out_feats = out_feats
        self._allow_zero_in_degree = allow_zero_in_degree
        self.negative_slope = negative_slope
        self.activation = activation
        self.fc = nn.Linear(in_feats, out_feats * num_heads, bias=False)
        self.attn_l = nn.Parameter(torch.empty(1, num_heads, out_feats))
        self.attn_r = nn.Parameter(torch.empty(1, num_heads, out_feats))
        self.bias = nn.Parameter(torch.empty(num_heads * out_feats))
        self.res_fc = nn.Linear(in_feats, num_heads * out_feats, bias=False)
        # GEMM operand precision of fc / res_fc (forward and both backward products): None =
        # fp32-accurate (the reference's fp32), torch.bfloat16 = bf16 operands with fp32
        # accumulation (BASELINE config 4, accuracy bar 2e-2).  Parameters stay fp32.
        self.proj_dtype = None
        self.reset_parameters()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        """Accept both DGL GATConv parameter layouts.  dgl 0.9.1 (README.md pins) keeps an
        explicit ``bias`` and a bias-free ``res_fc``; later DGL releases fold the bias into the
        residual Linear (``res_fc.bias``, no ``bias``) when ``res_fc`` projects.  The arithmetic
        is the same (res_fc(x) + b), so the folded form loads into ``bias`` here."""
        rb, b = prefix + "res_fc.bias", prefix + "bias"
        if rb in state_dict and b not in state_dict:
            state_dict[b] = state_dict.pop(rb)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                      unexpected_keys, error_msgs)

    def reset_parameters(self):
        gain = nn.init.calculate_gain("relu")
        nn.init.xavier_normal_(self.fc.weight, gain=gain)
        nn.init.xavier_normal_(self.attn_l, gain=gain)
        nn.init.xavier_normal_(self.attn_r, gain=gain)
        nn.init.constant_(self.bias, 0)
        nn.init.xavier_normal_(self.res_fc.weight, gain=gain)

    def _check_graph(self, graph):
        if not isinstance(graph, BatchedMolGraph):
            raise TypeError("graph must be a mvml_gat.BatchedMolGraph (see mvml_gat.batch)")
        if graph.device.type != "cuda":
            raise RuntimeError("graph must be moved to the GPU with .to('cuda') first")
        if graph.has_zero_in_degree and not self._allow_zero_in_degree:
            raise RuntimeError(
                "There are 0-in-degree nodes in the graph, output for those nodes will be invalid. "
                "Adding self-loop on the input graph by calling `g = dgl.add_self_loop(g)` will resolve "
                "the issue. Setting ``allow_zero_in_degree`` to be `True` when constructing this module "
                "will suppress the check and let the code run.")

    def fused(self, graph, feat, mode):
        self._check_graph(graph)
        return Fn.GATLayerFunction.apply(feat, self.fc.weight, self.res_fc.weight, self.attn_l,
                                         self.attn_r, self.bias, graph, self._num_heads,
                                         self._out_feats, self.negative_slope, mode,
                                         "bf16" if self.proj_dtype == torch.bfloat16 else None)

    def forward(self, graph, feat):
        rst = self.fused(graph, feat, Fn.MODE_FLATTEN).view(-1, self._num_heads, self._out_feats)
        if self.activation is not None:
            rst = self.activation(rst)
        return rst


class GATLayer(nn.Module):
    """dgllife.model.gnn.gat.GATLayer (0.3.0): gat_conv -> flatten(1) | mean(1) -> activation,
    fused into one kernel for the (flatten, ELU) and (mean, None) combinations GAT uses."""

    def __init__(self, in_feats, out_feats, num_heads, feat_drop=0.0, attn_drop=0.0, alpha=0.2,
                 residual=True, agg_mode="flatten", activation=None, bias=True,
                 allow_zero_in_degree=False):
        super().__init__()
        self.gat_conv = GATConv(in_feats, out_feats, num_heads, feat_drop, attn_drop, alpha,
                                residual, None, allow_zero_in_degree, bias)
        assert agg_mode in ["flatten", "mean"]
        self.agg_mode = agg_mode
        self.activation = activation

    def forward(self, bg, feats):
        act = self.activation
        if self.agg_mode == "flatten":
            if act is F.elu:
                return self.gat_conv.fused(bg, feats, Fn.MODE_FLATTEN_ELU)
            out = self.gat_conv.fused(bg, feats, Fn.MODE_FLATTEN)
        else:
            out = self.gat_conv.fused(bg, feats, Fn.MODE_MEAN)
        return act(out) if act is not None else out


class GAT(nn.Module):
    """dgllife.model.gnn.gat.GAT (0.3.0) with its defaults: 4 heads per layer, alpha 0.2,
    residual, 'flatten' + ELU for all but the last layer, 'mean' + no activation last."""

    def __init__(self, in_feats, hidden_feats=None, num_heads=None, feat_drops=None,
                 attn_drops=None, alphas=None, residuals=None, agg_modes=None, activations=None,
                 biases=None, allow_zero_in_degree=False):
        super().__init__()
        hidden_feats = list(hidden_feats) if hidden_feats is not None else [32, 32]
        n = len(hidden_feats)
        num_heads = num_heads or [4] * n
        feat_drops = feat_drops or [0.0] * n
        attn_drops = attn_drops or [0.0] * n
        alphas = alphas or [0.2] * n
        residuals = residuals or [True] * n
        if agg_modes is None:
            agg_modes = ["flatten"] * (n - 1) + ["mean"]
        if activations is None:
            activations = [F.elu] * (n - 1) + [None]
        biases = biases or [True] * n
        self.hidden_feats = hidden_feats
        self.num_heads = num_heads
        self.agg_modes = agg_modes
        self.gnn_layers = nn.ModuleList()
        for i in range(n):
            self.gnn_layers.append(GATLayer(in_feats, hidden_feats[i], num_heads[i], feat_drops[i],
                                            attn_drops[i], alphas[i], residuals[i], agg_modes[i],
                                            activations[i], biases[i], allow_zero_in_degree))
            in_feats = hidden_feats[i] * num_heads[i] if agg_modes[i] == "flatten" else hidden_feats[i]

    def reset_parameters(self):
        for layer in self.gnn_layers:
            layer.gat_conv.reset_parameters()

    def forward(self, g, feats):
        # inside the stack a flatten + ELU layer's output feeds only the next layer: its ELU
        # backward may run in that layer's data-gradient GEMM (functional.EluLink)
        prev, Fn.ELU_LINK[0] = Fn.ELU_LINK[0], True
        try:
            for gnn in self.gnn_layers:
                feats = gnn(g, feats)
        finally:
            Fn.ELU_LINK[0] = prev
        return feats


class Set2Set(nn.Module):
    """dgl.nn.pytorch.glob.Set2Set (0.9.1): lstm = nn.LSTM(2*input_dim, input_dim, n_layers)
    (the module is a parameter container; the recurrence runs on the HIP kernels)."""

    def __init__(self, input_dim, n_iters, n_layers):
        super().__init__()
        self.input_dim = input_dim
        self.output_dim = 2 * input_dim
        self.n_iters = n_iters
        self.n_layers = n_layers
        self.lstm = nn.LSTM(self.output_dim, self.input_dim, n_layers)
        self.reset_parameters()

    def reset_parameters(self):
        self.lstm.reset_parameters()

    def lstm_params(self):
        out = []
        for l in range(self.n_layers):
            out += [getattr(self.lstm, f"weight_ih_l{l}"), getattr(self.lstm, f"weight_hh_l{l}"),
                    getattr(self.lstm, f"bias_ih_l{l}"), getattr(self.lstm, f"bias_hh_l{l}")]
        return out

    def forward(self, graph, feat):
        return Fn.Set2SetFunction.apply(feat, graph, self.n_iters, self.n_layers, *self.lstm_params())


class GraphNorm(nn.Module):
    """torch_geometric.nn.GraphNorm (2.2.0).  forward(x, batch=None) normalises over the whole
    input like the reference (model.py:93); ``group_offsets`` (int64[G+1], rows) evaluates many
    reference mini-batches in one launch with independent statistics."""

    def __init__(self, in_channels, eps=1e-5):
        super().__init__()
        self.in_channels = in_channels
        self.eps = eps
        self.weight = nn.Parameter(torch.empty(in_channels))
        self.bias = nn.Parameter(torch.empty(in_channels))
        self.mean_scale = nn.Parameter(torch.empty(in_channels))
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.ones_(self.weight)
        nn.init.zeros_(self.bias)
        nn.init.ones_(self.mean_scale)

    def forward(self, x, batch=None, group_offsets=None):
        if batch is not None:
            raise NotImplementedError("GraphNorm: pass contiguous groups via group_offsets")
        if group_offsets is None:
            group_offsets = torch.tensor([0, x.shape[0]], dtype=torch.int64, device=x.device)
        return Fn.GraphNormFunction.apply(x, self.weight, self.bias, self.mean_scale,
                                          group_offsets, self.eps)


class GNNModule(nn.Module):
    """model.py:77-95 — GAT -> Set2Set -> GraphNorm -> Linear+ReLU+Dropout, on the HIP path.

    forward(graphs, atom_feats): graphs is a BatchedMolGraph already on the GPU, atom_feats
    (N, in_feats) float32 on the same device; returns (B, hidden_feats[-1]).  GraphNorm
    statistics are per ``graphs.group_offsets`` (default: the whole batch, as model.py:93).
    """

    def __init__(self, in_feats=64, hidden_feats=None, dropout=0.2, num_step_set2set=6,
                 num_layer_set2set=3, proj_dtype=None):
        super().__init__()
        if hidden_feats is None:
            raise TypeError("GNNModule needs hidden_feats (the reference indexes hidden_feats[-1])")
        hidden_feats = list(hidden_feats)
        self.conv = GAT(in_feats, hidden_feats)
        self.readout = Set2Set(input_dim=hidden_feats[-1], n_iters=num_step_set2set,
                               n_layers=num_layer_set2set)
        self.norm = GraphNorm(hidden_feats[-1] * 2)
        self.fc = nn.Sequential(nn.Linear(hidden_feats[-1] * 2, hidden_feats[-1]), nn.ReLU(),
                                nn.Dropout(p=dropout))
        self.set_projection_dtype(proj_dtype)

    def set_projection_dtype(self, dtype):
        """GAT projection GEMM precision: None (fp32-accurate, default) or torch.bfloat16
        (bf16 operands on MFMA, fp32 accumulate — BASELINE config 4)."""
        if dtype not in (None, torch.float32, torch.bfloat16):
            raise ValueError("proj_dtype must be None, torch.float32 or torch.bfloat16")
        for layer in self.conv.gnn_layers:
            layer.gat_conv.proj_dtype = None if dtype == torch.float32 else dtype

    def forward(self, graphs, atom_feats):
        node_x = self.conv(graphs, atom_feats)
        graph_x = self.readout(graphs, node_x)
        out = self.norm(graph_x, group_offsets=graphs.group_offsets_rows())
        # fc = Linear -> ReLU -> Dropout (model.py:86-87): the Dropout in place on the ReLU output
        return Fn.LinearReLUFunction.apply(out, self.fc[0].weight, self.fc[0].bias, Fn.dropout_p(self.fc[2]))
