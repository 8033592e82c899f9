"""Multi-view attention fusion head of MVP (model.py:23, 27-48, 54-72) on the HIP path — the
consumer of the graph view.

    MVFusion(final_hidden_feats=384, num_heads=12, num_classes=11, dropout)(smiles_x, graph_x, fp_x)

takes the three RAW view embeddings (B, 384) (what MVP gets from RNNModule, GNNModule and
FPNModule before its shared LayerNorm, model.py:54-56) and returns the logits (B, num_classes)
of model.py:72.  Parameter names / shapes equal MVP's, so ``MVP.state_dict()`` entries under
``norm_layer_module.``, ``conv.``, ``linear_{q,k,v}.``, ``norm_layer.``, ``mlp.`` load unchanged.
``bce_with_logits`` is main.py:91's BCEWithLogitsLoss.
"""
import math
import os

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from ._lib import call, ptr
from . import functional as _F
from .functional import (LinearReLUFunction, _c, _check_cuda_f32, _stream, absmax, colsum, gemm, slot,
                         gemm_batched)


class LinearFunction(torch.autograd.Function):
    """nn.Linear (model.py:44, the classifier) as one MFMA GEMM with a bias epilogue."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        _check_cuda_f32(x, "x")
        x = _c(x)
        M, K = x.shape
        Nout = weight.shape[0]
        y = torch.empty((M, Nout), dtype=torch.float32, device=x.device)
        weight = _c(weight)
        lm = ctx.lm = _F.linear_maxima(x, weight)
        _F.linear_fwd(x, weight, y, M, Nout, K, lm, bias=_c(bias))
        ctx.save_for_backward(x, weight)
        return y

    @staticmethod
    def backward(ctx, g_y):
        x, weight = ctx.saved_tensors
        g_y = _c(g_y)
        M, K = x.shape
        Nout = weight.shape[0]
        lm = ctx.lm
        if lm is not None:
            absmax(g_y, M, Nout, Nout, lm[0], 2)
        gw = torch.empty_like(weight)
        gemm(g_y, x, Nout, K, M, 1, 1, Nout, K, gw, K,
             amax=None if lm is None else (slot(lm[0], 2), slot(*lm[1])))
        gb = torch.empty((Nout,), dtype=torch.float32, device=x.device)
        colsum(g_y, M, Nout, Nout, gb)
        gx = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            _F.linear_dx(g_y, weight, gx, M, Nout, K, lm)
        return gx, gw, gb


# Q.K re-associated (mvml_token_attn_fold_*): s = (x M_h) . x with M_h = W_q,h^T W_k,h, so the
# token GEMMs run over 2 H D columns (P, V) instead of 3 H D (Q, K, V) in the forward, the data
# gradient and the weight gradient; False = the literal Q / K / V path (kept, tested).
FOLD_QK = True
# With FOLD_QK: the token attention and the Conv2d + ReLU run as ONE kernel each way
# (mvml_attn_conv_fwd / _bwd), the (B, 12, 3, 384) attention cube never leaves LDS; False = the
# separate mvml_token_attn_fold_* and mvml_conv3_* launches (kept, tested).
FUSE_ATTN_CONV = os.environ.get("MVML_FUSE_ATTN_CONV", "1") != "0"


def attn_conv_bytes(B, H, D, backward):
    """Algorithmic HBM bytes of mvml_attn_conv_fwd / _bwd (fp32): the forward reads pv (3 rows
    x 2 H D) and the keys (3 x D), writes P (H x 9) and the Conv2d output (H x (D - 2)) per
    molecule; the backward reads pv, the keys, P, the output and its gradient, writes g_pv and
    g_k.  The (H, 3, D) attention cube is on chip both ways (counted 0)."""
    pv, keys, p, out = 3 * 2 * H * D, 3 * D, H * 9, H * (D - 2)
    per = (pv + keys + p + out) if not backward else (2 * pv + 2 * keys + p + 2 * out)
    return 4 * B * per


class FusionAttnConvFunction(torch.autograd.Function):
    """model.py:54-71 up to the Conv2d+ReLU: shared LayerNorm of the three views, Q/K/V (one
    GEMM over the concatenated [W_q; W_k; W_v]), 3-token attention per head, Conv2d(nh, nh, 3)
    + ReLU.  Returns (B, nh * (dim - 2)) like ``self.conv(att).view(B, -1)`` before Dropout."""

    @staticmethod
    def forward(ctx, smiles_x, graph_x, fp_x, ln_w, ln_b, wq, wk, wv, conv_w, conv_b, eps, p=0.0):
        for t, n in ((smiles_x, "smiles_x"), (graph_x, "graph_x"), (fp_x, "fp_x")):
            _check_cuda_f32(t, n)
        B, D = graph_x.shape
        H = wq.shape[0] // D
        dev = graph_x.device
        st = _stream(dev)
        f32 = dict(dtype=torch.float32, device=dev)
        # the shared LayerNorm, one launch per view, each writing its rows 3b+t of Xn (no stacked
        # copy of the three embeddings; the backward returns each view's gradient contiguous)
        views = [_c(smiles_x), _c(graph_x), _c(fp_x)]
        Xn = torch.empty((3 * B, D), **f32)
        Xn3 = Xn.view(B, 3, D)
        mean = torch.empty((3, B), **f32)
        rstd = torch.empty((3, B), **f32)
        for t, xt in enumerate(views):
            call("mvml_layernorm_fwd", B, D, ptr(xt), D, ptr(_c(ln_w)), ptr(_c(ln_b)), float(eps),
                 ptr(Xn3[:, t]), 3 * D, ptr(mean[t]), ptr(rstd[t]), st)
        P = torch.empty((B, H, 3, 3), **f32)
        scale = 1.0 / math.sqrt(D)
        HD = H * D
        fold = FOLD_QK
        fused = fold and FUSE_ATTN_CONV
        att = None if fused else torch.empty((B, H, 3, D), **f32)
        out = torch.empty((B, H, D - 2), **f32)
        if fold:
            wq3, wk3 = _c(wq).view(H, D, D), _c(wk).view(H, D, D)
            # Bcat [D, 2 H D] = [M_1 .. M_H | W_v^T]: M_h[i][j] = sum_o Wq_h[o][i] Wk_h[o][j]
            Bcat = torch.empty((D, 2 * HD), **f32)
            gemm_batched(wq3, wk3, D, D, D, 1, 1, D, D, Bcat, 2 * HD, H, D * D, D * D, D)
            # W_v^T into Bcat's right half: parameter layout (7 MB), not a product
            call("mvml_transpose", HD, D, ptr(_c(wv)), D, ptr(Bcat[:, HD:]), 2 * HD, st)
            PV = torch.empty((3 * B, 2 * HD), **f32)  # rows 3b+t: [x M_1 .. x M_H | x W_v^T]
            if _F.GEMM_ALGO == "f16x2" and _F.ROW_SCALES:  # every token row at its own scale
                bmx = _F.zeros(1, dtype=torch.int32, device=dev)
                absmax(Bcat, D, 2 * HD, 2 * HD, bmx, 0)
                gemm(Xn, Bcat, 3 * B, 2 * HD, D, 0, 1, D, 2 * HD, PV, 2 * HD, amax=(None, slot(bmx, 0)),
                     arows=_F.absmax_rows(Xn, 3 * B, D, D),
                     bil4=_F.split_il4(Bcat, D, 2 * HD, 2 * HD, slot(bmx, 0)))
            else:
                gemm(Xn, Bcat, 3 * B, 2 * HD, D, 0, 1, D, 2 * HD, PV, 2 * HD)
            if fused:
                # the Dropout after the ReLU (model.py:36) in the kernel's store (the parity tests'
                # ReLU-side capture needs the undropped output: then it runs separately below)
                fp = p if (p > 0.0 and _F.DEBUG_CAPTURE is None) else 0.0
                _lib.call_tag[0] = {"bytes": attn_conv_bytes(B, H, D, False)}
                call("mvml_attn_conv_fwd", B, H, D, ptr(PV), 2 * HD, ptr(Xn), D, float(scale),
                     ptr(_c(conv_w)), ptr(_c(conv_b)), ptr(P), ptr(out), float(fp),
                     _F.dropout_seed() if fp > 0.0 else 0, st)
                if fp > 0.0:
                    p = 0.0
                    ctx.g_scale = float(np.float32(1.0 / (1.0 - fp)))
            else:
                call("mvml_token_attn_fold_fwd", B, H, D, ptr(PV), 2 * HD, ptr(Xn), D, float(scale),
                     ptr(att), ptr(P), st)
            saved = (Bcat, PV)
        else:
            Wqkv = torch.cat([_c(wq), _c(wk), _c(wv)], dim=0)  # (3 H D, D)
            QKV = torch.empty((3 * B, 3 * HD), **f32)
            gemm(Xn, Wqkv, 3 * B, 3 * HD, D, 0, 0, D, D, QKV, 3 * HD)
            call("mvml_token_attn_fwd", B, H, D, ptr(QKV), 3 * HD, float(scale), ptr(att), ptr(P), st)
            saved = (Wqkv, QKV)
        if not fused:
            call("mvml_conv3_fwd", B, H, H, D, ptr(att), ptr(_c(conv_w)), ptr(_c(conv_b)), ptr(out), st)
        if _F.DEBUG_CAPTURE is not None:  # the ReLU sides the product took (parity tests)
            _F.DEBUG_CAPTURE["conv_out"] = out.detach().clone()
        # the Dropout after the ReLU (model.py:36), in place where the kernel did not apply it:
        # the backward needs no mask either way
        if p > 0.0 or not hasattr(ctx, "g_scale"):
            ctx.g_scale = _F.relu_dropout_(out, p)
        ctx.save_for_backward(*views, Xn, mean, rstd, ln_w, wq, wk, wv, *saved, P, att, out, conv_w)
        ctx.dims = (B, D, H, scale, fold, fused)
        return out.view(B, H * (D - 2))

    @staticmethod
    def backward(ctx, g_out):
        x0, x1, x2, Xn, mean, rstd, ln_w, wq, wk, wv, S0, S1, P, att, out, conv_w = ctx.saved_tensors
        views = (x0, x1, x2)
        B, D, H, scale, fold, fused = ctx.dims
        dev = x0.device
        st = _stream(dev)
        f32 = dict(dtype=torch.float32, device=dev)
        L = _lib.lib()
        g_out = _c(g_out)
        g_cw = torch.empty_like(conv_w)
        g_cb = torch.empty((H,), **f32)
        if not fused:
            g_att = torch.empty_like(att)
            wp, wn = _lib.ws_ptr_size(L.mvml_conv3_bwd_workspace_size(B), dev)
            call("mvml_conv3_bwd", B, H, H, D, ptr(att), ptr(_c(conv_w)), ptr(out), ptr(g_out),
                 ptr(g_att), ptr(g_cw), ptr(g_cb), wp, wn, st)
        HD = H * D
        gXn = torch.empty((3 * B, D), **f32)
        if fold:
            Bcat, PV = S0, S1
            gPV = torch.empty((3 * B, 2 * HD), **f32)
            amx = None
            if _F.GEMM_ALGO == "f16x2":  # split-fp16 maxima: gPV (folded by the kernel), Xn, Bcat
                amx = _F.zeros(3, dtype=torch.int32, device=dev)
            # g_k (the keys' gradient, summed over heads) lands in gXn: the GEMMs add onto it
            # per-row |gPV| maxima for the data-gradient product (folded by the fused kernel)
            gpr = None
            if amx is not None and _F.ROW_SCALES:
                gpr = _F.zeros(3 * B, dtype=torch.int32, device=dev)
            if fused:
                wp, wn = _lib.ws_ptr_size(L.mvml_attn_conv_bwd_workspace_size(B), dev)
                _lib.call_tag[0] = {"bytes": attn_conv_bytes(B, H, D, True)}
                call("mvml_attn_conv_bwd", B, H, D, ptr(PV), 2 * HD, ptr(Xn), D, float(scale),
                     ptr(P), ptr(_c(conv_w)), ptr(out), ptr(g_out), float(ctx.g_scale), ptr(gPV), 2 * HD,
                     ptr(gXn), D,
                     slot(amx, 0), ptr(gpr), ptr(g_cw), ptr(g_cb), wp, wn, st)
            else:
                call("mvml_token_attn_fold_bwd", B, H, D, ptr(PV), 2 * HD, ptr(Xn), D, float(scale),
                     ptr(P), ptr(g_att), ptr(gPV), 2 * HD, ptr(gXn), D, slot(amx, 0), st)
                if gpr is not None:
                    _F.absmax_rows(gPV, 3 * B, 2 * HD, 2 * HD, gpr)
            if amx is not None:
                absmax(Xn, 3 * B, D, D, amx, 1)
                if _F.DEBUG_CAPTURE is not None:
                    _F.DEBUG_CAPTURE["gpv_amax"] = (gPV.clone(), amx[0:1].clone())
                absmax(Bcat, D, 2 * HD, 2 * HD, amx, 2)
                bil = _F.split_il4(Bcat, D, 2 * HD, 2 * HD, slot(amx, 2))
            G2 = torch.empty((2 * HD, D), **f32)  # [h D + j][i] = dL/dM_h[i][j]; then dL/dW_v
            gemm(gPV, Xn, 2 * HD, D, 3 * B, 1, 1, 2 * HD, D, G2, D,
                 amax=None if amx is None else (slot(amx, 0), slot(amx, 1)))
            wq3, wk3 = _c(wq).view(H, D, D), _c(wk).view(H, D, D)
            gWq = torch.empty((H, D, D), **f32)
            gWk = torch.empty((H, D, D), **f32)
            # per head h (G2 rows h D .. h D + D): W_k,h dM_h^T and W_q,h dM_h
            gemm_batched(wk3, G2, D, D, D, 0, 1, D, D, gWq, D, H, D * D, D * D, D * D)
            gemm_batched(wq3, G2, D, D, D, 0, 0, D, D, gWk, D, H, D * D, D * D, D * D)
            if amx is not None and _F.ROW_SCALES:  # every token row's gradient at its own scale
                gemm(gPV, Bcat, 3 * B, D, 2 * HD, 0, 0, 2 * HD, 2 * HD, gXn, D, beta=1.0,
                     amax=(None, slot(amx, 2)), arows=gpr, bil4=bil)
            else:
                gemm(gPV, Bcat, 3 * B, D, 2 * HD, 0, 0, 2 * HD, 2 * HD, gXn, D, beta=1.0,
                     amax=None if amx is None else (slot(amx, 0), slot(amx, 2)))
            g_wq, g_wk, g_wv = gWq.view(HD, D), gWk.view(HD, D), G2[HD:]
        else:
            Wqkv, QKV = S0, S1
            gQKV = torch.empty((3 * B, 3 * HD), **f32)
            call("mvml_token_attn_bwd", B, H, D, ptr(QKV), 3 * HD, float(scale), ptr(P), ptr(g_att),
                 ptr(gQKV), 3 * HD, st)
            gW = torch.empty_like(Wqkv)
            gemm(gQKV, Xn, 3 * HD, D, 3 * B, 1, 1, 3 * HD, D, gW, D)
            gemm(gQKV, Wqkv, 3 * B, D, 3 * HD, 0, 1, 3 * HD, D, gXn, D)
            g_wq, g_wk, g_wv = gW[:HD], gW[HD:2 * HD], gW[2 * HD:]
        gXn3 = gXn.view(B, 3, D)
        gyxh = torch.empty((3, B, D), **f32)
        gX = []
        for t, xt in enumerate(views):
            gX.append(torch.empty((B, D), **f32))
            call("mvml_layernorm_bwd", B, D, ptr(xt), D, ptr(_c(ln_w)), ptr(mean[t]), ptr(rstd[t]),
                 ptr(gXn3[:, t]), 3 * D, ptr(gX[t]), D, ptr(gyxh[t]), st)
        g_lnw = torch.empty((D,), **f32)
        g_lnb = torch.empty((D,), **f32)
        colsum(gyxh, 3 * B, D, D, g_lnw)
        colsum(gXn, 3 * B, D, D, g_lnb)
        return (gX[0], gX[1], gX[2], g_lnw, g_lnb, g_wq, g_wk, g_wv, g_cw, g_cb, None, None)


class BCEWithLogitsFunction(torch.autograd.Function):
    """torch.nn.BCEWithLogitsLoss() (mean), main.py:91."""

    @staticmethod
    def forward(ctx, logits, labels):
        _check_cuda_f32(logits, "logits")
        z, y = _c(logits), _c(labels.float())
        terms = torch.empty_like(z)
        gz = torch.empty_like(z)
        n = z.numel()
        call("mvml_bce_logits", n, ptr(z), ptr(y), ptr(terms), ptr(gz), _stream(z.device))
        ctx.save_for_backward(gz)
        loss = torch.empty((1,), dtype=torch.float32, device=z.device)
        colsum(terms, n, 1, 1, loss, alpha=1.0 / n)  # the mean, one native column sum
        return loss.view(())

    @staticmethod
    def backward(ctx, g):
        (gz,) = ctx.saved_tensors
        out = torch.empty_like(gz)
        call("mvml_scale_by", gz.numel(), ptr(gz), ptr(_c(g)), ptr(out), _stream(gz.device))
        return out, None


def bce_with_logits(logits, labels):
    return BCEWithLogitsFunction.apply(logits, labels)


class MVFusion(nn.Module):
    """The fusion part of MVP (model.py:23, 27-48, 54-72) with MVP's parameter names."""

    def __init__(self, final_hidden_feats=384, num_heads=12, num_classes=11, dropout=0.2):
        super().__init__()
        if final_hidden_feats != 384 or num_heads != 12:
            raise ValueError(
                "the HIP fusion kernels are built for the reference configuration (config.py: "
                f"hidden_feats[-1] = 384, head = 12); got {final_hidden_feats} / {num_heads}")
        d = final_hidden_feats
        self.final_hidden_feats, self.num_heads = d, num_heads
        self.norm_layer_module = nn.LayerNorm(d)
        self.conv = nn.Sequential(nn.Conv2d(num_heads, num_heads, kernel_size=3), nn.ReLU(),
                                  nn.Dropout(dropout))
        self.dim_in, self.dim_k, self.dim_v = d, d * num_heads, d * num_heads
        self.linear_q = nn.Linear(d, self.dim_k, bias=False)
        self.linear_k = nn.Linear(d, self.dim_k, bias=False)
        self.linear_v = nn.Linear(d, self.dim_v, bias=False)
        self._norm_fact = 1 / math.sqrt(self.dim_k // num_heads)
        self.norm_layer = nn.LayerNorm((d - 2) * num_heads)  # constructed, unused (model.py:39)
        self.mlp = nn.Sequential(nn.Linear((d - 2) * num_heads, 1024), nn.ReLU(), nn.Dropout(dropout),
                                 nn.Linear(1024, num_classes))

    def forward(self, smiles_x, graph_x, fp_x):
        ln = self.norm_layer_module
        out = FusionAttnConvFunction.apply(smiles_x, graph_x, fp_x, ln.weight, ln.bias,
                                           self.linear_q.weight, self.linear_k.weight,
                                           self.linear_v.weight, self.conv[0].weight,
                                           self.conv[0].bias, ln.eps, _F.dropout_p(self.conv[2]))
        # conv = Conv2d -> ReLU -> Dropout, mlp = Linear -> ReLU -> Dropout -> Linear: each
        # Dropout in place on its ReLU output (mvml_dropout_fwd; the backward needs no mask)
        out = LinearReLUFunction.apply(out, self.mlp[0].weight, self.mlp[0].bias, _F.dropout_p(self.mlp[2]))
        return LinearFunction.apply(out, self.mlp[3].weight, self.mlp[3].bias)


class FPNModule(nn.Module):
    """The fingerprint view's MLP, model.py:138-155, on the HIP GEMMs:
    fc1 (2513 -> fp_2_dim) -> Dropout -> ReLU -> fc2 (-> out_feats), parameter names as in the
    reference.  fc1 + ReLU run as one GEMM with a bias+ReLU epilogue and the Dropout follows,
    in place: ReLU(mask * z / (1-p)) == mask * ReLU(z) / (1-p) exactly, and the mask is drawn
    for the same shape, so this equals the reference order.  The 2513-bit fingerprints themselves (MACCS,
    ErG, PubChem, Morgan; dataset.py:37-45) need RDKit and are out of scope."""

    def __init__(self, fp_2_dim, out_feats, dropout=0.2):
        super().__init__()
        self.fp_2_dim = fp_2_dim
        self.dropout_fpn = dropout
        self.out_feats = out_feats
        self.fp_dim = 2513
        self.fc1 = nn.Linear(self.fp_dim, self.fp_2_dim)
        self.act_func = nn.ReLU()
        self.fc2 = nn.Linear(self.fp_2_dim, self.out_feats)
        self.dropout = nn.Dropout(p=self.dropout_fpn)

    def forward(self, fp):
        h = LinearReLUFunction.apply(fp, self.fc1.weight, self.fc1.bias, _F.dropout_p(self.dropout))
        return LinearFunction.apply(h, self.fc2.weight, self.fc2.bias)
