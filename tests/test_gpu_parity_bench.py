"""GPU parity at the bench's OWN sizes: the split-fp16 GEMMs take their
operand scales from batch-global |max| values, so precision must be shown on the batches the
headline runs, not only on 192-molecule ones.  The float64 oracle (oracle/gnn_ref.py,
oracle/fusion_ref.py — the checker, never the product) runs on the GPU here, in chunks of whole
GraphNorm groups: every molecule's GAT / Set2Set / fc rows depend only on its own atoms and its
group, so the chunks' forward values are exactly the whole batch's, and the parameter gradients
(sums over molecules) accumulate across the chunks' autograd passes in float64.

Cases (BASELINE.json configs):
* config 2 as written: single GAT layers 0 (74 -> 4x192, flatten + ELU) and 1 (768 -> 4x384,
  mean) on synth.config2(65536) — 1.64 M atoms, 5.18 M edges; layer 1's input is the
  product's own layer-0 output on the same batch;
* config 3, the bench's first step batch: molecules [0, 65536) of the 1 M-molecule
  synth.Config3Set (1.75 M atoms, 5.41 M edges, 1024 GraphNorm groups of 64) through
  GNNModule -> MVFusion -> BCEWithLogits, forward and every gradient.

Bar (north_star): the flat 1e-5 norm-wise relative error (max |a - b| / max |b|) against
float64 for every output and every gradient, no exception (at this size the Set2Set LSTM bias
gradients, whose sums cancel in small batches, sit at 2.7e-6).  Every tensor's error, the
bar and e32 (what the SAME oracle run in fp32 loses on that tensor) go to
gpurun_out/parity_margins/<case>.json (copied to profiles/r03_parity_margins.json).

Kinks: the product's own fp32 side of every LeakyReLU (GAT logits) and ReLU (GNNModule.fc,
the fusion Conv2d and MLP) is captured from its outputs and the float64 oracle is evaluated on
that side (gnn_ref.leaky_relu_branch / relu_branch); the test asserts that sides disagreeing
with float64 lie within 1e-6 (relative to the tensor's max) of the kink, and are rare.
"""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as TF

from _util import graph_dict, model_pair
from mvml_gat import functional as Fn
from mvml_gat import synth
from oracle import gnn_ref

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 1e-5
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT_DIR = os.environ.get("MVML_MARGINS_DIR", os.path.join(ROOT, "gpurun_out", "parity_margins"))
H = 4


def _rel(a, b):
    """Norm-wise relative error, computed on the GPU in float64."""
    a = a.detach().to(DEV, torch.float64)
    b = b.detach().to(DEV, torch.float64)
    den = b.abs().max().item()
    return (a - b).abs().max().item() / (den if den > 0 else 1.0)


def _write(case, rec):
    os.makedirs(OUT_DIR, exist_ok=True)
    with open(os.path.join(OUT_DIR, case + ".json"), "w") as f:
        json.dump(rec, f, indent=1, sort_keys=True)


def _offsets(sb):
    return (np.concatenate([[0], np.cumsum(sb.num_nodes)]).astype(np.int64),
            np.concatenate([[0], np.cumsum(sb.num_edges)]).astype(np.int64))


def _chunk(sb, noff, m0, m1, group_size):
    """Oracle view of molecules [m0, m1): graph dict (chunk-local ids, on the GPU) and the
    global node range."""
    part = synth.slice_batch(sb, m0, m1)
    gd = graph_dict(part, group_size=group_size)
    for k in ("src", "dst"):
        gd[k] = torch.as_tensor(gd[k], dtype=torch.long, device=DEV)
    return gd, int(noff[m0]), int(noff[m1])


def _leaky_sides(elr, gd, n0):
    """The product's LeakyReLU side per (edge, head) of a chunk: its fp32 (el[src] + er[dst]) > 0."""
    src, dst = gd["src"] + n0, gd["dst"] + n0
    return (elr[src, :H] + elr[dst, H:]) > 0


class _Kinks:
    """Counts sides that disagree with float64 and checks each lies at its kink."""

    def __init__(self):
        self.flips, self.total, self.worst = {}, {}, {}

    def add(self, name, side, pre64):
        with torch.no_grad():
            bad = side != (pre64 > 0)
            n = int(bad.sum())
            self.flips[name] = self.flips.get(name, 0) + n
            self.total[name] = self.total.get(name, 0) + pre64.numel()
            if n:
                w = pre64[bad].abs().max().item() / max(pre64.abs().max().item(), 1e-300)
                self.worst[name] = max(self.worst.get(name, 0.0), w)

    def check(self):
        for name, n in self.flips.items():
            assert self.worst.get(name, 0.0) <= 1e-6, (name, self.worst[name])
            assert n <= max(2, self.total[name] // 10000), (name, n)
        return {k: {"flips": v, "elements": self.total[k], "worst_rel_distance": self.worst.get(k, 0.0)}
                for k, v in self.flips.items()}


def _gat_logits64(X, gd, p, Fo):
    with torch.no_grad():
        Z = (X @ p["fc.weight"].t()).view(X.shape[0], H, Fo)
        el, er = (Z * p["attn_l"]).sum(-1), (Z * p["attn_r"]).sum(-1)
        return el[gd["src"]] + er[gd["dst"]]


def _capture_fwd(fn):
    cap = {}
    Fn.DEBUG_CAPTURE = cap
    try:
        res = fn()
    finally:
        Fn.DEBUG_CAPTURE = None
    return res, cap


# ----------------------------------------------------------------------------- config 2
@pytest.mark.timeout(900)
@pytest.mark.parametrize("layer", [0, 1])
def test_gat_layer_config2_as_written(layer):
    """BASELINE config 2: one GAT layer over all 65,536 molecules in ONE product launch
    sequence, forward + dX + every parameter gradient against float64."""
    n_mols, chunk = 65536, 8192
    sb = synth.config2(n_mols, seed=0)
    noff, _ = _offsets(sb)
    prod, ref = model_pair(seed=20 + layer)
    Fo = 192 if layer == 0 else 384
    mode, act = ("flatten", TF.elu) if layer == 0 else ("mean", None)
    g = sb.to_graph().to(DEV)
    with torch.no_grad():
        X = g.ndata["h"] if layer == 0 else prod.conv.gnn_layers[0].to(DEV)(g, g.ndata["h"])
    X = X.detach().clone()
    conv_p = prod.conv.gnn_layers[layer].to(DEV)
    Xp = X.clone().requires_grad_()
    out_p, cap = _capture_fwd(lambda: conv_p(g, Xp))
    elr = cap["elr_fwd"][0]
    gout = torch.randn(out_p.shape, generator=torch.Generator(device=DEV).manual_seed(7 + layer),
                       device=DEV, dtype=torch.float64)
    out_p.backward(gout.float())
    torch.cuda.synchronize()

    conv_r = ref.conv.gnn_layers[layer].gat_conv
    p64 = {"fc.weight": conv_r.fc.weight, "res_fc.weight": conv_r.res_fc.weight,
           "attn_l": conv_r.attn_l, "attn_r": conv_r.attn_r, "bias": conv_r.bias}
    p64 = {k: v.detach().to(DEV, torch.float64).requires_grad_() for k, v in p64.items()}
    out_r = torch.empty(out_p.shape, dtype=torch.float64, device=DEV)
    gX_r = torch.empty(X.shape, dtype=torch.float64, device=DEV)
    kinks = _Kinks()
    for m0 in range(0, n_mols, chunk):
        m1 = min(n_mols, m0 + chunk)
        gd, n0, n1 = _chunk(sb, noff, m0, m1, None)
        Xc = X[n0:n1].double().requires_grad_()
        side = _leaky_sides(elr, gd, n0)
        kinks.add(f"gat{layer}_leaky", side, _gat_logits64(Xc.detach(), gd, p64, Fo))
        oc = gnn_ref.gat_layer_ref(gd["src"], gd["dst"], Xc, p64, H, Fo, mode, act, branch=side)
        oc.backward(gout[n0:n1])
        out_r[n0:n1] = oc.detach()
        gX_r[n0:n1] = Xc.grad
        del oc, Xc
    c = conv_p.gat_conv
    errs = {"out": _rel(out_p, out_r), "dX": _rel(Xp.grad, gX_r)}
    for name, pp in (("fc.weight", c.fc.weight), ("res_fc.weight", c.res_fc.weight),
                     ("attn_l", c.attn_l), ("attn_r", c.attn_r), ("bias", c.bias)):
        errs[name] = _rel(pp.grad, p64[name].grad)
    rec = {"case": f"config2_layer{layer}", "molecules": n_mols, "atoms": int(X.shape[0]),
           "edges": g.num_edges(), "gemm_algo": Fn.GEMM_ALGO,
           "tensors": {k: {"err": e, "bar": TOL} for k, e in errs.items()},
           "kinks": kinks.check()}
    _write(f"config2_layer{layer}", rec)
    for k, e in errs.items():
        assert e < TOL, (k, e)


# ----------------------------------------------------------------------------- config 3
@pytest.mark.timeout(1200)
def test_gnn_fusion_config3_bench_batch():
    """The bench's first step batch (molecules [0, 65536) of the 1 M-molecule config-3 set,
    1024 GraphNorm groups of 64): GNNModule -> MVFusion -> BCEWithLogits in eval mode, the
    logits, the loss, the two other views' input gradients and EVERY parameter gradient of the
    view and the fusion head against float64 (and fp32, for the conditioning measurement)."""
    sb = synth.Config3Set(1_000_000, seed=0).molecules(0, 65536)
    _gnn_fusion_case(sb, 64, 4096, "config3_bench_batch")


# ----------------------------------------------------------------------------- config 5
@pytest.mark.timeout(1500)
@pytest.mark.parametrize("big_window", [1, 0])
def test_gnn_fusion_config5_bench_batch(big_window):
    """the config-5 bench batch as bench.py builds it (synth.config5(8192,
    seed=1): 150-400-atom molecules with 1-4 hubs of in-degree 32-128, 128 GraphNorm groups of
    64), GNNModule -> MVFusion -> BCE, forward and every gradient against float64, on the
    production kernels (big windows; the head-mean layer's backward by source atom) and on the
    per-atom fallback pair (source-atom backward off)."""
    from mvml_gat._lib import option
    sb = synth.config5(8192, seed=1)
    with option("big_window", big_window), option("mean_src", big_window):
        _gnn_fusion_case(sb, 64, 256, f"config5_bench_batch_bigwindow{big_window}")


def _gnn_fusion_case(sb, gs, chunk, case):
    from mvml_gat import MVFusion, bce_with_logits
    from oracle.fusion_ref import MVFusionRef
    n_mols = sb.batch_size
    noff, _ = _offsets(sb)
    prod, ref = model_pair(seed=31)
    torch.manual_seed(32)
    fref = MVFusionRef(384, 12, 11, 0.5)
    with torch.no_grad():
        fref.norm_layer_module.weight.uniform_(0.5, 1.5)
        fref.norm_layer_module.bias.uniform_(-0.2, 0.2)
    fus = MVFusion(384, 12, 11, 0.5)
    fus.load_state_dict(fref.state_dict())
    prod, fus = prod.to(DEV).eval(), fus.to(DEV).eval()
    gen = torch.Generator(device=DEV).manual_seed(33)
    sx = torch.randn((n_mols, 384), device=DEV, generator=gen)
    fx = torch.randn((n_mols, 384), device=DEV, generator=gen)
    y = (torch.rand((n_mols, 11), device=DEV, generator=gen) > 0.8).float()
    g = sb.to_graph(group_size=gs).to(DEV)
    sxp, fxp = sx.clone().requires_grad_(), fx.clone().requires_grad_()

    def fwd():
        return fus(sxp, prod(g, g.ndata["h"]), fxp)
    z_p, cap = _capture_fwd(fwd)
    loss_p = bce_with_logits(z_p, y)
    loss_p.backward()
    torch.cuda.synchronize()
    elrs = cap["elr_fwd"]
    fc_out, mlp_out = cap["relu_out"]
    conv_out = cap["conv_out"]

    models = {}
    for dt in (torch.float64, torch.float32):
        r = type(ref)(74, [192, 384], 0.5, 6, 3)
        r.load_state_dict(ref.state_dict())
        f = MVFusionRef(384, 12, 11, 0.5)
        f.load_state_dict(fref.state_dict())
        models[dt] = (r.to(DEV, dt).eval(), f.to(DEV, dt).eval())
    kinks = _Kinks()
    # the oracle's nn.LSTM on the GPU would dispatch to MIOpen, whose RNN backward refuses eval
    # mode: the native (aten) LSTM keeps the oracle's semantics and runs its backward in eval
    nocudnn = torch.backends.cudnn.flags(enabled=False)
    nocudnn.__enter__()
    z_r = torch.empty((n_mols, 11), dtype=torch.float64, device=DEV)
    gsx, gfx = {}, {}
    loss_r = {}
    for dt, (r, f) in models.items():
        gsx[dt] = torch.empty((n_mols, 384), dtype=dt, device=DEV)
        gfx[dt] = torch.empty((n_mols, 384), dtype=dt, device=DEV)
        loss_r[dt] = 0.0
        lp = r.layer_params()
        for m0 in range(0, n_mols, chunk):
            m1 = min(n_mols, m0 + chunk)
            gd, n0, n1 = _chunk(sb, noff, m0, m1, gs)
            X = g.ndata["h"][n0:n1].to(dt)
            br = [_leaky_sides(e, gd, n0) for e in elrs]
            fcb, mlpb = fc_out[m0:m1] > 0, mlp_out[m0:m1] > 0
            convb = (conv_out[m0:m1] > 0).unsqueeze(2)
            sxc = sx[m0:m1].to(dt).requires_grad_()
            fxc = fx[m0:m1].to(dt).requires_grad_()
            hooks = {}
            if dt == torch.float64:
                with torch.no_grad():
                    kinks.add("gat0_leaky", br[0], _gat_logits64(X, gd, lp[0], 192))
                    h1 = gnn_ref.gat_layer_ref(gd["src"], gd["dst"], X, lp[0], H, 192, "flatten",
                                               TF.elu, branch=br[0])
                    kinks.add("gat1_leaky", br[1], _gat_logits64(h1, gd, lp[1], 384))
                    del h1
                for name, mod in (("gnn_fc_relu", r.fc[0]), ("conv_relu", f.conv[0]),
                                  ("mlp_relu", f.mlp[0])):
                    mod.register_forward_hook(lambda m, i, o, name=name: hooks.__setitem__(name, o.detach()))
            out = r(gd, X, branches=br, fc_branch=fcb)
            zc = f(sxc, out, fxc, conv_branch=convb, mlp_branch=mlpb)
            lc = TF.binary_cross_entropy_with_logits(zc, y[m0:m1].to(dt), reduction="sum") / (n_mols * 11)
            lc.backward()
            loss_r[dt] += lc.item()
            gsx[dt][m0:m1] = sxc.grad
            gfx[dt][m0:m1] = fxc.grad
            if dt == torch.float64:
                z_r[m0:m1] = zc.detach()
                kinks.add("gnn_fc_relu", fcb, hooks["gnn_fc_relu"])
                kinks.add("conv_relu", convb, hooks["conv_relu"])
                kinks.add("mlp_relu", mlpb, hooks["mlp_relu"])
                for mod in (r.fc[0], f.conv[0], f.mlp[0]):
                    mod._forward_hooks.clear()
            del out, zc, lc
    nocudnn.__exit__(None, None, None)
    (r64, f64), (r32, f32) = models[torch.float64], models[torch.float32]
    tensors = {"logits": {"err": _rel(z_p, z_r), "bar": TOL},
               "loss": {"err": abs(loss_p.item() - loss_r[torch.float64]) / abs(loss_r[torch.float64]),
                        "bar": TOL},
               "d_smiles_x": {"err": _rel(sxp.grad, gsx[torch.float64]), "bar": TOL},
               "d_fp_x": {"err": _rel(fxp.grad, gfx[torch.float64]), "bar": TOL}}
    for prefix, pm, m64, m32 in (("gnn.", prod, r64, r32), ("fusion.", fus, f64, f32)):
        p64, p32 = dict(m64.named_parameters()), dict(m32.named_parameters())
        for n, p in pm.named_parameters():
            if p.grad is None:
                assert p64[n].grad is None, n  # the unused norm_layer (model.py:39)
                continue
            e = _rel(p.grad, p64[n].grad)
            e32 = _rel(p32[n].grad, p64[n].grad)
            tensors[prefix + n] = {"err": e, "bar": TOL, "e32": e32}
    rec = {"case": case, "molecules": n_mols, "atoms": g.num_nodes(),
           "edges": g.num_edges(), "graphnorm_groups": n_mols // gs, "gemm_algo": Fn.GEMM_ALGO,
           "row_scales": Fn.ROW_SCALES, "tensors": tensors, "kinks": kinks.check()}
    _write(case, rec)
    for n, t in tensors.items():
        assert t["err"] < t["bar"], (n, t)
