"""mvml_gat_layer_bwd: a GATConv's whole backward as ONE C call, called
through the ctypes handle of libmvml_gat.so with the forward's saved tensors, is BITWISE the
gradient the Python layer (GATLayerFunction.backward: the same launches) gives — for the
flatten + ELU layer on the 74 atom features and the head-mean layer on 768-wide rows."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

import contextlib

from mvml_gat import functional as Fn
from mvml_gat import synth
from mvml_gat._lib import lib, option, ptr, stream_ptr
from mvml_gat.nn import GATLayer

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("layer", [0, 1])
@pytest.mark.parametrize("case", ["config2", "config5"])
def test_gat_layer_bwd_one_call_bitwise(layer, case):
    sb = synth.config2(96, seed=3) if case == "config2" else synth.config5(2, seed=4)
    g = sb.to_graph().to(DEV)
    N, E = g.num_nodes(), g.num_edges()
    torch.manual_seed(layer)
    H = 4
    if layer == 0:
        Fin, Fo = 74, 192
        m = GATLayer(Fin, Fo, H, agg_mode="flatten", activation=F.elu).to(DEV)
        X = torch.as_tensor(sb.feats, dtype=torch.float32, device=DEV)
    else:
        Fin, Fo = 768, 384
        m = GATLayer(Fin, Fo, H, agg_mode="mean").to(DEV)
        X = torch.randn(N, Fin, device=DEV)
    X = X.clone().requires_grad_()
    out = m(g, X)
    Xp, Wcat, Y, attn, elr, outs, attn_l, attn_r, attn_lr = out.grad_fn.saved_tensors
    gout = torch.randn(out.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(9))
    out.backward(gout)
    torch.cuda.synchronize()

    L = lib()
    HF = H * Fo
    wsz = L.mvml_gat_layer_bwd_workspace_size(N, E, H, Fo, Fin, layer)
    ws = torch.empty(max(wsz, 256), dtype=torch.uint8, device=DEV)
    g_X = torch.empty((N, Fin), device=DEV)
    g_fc = torch.empty((HF, Fin), device=DEV)
    g_res = torch.empty((HF, Fin), device=DEV)
    g_attn = torch.empty((2, HF), device=DEV)
    g_bias = torch.empty((HF,), device=DEV)
    # the aggregation backward's kernel choice is a process option (mvml_set_option), as for
    # mvml_gat_agg_bwd: set it the way the Python layer did for this batch
    flat_src = Fn.FLAT_SRC_AUTO and layer == 0 and Fn._large_batch(g)
    with option("flat_src", 2) if flat_src else contextlib.nullcontext():
        rc = L.mvml_gat_layer_bwd(N, ptr(g.node_groups), g.num_node_groups, ptr(g.in_rowptr), ptr(g.in_src),
                                  ptr(g.out_rowptr), ptr(g.out_dst), ptr(g.out_inslot), E, H, Fo, Fin, layer,
                                  ctypes.c_float(0.2), ptr(Xp), ptr(Wcat), ptr(attn_lr), ptr(Y), Y.stride(0),
                                  ptr(elr), ptr(attn), ptr(outs), ptr(gout.contiguous()), ptr(g_X), ptr(g_fc),
                                  ptr(g_res), ptr(g_attn), ptr(g_bias), ptr(ws), ws.numel(), stream_ptr())
    assert rc == 0, L.mvml_last_error().decode()
    torch.cuda.synchronize()
    conv = m.gat_conv
    assert torch.equal(g_X, X.grad)
    assert torch.equal(g_fc, conv.fc.weight.grad)
    assert torch.equal(g_res, conv.res_fc.weight.grad)
    assert torch.equal(g_attn[0], conv.attn_l.grad.reshape(-1))
    assert torch.equal(g_attn[1], conv.attn_r.grad.reshape(-1))
    assert torch.equal(g_bias, conv.bias.grad)


def test_gat_layer_bwd_workspace_checked():
    """A workspace below mvml_gat_layer_bwd_workspace_size is refused (no device work)."""
    L = lib()
    need = L.mvml_gat_layer_bwd_workspace_size(100, 300, 4, 192, 74, 0)
    assert need > 0
    z = torch.zeros(1, device=DEV)
    rc = L.mvml_gat_layer_bwd(100, ptr(z), 1, ptr(z), ptr(z), ptr(z), ptr(z), ptr(z), 300, 4, 192, 74, 0,
                              ctypes.c_float(0.2), ptr(z), ptr(z), ptr(z), ptr(z), 1600, ptr(z), ptr(z), ptr(z),
                              ptr(z), None, ptr(z), ptr(z), ptr(z), ptr(z), ptr(z), need - 1, stream_ptr())
    assert rc == 3, rc
    assert b"workspace too small" in L.mvml_last_error()
