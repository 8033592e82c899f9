"""GPU parity of the multi-view fusion head (model.py:28-48, 57-72) and
BCEWithLogitsLoss (main.py:91): the HIP path (through the C ABI) against the float64 CPU
restatement oracle/fusion_ref.py on identical seeded weights and inputs.

Bar: fp32 outputs and gradients within 1e-5 norm-wise relative error (TOL)."""
import math

import pytest
import torch

from conftest import rel_err
from oracle.fusion_ref import MVFusionRef, bce_logits_ref

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 1e-5


def _pair(B, seed=0, dim=384, heads=12, classes=11):
    """Natural (unshifted) biases everywhere: with ~10^5 ReLU inputs an fp32 pre-activation
    within rounding of 0 can take a different side than fp64's, and that one kink moves a
    gradient by O(1) — a property of ReLU, not of the kernels — so the parity test evaluates the
    float64 oracle on the product's own side of every ReLU (_relu_sides)."""
    from mvml_gat import MVFusion
    torch.manual_seed(seed)
    ref = MVFusionRef(dim, heads, classes, dropout=0.5).double().eval()
    with torch.no_grad():  # non-trivial LayerNorm affine parameters
        ref.norm_layer_module.weight.uniform_(0.5, 1.5)
        ref.norm_layer_module.bias.uniform_(-0.2, 0.2)
    mod = MVFusion(dim, heads, classes, dropout=0.5).to(DEV).eval()
    mod.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    g = torch.Generator().manual_seed(seed + 1)
    xs = [torch.randn(B, dim, generator=g, dtype=torch.float64) * s for s in (1.0, 0.3, 2.0)]
    return ref, mod, xs


def _relu_sides(mod, xd):
    """Run the product forward with the kink capture on: (logits, conv side, MLP side) — the
    sides its fp32 arithmetic took, read off its post-ReLU outputs (> 0)."""
    from mvml_gat import functional as Fn
    cap = {}
    Fn.DEBUG_CAPTURE = cap
    try:
        zd = mod(*xd)
    finally:
        Fn.DEBUG_CAPTURE = None
    conv = (cap["conv_out"] > 0).unsqueeze(2).cpu()
    mlp = (cap["relu_out"][-1] > 0).cpu()
    return zd, conv, mlp


def _check_relu_flips(ref, xr, conv, mlp):
    """Sides that differ from float64's own must be at the kink (|pre| <= 1e-6 of the max)."""
    pre = {}
    hs = [ref.conv[0].register_forward_hook(lambda m, i, o: pre.__setitem__("conv", o.detach())),
          ref.mlp[0].register_forward_hook(lambda m, i, o: pre.__setitem__("mlp", o.detach()))]
    with torch.no_grad():
        ref(*xr, conv_branch=conv, mlp_branch=mlp)
    for h in hs:
        h.remove()
    flips = 0
    for side, p in ((conv, pre["conv"]), (mlp, pre["mlp"])):
        bad = side != (p > 0)
        flips += int(bad.sum())
        if bad.any():
            assert p[bad].abs().max().item() <= 1e-6 * p.abs().max().item()
        assert int(bad.sum()) <= max(2, p.numel() // 10000)
    return flips


@pytest.mark.parametrize("path", ["fused", "fold", "qkv"])
@pytest.mark.parametrize("B", [1, 5, 64, 300, 2048])
def test_fusion_forward_backward_parity(B, path, monkeypatch):
    """fused: Q.K re-associated, attention + Conv2d in one kernel each way (mvml_attn_conv_*,
    the default); fold: the same with separate mvml_token_attn_fold_* / mvml_conv3_* launches;
    qkv: the literal Q / K / V GEMM + mvml_token_attn_*.  Natural biases: both ReLUs see both
    branches (the zeroed one drives the conv backward's and relu_bwd's masking), the oracle
    follows the product's side at each kink."""
    import mvml_gat.fusion as fu
    monkeypatch.setattr(fu, "FOLD_QK", path != "qkv")
    monkeypatch.setattr(fu, "FUSE_ATTN_CONV", path == "fused")
    ref, mod, xs = _pair(B, seed=B)
    xr = [x.clone().requires_grad_(True) for x in xs]
    xd = [x.float().to(DEV).requires_grad_(True) for x in xs]
    zd, conv, mlp = _relu_sides(mod, xd)
    # both branches of both ReLUs are exercised
    if B >= 64:
        for side in (conv, mlp):
            frac = side.double().mean().item()
            assert 0.05 < frac < 0.95, frac
    _check_relu_flips(ref, [x.detach() for x in xr], conv, mlp)
    zr = ref(*xr, conv_branch=conv, mlp_branch=mlp)
    assert rel_err(zd, zr) < TOL
    up = torch.randn(zr.shape, generator=torch.Generator().manual_seed(7), dtype=torch.float64)
    (zr * up).sum().backward()
    (zd * up.float().to(DEV)).sum().backward()
    for a, b in zip(xd, xr):
        assert rel_err(a.grad, b.grad) < TOL
    pr = dict(ref.named_parameters())
    bars = {}
    if B >= 2048:  # the named cancellation case, measured: fp32 itself loses > 1e-6 there
        bars["conv.0.bias"] = _cancellation_bar(ref, xs, conv, mlp, up, "conv.0.bias")
    for name, p in mod.named_parameters():
        if name.startswith("norm_layer."):
            assert p.grad is None  # constructed but unused, as in the reference
            continue
        assert rel_err(p.grad, pr[name].grad) < bars.get(name, TOL), name


def _cancellation_bar(ref64, xs, conv, mlp, up, name):
    """Conv2d bias gradient = sum over B x 382 x 12 upstream elements whose signs are random:
    at B = 2048 the sum is ~10^3 times smaller than the sum of magnitudes, so the rounding of
    each fp32 upstream element (Linear backward) adds up past 1e-5 of the result — in any fp32
    implementation.  The bar is max(1e-5, 4 x e32), e32 = the SAME oracle in fp32 against fp64,
    and e32 must really be large (the exception is the batch's, not the kernel's)."""
    ref32 = MVFusionRef(384, 12, 11, dropout=0.5).eval()
    ref32.load_state_dict({k: v.float() for k, v in ref64.state_dict().items()})
    xr = [x.float().requires_grad_(True) for x in xs]
    z = ref32(*xr, conv_branch=conv, mlp_branch=mlp)
    (z * up.float()).sum().backward()
    e32 = rel_err(dict(ref32.named_parameters())[name].grad, dict(ref64.named_parameters())[name].grad)
    assert e32 > 1e-6, e32
    return max(TOL, 4 * e32)


def test_bce_with_logits_parity():
    from mvml_gat import bce_with_logits
    g = torch.Generator().manual_seed(3)
    z = torch.randn(300, 11, generator=g, dtype=torch.float64) * 4
    y = (torch.rand(300, 11, generator=g) > 0.5).double()
    zr = z.clone().requires_grad_(True)
    lr = bce_logits_ref(zr, y)
    lr.backward()
    zd = z.float().to(DEV).requires_grad_(True)
    ld = bce_with_logits(zd, y.float().to(DEV))
    ld.backward()
    assert abs(ld.item() - lr.item()) <= TOL * abs(lr.item())
    assert rel_err(zd.grad, zr.grad) < TOL


@pytest.mark.parametrize("W", [3, 17, 384])
def test_conv3_kernel_edges(W):
    """Conv2d(12, 12, 3)+ReLU kernel and its backward at the narrowest / odd / full widths."""
    from mvml_gat._lib import call, lib, ptr, ws_ptr_size
    g = torch.Generator().manual_seed(W)
    B = 7
    x = torch.randn(B, 12, 3, W, generator=g, dtype=torch.float64)
    w = torch.randn(12, 12, 3, 3, generator=g, dtype=torch.float64) * 0.2
    b = torch.randn(12, generator=g, dtype=torch.float64) * 0.1
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = torch.relu(torch.nn.functional.conv2d(xr, wr, br)).view(B, 12, W - 2)
    gy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    (yr * gy).sum().backward()
    xd, wd, bd, gyd = (t.float().to(DEV).contiguous() for t in (x, w, b, gy))
    yd = torch.empty(B, 12, W - 2, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    call("mvml_conv3_fwd", B, 12, 12, W, ptr(xd), ptr(wd), ptr(bd), ptr(yd), st)
    assert rel_err(yd, yr) < TOL
    gx, gw, gb = torch.empty_like(xd), torch.empty_like(wd), torch.empty_like(bd)
    wp, wn = ws_ptr_size(lib().mvml_conv3_bwd_workspace_size(B), DEV)
    call("mvml_conv3_bwd", B, 12, 12, W, ptr(xd), ptr(wd), ptr(yd), ptr(gyd), ptr(gx), ptr(gw),
         ptr(gb), wp, wn, st)
    assert rel_err(gx, xr.grad) < TOL
    assert rel_err(gw, wr.grad) < TOL
    assert rel_err(gb, br.grad) < TOL


def test_fusion_deterministic_bitwise():
    _, mod, xs = _pair(33, seed=11)
    outs = []
    for _ in range(2):
        xd = [x.float().to(DEV).requires_grad_(True) for x in xs]
        mod.zero_grad()
        z = mod(*xd)
        z.sum().backward()
        outs.append([z.detach().clone()] + [x.grad.clone() for x in xd] +
                    [p.grad.clone() for n, p in mod.named_parameters() if p.grad is not None])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B", [1, 64, 300])
def test_fpn_module_parity(B):
    """Fingerprint-view MLP (model.py:138-155): 2513 fingerprint bits -> 128 -> 384, eval mode,
    forward and gradients against the float64 restatement."""
    from mvml_gat import FPNModule
    from oracle.fusion_ref import FPNModuleRef
    torch.manual_seed(B)
    ref = FPNModuleRef(128, 384, 0.5).double().eval()
    mod = FPNModule(128, 384, 0.5).to(DEV).eval()
    mod.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    g = torch.Generator().manual_seed(B + 1)
    fp = (torch.rand(B, 2513, generator=g) > 0.7).double()
    fp[:, 167:608] = torch.rand(B, 441, generator=g, dtype=torch.float64) * 3  # ErG block: real-valued
    xr = fp.clone().requires_grad_(True)
    xd = fp.float().to(DEV).requires_grad_(True)
    zr, zd = ref(xr), mod(xd)
    assert rel_err(zd, zr) < TOL
    up = torch.randn(zr.shape, generator=g, dtype=torch.float64)
    (zr * up).sum().backward()
    (zd * up.float().to(DEV)).sum().backward()
    assert rel_err(xd.grad, xr.grad) < TOL
    pr = dict(ref.named_parameters())
    for name, p in mod.named_parameters():
        assert rel_err(p.grad, pr[name].grad) < TOL, name


@pytest.mark.parametrize("B", [5, 1000])
def test_fusion_fold_bwd_gpv_max(B):
    """mvml_token_attn_fold_bwd folds max |g_pv| (the split-fp16 scale of the two GEMMs that
    read it) into its stores: equal to the max of the tensor it wrote."""
    from mvml_gat import functional as Fn
    if Fn.GEMM_ALGO != "f16x2":
        pytest.skip("the folded max feeds the split-fp16 GEMMs only")
    _, mod, xs = _pair(B, seed=3)
    xd = [x.float().to(DEV).requires_grad_(True) for x in xs]
    cap = {}
    Fn.DEBUG_CAPTURE = cap
    try:
        mod(*xd).sum().backward()
        torch.cuda.synchronize()
    finally:
        Fn.DEBUG_CAPTURE = None
    gpv, amx = cap["gpv_amax"]
    got = amx.cpu().view(torch.float32).item()
    assert got == gpv.abs().max().item() and got > 0


@pytest.mark.parametrize("B", [1, 300, 2048])
def test_attn_conv_fused_matches_unfused(B, monkeypatch):
    """mvml_attn_conv_fwd / _bwd against the separate fold-attention + conv3 launches: the
    logits, every input gradient and the Q / K / V weight gradients bit-identical (same cube,
    same attention arithmetic, same head order of the keys' gradient sum); the Conv2d weight /
    bias gradients (different summation order of the column sums) within 1e-5."""
    import mvml_gat.fusion as fu
    _, mod, xs = _pair(B, seed=5)
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(fu, "FUSE_ATTN_CONV", fused)
        mod.zero_grad()
        xd = [x.float().to(DEV).requires_grad_(True) for x in xs]
        z = mod(*xd)
        (z * torch.linspace(-1, 1, z.numel(), device=DEV).view(z.shape)).sum().backward()
        res[fused] = (z.detach().clone(), [x.grad.clone() for x in xd],
                      {n: p.grad.clone() for n, p in mod.named_parameters() if p.grad is not None})
    (z1, gx1, gp1), (z0, gx0, gp0) = res[True], res[False]
    assert torch.equal(z1, z0)
    for a, b in zip(gx1, gx0):
        assert torch.equal(a, b)
    for n in gp0:
        if n.startswith("conv."):
            assert rel_err(gp1[n], gp0[n]) < 1e-5, n
        else:
            assert torch.equal(gp1[n], gp0[n]), n


@pytest.mark.parametrize("B", [1, 7, 300])
def test_attn_conv_abi_matches_separate_kernels(B):
    """The fused C-ABI entries against the separate ones on the same device inputs: P, the
    Conv2d output, g_pv, g_k and max |g_pv| bit-identical; the Conv2d weight / bias gradients
    within 1e-5 (another column-sum order)."""
    import math
    from mvml_gat._lib import call, lib, ptr, ws_ptr_size
    g = torch.Generator(device=DEV).manual_seed(B)
    H, D = 12, 384
    PV = torch.randn(3 * B, 2 * H * D, device=DEV, generator=g)
    Xn = torch.randn(3 * B, D, device=DEV, generator=g)
    w = torch.randn(12, 12, 3, 3, device=DEV, generator=g) * 0.1
    bias = torch.randn(12, device=DEV, generator=g) * 0.1
    gout = torch.randn(B, 12, D - 2, device=DEV, generator=g)
    sc = 1.0 / math.sqrt(D)
    st = torch.cuda.current_stream().cuda_stream
    L = lib()
    res = {}
    for fused in (True, False):
        P = torch.empty(B, H, 3, 3, device=DEV)
        out = torch.empty(B, 12, D - 2, device=DEV)
        gPV = torch.empty_like(PV)
        gk = torch.empty_like(Xn)
        gw, gb = torch.empty_like(w), torch.empty_like(bias)
        amx = torch.zeros(1, dtype=torch.int32, device=DEV)
        if fused:
            call("mvml_attn_conv_fwd", B, H, D, ptr(PV), 2 * H * D, ptr(Xn), D, sc, ptr(w), ptr(bias),
                 ptr(P), ptr(out), 0.0, 0, st)
            wp, wn = ws_ptr_size(L.mvml_attn_conv_bwd_workspace_size(B), DEV)
            rows = torch.zeros(3 * B, dtype=torch.int32, device=DEV)
            call("mvml_attn_conv_bwd", B, H, D, ptr(PV), 2 * H * D, ptr(Xn), D, sc, ptr(P), ptr(w),
                 ptr(out), ptr(gout), 1.0, ptr(gPV), 2 * H * D, ptr(gk), D, ptr(amx), ptr(rows), ptr(gw),
                 ptr(gb), wp, wn, st)
            # the folded per-row maxima equal a pass over the written rows
            torch.cuda.synchronize()
            assert torch.equal(rows.view(torch.float32), gPV.abs().amax(1))
        else:
            att = torch.empty(B, H, 3, D, device=DEV)
            call("mvml_token_attn_fold_fwd", B, H, D, ptr(PV), 2 * H * D, ptr(Xn), D, sc, ptr(att),
                 ptr(P), st)
            call("mvml_conv3_fwd", B, 12, 12, D, ptr(att), ptr(w), ptr(bias), ptr(out), st)
            gatt = torch.empty_like(att)
            wp, wn = ws_ptr_size(L.mvml_conv3_bwd_workspace_size(B), DEV)
            call("mvml_conv3_bwd", B, 12, 12, D, ptr(att), ptr(w), ptr(out), ptr(gout), ptr(gatt),
                 ptr(gw), ptr(gb), wp, wn, st)
            call("mvml_token_attn_fold_bwd", B, H, D, ptr(PV), 2 * H * D, ptr(Xn), D, sc, ptr(P),
                 ptr(gatt), ptr(gPV), 2 * H * D, ptr(gk), D, ptr(amx), st)
        torch.cuda.synchronize()
        res[fused] = dict(P=P, out=out, gPV=gPV, gk=gk, amx=amx, gw=gw, gb=gb)
    diff = {k: (res[True][k].double() - res[False][k].double()).abs().max().item()
            for k in ("P", "out", "gPV", "gk", "amx")}
    assert all(v == 0 for v in diff.values()), diff
    assert rel_err(res[True]["gw"], res[False]["gw"]) < 1e-5
    assert rel_err(res[True]["gb"], res[False]["gb"]) < 1e-5
