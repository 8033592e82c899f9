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


@pytest.mark.parametrize("fold", [True, False])
@pytest.mark.parametrize("B", [1, 5, 64, 300, 2048])
def test_fusion_forward_backward_parity(B, fold, monkeypatch):
    """fold: the Q.K re-associated path (mvml_token_attn_fold_*, the default); False: the
    literal Q / K / V GEMM + mvml_token_attn_*.  Natural biases: both ReLUs see both branches
    (the zeroed one drives conv3_bwd's and relu_bwd's masking), the oracle follows the
    product's side at each kink."""
    import mvml_gat.fusion as fu
    monkeypatch.setattr(fu, "FOLD_QK", fold)
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
    for name, p in mod.named_parameters():
        if name.startswith("norm_layer."):
            assert p.grad is None  # constructed but unused, as in the reference
            continue
        assert rel_err(p.grad, pr[name].grad) < TOL, name


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
