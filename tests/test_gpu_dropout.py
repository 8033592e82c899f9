"""nn.Dropout on the HIP path (mvml_dropout_fwd; model.py:87 GNNModule.fc, model.py:36 / 46 the
fusion head's conv and MLP): training-mode Dropout follows a ReLU in every use, so it runs in
place on the ReLU output and the backward reads the dropped output instead of a mask
(mvml_relu_bwd / mvml_attn_conv_bwd with the 1 / (1 - p) scale).

The draws cannot equal torch's (another generator), so the tests pin what Dropout IS:
  * kept elements are exactly x * (1 / (1 - p)) (torch's fused_dropout arithmetic), dropped
    ones 0, the kept fraction within 6 sigma of 1 - p, the mask a function of (seed, index)
    only (same seed: same mask, vector and scalar paths agree; another seed: another mask);
  * Linear + ReLU + Dropout (training) equals torch autograd of relu(x W^T + b) * M / (1 - p)
    with M the mask the forward drew — output and every gradient;
  * the fused attention + conv + ReLU + Dropout: the kernel's in-store Dropout draws exactly
    mvml_dropout_fwd's mask for the same seed, and its gradients with p equal (bitwise) those
    of the p = 0 kernel fed g_out * M / (1 - p);
  * eval mode and p = 0 launch nothing and change nothing."""
import pytest
import torch

from mvml_gat import functional as Fn
from mvml_gat._lib import call, ptr, stream_ptr

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _drop(x, p, seed, out=None):
    y = torch.empty_like(x) if out is None else out
    call("mvml_dropout_fwd", x.numel(), ptr(x), ptr(y), float(p), int(seed), stream_ptr())
    return y


@pytest.mark.parametrize("p", [0.2, 0.5])
def test_dropout_kernel_semantics(p):
    n = 1_000_003  # ragged: the scalar tail runs
    x = torch.randn(n, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1)) + 10.0  # no zeros
    y = _drop(x, p, seed=12345)
    torch.cuda.synchronize()
    kept = y != 0
    s = torch.tensor(1.0 / (1.0 - p), dtype=torch.float32, device=DEV)
    assert torch.equal(y[kept], x[kept] * s)
    frac = kept.double().mean().item()
    sigma = (p * (1 - p) / n) ** 0.5
    assert abs(frac - (1 - p)) < 6 * sigma, (frac, 1 - p)
    # deterministic in (seed, index); in place == out of place
    assert torch.equal(_drop(x, p, seed=12345), y)
    z = x.clone()
    _drop(z, p, seed=12345, out=z)
    assert torch.equal(z, y)
    # another seed: another mask (of ~n p (1 - p) x 2 differing positions, essentially all)
    k2 = _drop(x, p, seed=12346) != 0
    assert (k2 != kept).double().mean().item() > p * (1 - p)
    # misaligned pointers take the scalar path: the same mask for the same element index
    xs = x[1:]
    assert torch.equal(_drop(xs, p, 99), _drop(xs.clone(), p, 99))
    # consecutive elements are not correlated (adjacent keep decisions independent)
    a, b = kept[:-1].double(), kept[1:].double()
    both = (a * b).mean().item()
    assert abs(both - (1 - p) ** 2) < 8 * ((1 - p) ** 2 * (1 - (1 - p) ** 2) / n) ** 0.5


def test_dropout_p0_is_identity():
    x = torch.randn(4099, device=DEV)
    assert torch.equal(_drop(x, 0.0, 5), x)
    y = x.clone()
    assert Fn.relu_dropout_(y, 0.0) == 1.0 and torch.equal(y, x)


@pytest.mark.parametrize("p", [0.2, 0.5])
def test_linear_relu_dropout_matches_torch_autograd(p):
    torch.manual_seed(3)
    M, K, Nout = 2000, 384, 1024
    x = torch.randn(M, K, device=DEV, requires_grad=True)
    w = (torch.randn(Nout, K, device=DEV) * 0.05).requires_grad_()
    b = (torch.randn(Nout, device=DEV) * 0.1).requires_grad_()
    cap = {}
    Fn.DEBUG_CAPTURE = cap
    try:
        y = Fn.LinearReLUFunction.apply(x, w, b, p)
    finally:
        Fn.DEBUG_CAPTURE = None
    gy = torch.randn(M, Nout, device=DEV)
    y.backward(gy)
    # reference in float64 with the forward's own mask, on the product's own side of every
    # ReLU (a pre-activation within fp32 rounding of 0 may take the other side in float64)
    side = (cap["relu_out"][0] > 0).double()
    xd, wd, bd = (t.detach().double().requires_grad_() for t in (x, w, b))
    z = (xd @ wd.t() + bd) * side
    m = (y.detach() != 0).double()
    # a kept element with ReLU output 0 reads 0 too: "dropped" for this mask, but its value and
    # gradient are 0 either way
    yr = z * m / (1 - p)
    yr.backward(gy.double())
    tol = 1e-5
    assert (y.double() - yr).norm() / yr.norm() < tol
    for mine, ref in ((x.grad, xd.grad), (w.grad, wd.grad), (b.grad, bd.grad)):
        assert (mine.double() - ref).norm() / ref.norm() < tol
    pos = side > 0
    frac = (m.bool() & pos).sum().item() / pos.sum().item()
    assert abs(frac - (1 - p)) < 0.01, frac


def test_attn_conv_dropout_gradient_is_masked_scaled():
    from mvml_gat import MVFusion
    from mvml_gat.fusion import FusionAttnConvFunction
    torch.manual_seed(0)
    B, D = 512, 384
    mod = MVFusion(D, 12, 11, dropout=0.3).to(DEV)
    ln = mod.norm_layer_module
    xs = [torch.randn(B, D, device=DEV) for _ in range(3)]
    args = (ln.weight, ln.bias, mod.linear_q.weight, mod.linear_k.weight, mod.linear_v.weight,
            mod.conv[0].weight, mod.conv[0].bias, ln.eps)

    def run(p, g):
        for t in mod.parameters():
            t.grad = None
        out = FusionAttnConvFunction.apply(*xs, *args, p)
        out.backward(g)
        return out.detach(), {n: t.grad.clone() for n, t in mod.named_parameters() if t.grad is not None}

    g = torch.randn(B, 12 * (D - 2), device=DEV)
    out_p, grads_p = run(0.3, g)
    out_0, _ = run(0.0, g)
    s = torch.tensor(1.0 / (1.0 - 0.3), dtype=torch.float32, device=DEV)
    kept = out_p != 0
    assert torch.equal(out_p[kept], out_0[kept] * s)
    assert torch.all(out_0[~kept] >= 0)
    _, grads_ref = run(0.0, g * kept.float() * s)
    assert grads_p.keys() == grads_ref.keys() and grads_p
    for n in grads_p:
        assert torch.equal(grads_p[n], grads_ref[n]), n


def test_eval_mode_draws_nothing():
    from mvml_gat import MVFusion
    mod = MVFusion(384, 12, 11, dropout=0.5).to(DEV).eval()
    xs = [torch.randn(64, 384, device=DEV) for _ in range(3)]
    with torch.no_grad():
        a = mod(*xs)
        b = mod(*xs)
    assert torch.equal(a, b)
    assert Fn.dropout_p(mod.conv[2]) == 0.0 and Fn.dropout_p(mod.mlp[2]) == 0.0


def test_attn_conv_store_dropout_is_the_standalone_mask():
    """mvml_attn_conv_fwd with drop_p: bitwise mvml_dropout_fwd (same seed) of its p = 0 output."""
    from mvml_gat._lib import lib
    torch.manual_seed(5)
    B, H, D = 300, 12, 384
    PV = torch.randn(3 * B, 2 * H * D, device=DEV) * 0.05
    Xn = torch.randn(3 * B, D, device=DEV)
    w = torch.randn(H, H, 3, 3, device=DEV) * 0.1
    bias = torch.randn(H, device=DEV) * 0.1
    P = torch.empty(B, H, 3, 3, device=DEV)
    outs = []
    for p, seed in ((0.0, 0), (0.35, 424242)):
        out = torch.empty(B, H, D - 2, device=DEV)
        rc = lib().mvml_attn_conv_fwd(B, H, D, ptr(PV), 2 * H * D, ptr(Xn), D, 1.0 / D ** 0.5, ptr(w), ptr(bias),
                                      ptr(P), ptr(out), p, seed, stream_ptr())
        assert rc == 0
        outs.append(out)
    ref = _drop(outs[0], 0.35, 424242)
    torch.cuda.synchronize()
    assert torch.equal(outs[1], ref)
    assert 0.5 < (outs[1] != 0).double().mean().item() / max((outs[0] != 0).double().mean().item(), 1e-9) < 0.8
