"""The small layout kernels that keep PyTorch's own kernels out of the training step
(norm.hip: mvml_copy_cols, mvml_fill_zero, mvml_lstm_pack_weights, mvml_transpose,
mvml_scale_by): each BITWISE equal to the torch expression it replaces (pure data movement, or
one fp32 multiply), on ragged shapes and on both the 16-B and the scalar paths."""
import pytest
import torch

from mvml_gat import functional as Fn
from mvml_gat._lib import call, ptr, stream_ptr

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("rows,cols,lds,ldd", [(1000, 8, 1600, 8), (777, 768, 1152, 768), (33, 13, 29, 17),
                                               (5, 4, 0, 4)])
def test_copy_cols(rows, cols, lds, ldd):
    src = torch.randn(max(rows * lds, cols) + 3, device=DEV)
    dst = torch.full((rows * ldd + 3,), -7.0, device=DEV)
    call("mvml_copy_cols", rows, cols, ptr(src), lds, ptr(dst), ldd, stream_ptr())
    s = src[:cols].expand(rows, cols) if lds == 0 else src[:rows * lds].view(rows, lds)[:, :cols]
    d = dst[:rows * ldd].view(rows, ldd)
    assert torch.equal(d[:, :cols], s)
    assert torch.all(d[:, cols:] == -7.0) and torch.all(dst[rows * ldd:] == -7.0)
    # misaligned pointers: the scalar path, same result
    dst2 = torch.zeros(rows * ldd + 1, device=DEV)
    call("mvml_copy_cols", rows, cols, ptr(src), lds, ptr(dst2[1:]), ldd, stream_ptr())
    assert torch.equal(dst2[1:].view(rows, ldd)[:, :cols], s)


def test_copy2d_helper_views():
    a = torch.randn(64, 3, 384, device=DEV)
    out = Fn.copy2d(torch.empty(64, 384, device=DEV), a[:, 1])
    assert torch.equal(out, a[:, 1])
    b = torch.randn(5, device=DEV)
    rep = torch.empty(4, 5, device=DEV)
    Fn.copy2d(rep, b.view(1, 5).expand(4, 5))
    assert torch.equal(rep, b.expand(4, 5))


def test_fill_zero_contiguous_and_pitched():
    t = torch.randn(7, 11, 5, device=DEV)
    Fn.zero_(t)
    assert torch.count_nonzero(t) == 0
    big = torch.randn(50, 96, device=DEV)
    ref = big.clone()
    ref[:, 32:] = 0
    Fn.zero_(big[:, 32:])
    assert torch.equal(big, ref)
    # the vector-store kernel (aligned pitched slices, Set2Set's recurrent-state columns at the
    # bench's size: more rows than one grid sweep) and the runtime's 2-D memset (unaligned start)
    for rows, cols, c0 in ((65536, 1152, 384), (50, 96, 33), (9, 8, 4)):
        big = torch.randn(rows, cols, device=DEV)
        ref = big.clone()
        ref[:, c0:] = 0
        Fn.zero_(big[:, c0:])
        assert torch.equal(big, ref), (rows, cols, c0)
    z = Fn.zeros((3, 1000), dtype=torch.int32, device=DEV)
    assert z.dtype == torch.int32 and torch.count_nonzero(z) == 0


@pytest.mark.parametrize("D,kin", [(384, 768), (384, 384), (8, 3)])
def test_lstm_pack_weights(D, kin):
    w_ih = torch.randn(4 * D, kin, device=DEV)
    w_hh = torch.randn(4 * D, D, device=DEV)
    wcat = torch.empty(4 * D, kin + D, device=DEV)
    wperm = torch.empty_like(wcat)
    call("mvml_lstm_pack_weights", D, kin, ptr(w_ih), ptr(w_hh), ptr(wcat), ptr(wperm), stream_ptr())
    ref = torch.cat([w_ih, w_hh], dim=1)
    assert torch.equal(wcat, ref)
    assert torch.equal(wperm, ref.view(4, D, kin + D).transpose(0, 1).reshape(4 * D, kin + D))


@pytest.mark.parametrize("rows,cols", [(4608, 384), (37, 70), (1, 33)])
def test_transpose(rows, cols):
    src = torch.randn(rows, cols, device=DEV)
    dst = torch.full((cols, rows + 5), 3.0, device=DEV)
    call("mvml_transpose", rows, cols, ptr(src), cols, ptr(dst), rows + 5, stream_ptr())
    assert torch.equal(dst[:, :rows], src.t())
    assert torch.all(dst[:, rows:] == 3.0)


def test_scale_by():
    x = torch.randn(100003, device=DEV)
    s = torch.tensor(0.37, device=DEV)
    y = torch.empty_like(x)
    call("mvml_scale_by", x.numel(), ptr(x), ptr(s), ptr(y), stream_ptr())
    assert torch.equal(y, x * s)


def test_bce_mean_and_backward_match_torch():
    from mvml_gat import bce_with_logits
    z = (torch.randn(4096, 11, device=DEV) * 3).requires_grad_()
    y = (torch.rand(4096, 11, device=DEV) > 0.7).float()
    loss = bce_with_logits(z, y)
    loss.backward(torch.tensor(2.0, device=DEV))
    zr = z.detach().double().requires_grad_()
    ref = torch.nn.functional.binary_cross_entropy_with_logits(zr, y.double())
    (2 * ref).backward()
    assert loss.shape == () and abs(loss.item() - ref.item()) <= 1e-6 * abs(ref.item())
    assert (z.grad.double() - zr.grad).abs().max().item() <= 1e-6 * zr.grad.abs().max().item()
