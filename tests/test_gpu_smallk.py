"""Small-K split-fp16 products (gemm_smallk_kernel behind mvml_gemm_f16x2_rows):
layer 1's projection X [N_atoms, 76] x Wcat [1544, 76]^T as a wave-per-64-columns memory kernel.

Checks, on ragged shapes (M, N not multiples of the 16-row block / 64-column slab; K = 4 .. 96,
every k-step count 1 .. 6 incl. the 16-deep tail) with rows spread over 2^-28 .. 2^12:
  * every row within 1e-5 of the float64 product relative to its own max (the tiles' bar);
  * the 256x256 tile path (option smallk = 0) agrees to fp32-GEMM accuracy (not bitwise: the
    MFMA shape changes the summation order);
  * B as its interleaved split image (il4) and as fp32 split in the kernel: bitwise equal;
  * non-temporal and plain stores: bitwise equal;
  * a row's result does not depend on the other rows of the launch (bitwise);
  * the pitch padding of C (ldc > N) is left untouched; bias + ReLU epilogue.
"""
import pytest
import torch

from mvml_gat._lib import call, lib, option, ptr, stream_ptr, ws_ptr_size
from mvml_gat.functional import absmax, absmax_rows, slot

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 1e-5
SHAPES = [(1, 4, 4), (17, 8, 12), (1000, 68, 76), (4099, 1544, 76), (300, 60, 80), (2000, 200, 16),
          (513, 64, 32), (77, 100, 44), (130, 1548, 64), (40, 12, 48),
          # K 84 .. 96: the KS16 = 6 plan (three 16x16x32 steps, no 16-deep tail)
          (1000, 200, 84), (333, 1544, 92), (2048, 64, 96)]


def _inputs(M, N, K, seed):
    g = torch.Generator().manual_seed(seed)
    exps = torch.tensor([-12, 0, 8, 12, 16, 20, 24, 28], dtype=torch.float64)
    A = (torch.randn(M, K, generator=g, dtype=torch.float64) *
         torch.pow(2.0, -exps[torch.arange(M) % len(exps)]).unsqueeze(1)).float()
    if M > 7:
        A[7] = 0.0
    B = torch.randn(N, K, generator=g).float()
    return A, B


def _run(A, B, M, N, K, il4=True, bias=None, act=0, ldc=None, smallk=1):
    st = stream_ptr()
    Ad, Bd = A.to(DEV), B.to(DEV)
    bmx = torch.zeros(1, dtype=torch.int32, device=DEV)
    absmax(Bd, N, K, K, bmx, 0)
    rows = absmax_rows(Ad, M, K, K)
    img = None
    if il4:
        img = torch.empty_like(Bd)
        call("mvml_split_f16x2_il4", N, K, ptr(Bd), K, slot(bmx, 0), ptr(img), st)
    ldc = ldc or N
    C = torch.full((M, ldc), float("nan"), device=DEV)
    wp, wn = ws_ptr_size(lib().mvml_gemm_workspace_size(M, N, K), DEV)
    bd = None if bias is None else bias.to(DEV)
    with option("smallk", smallk):
        call("mvml_gemm_f16x2_rows", M, N, K, ptr(Ad), K, ptr(Bd), K, 0, ptr(img), ptr(rows), slot(bmx, 0),
             ptr(bd), 0.0, act, ptr(C), ldc, wp, wn, st)
    torch.cuda.synchronize()
    return C


@pytest.mark.parametrize("shape", SHAPES)
def test_smallk_rows_accuracy(shape):
    M, N, K = shape
    A, B = _inputs(M, N, K, 3 + K)
    ref = A.double() @ B.double().t()
    C = _run(A, B, M, N, K).double().cpu()
    den = ref.abs().max(1).values.clamp_min(1e-300)
    d = (C - ref).abs().max(1).values / den
    if M > 7:
        assert float(C[7].abs().max()) == 0.0
        d[7] = 0.0
    assert float(d.max()) < TOL, (shape, float(d.max()))


@pytest.mark.parametrize("shape", [(4099, 1544, 76), (1000, 68, 76), (300, 60, 80), (77, 100, 44)])
def test_smallk_matches_tile_path(shape):
    M, N, K = shape
    A, B = _inputs(M, N, K, 11)
    c1 = _run(A, B, M, N, K, smallk=1).double()
    c0 = _run(A, B, M, N, K, smallk=0).double()
    den = c0.abs().amax(1).clamp_min(1e-30)
    assert float(((c1 - c0).abs().amax(1) / den).max()) < 2e-6


@pytest.mark.parametrize("shape", [(4099, 1544, 76), (17, 8, 12), (300, 60, 80)])
def test_smallk_il4_and_store_kinds_bitwise(shape):
    M, N, K = shape
    A, B = _inputs(M, N, K, 5)
    base = _run(A, B, M, N, K, il4=True, smallk=1)
    assert torch.equal(base, _run(A, B, M, N, K, il4=False, smallk=1))
    assert torch.equal(base, _run(A, B, M, N, K, il4=True, smallk=2))


def test_smallk_batch_invariant():
    M, N, K = 3001, 1544, 76
    A, B = _inputs(M, N, K, 9)
    A[:50] *= 1e4
    full = _run(A, B, M, N, K)
    for lo, hi in ((0, 300), (300, 3001), (777, 1001), (3000, 3001)):
        part = _run(A[lo:hi].contiguous(), B, hi - lo, N, K)
        assert torch.equal(part, full[lo:hi]), (lo, hi)


def test_smallk_pitch_bias_relu():
    M, N, K = 1111, 1544, 76
    A, B = _inputs(M, N, K, 13)
    bias = torch.randn(N)
    ldc = 1552
    C = _run(A, B, M, N, K, bias=bias, act=1, ldc=ldc).cpu()
    assert torch.isnan(C[:, N:]).all()  # the pitch padding is not written
    ref = torch.relu(A.double() @ B.double().t() + bias.double())
    den = (A.double() @ B.double().t()).abs().max(1).values.clamp_min(1e-30) + bias.double().abs().max()
    d = (C[:, :N].double() - ref).abs().max(1).values / den
    assert float(d.max()) < TOL
    C0 = _run(A, B, M, N, K, bias=bias, act=1, ldc=ldc, smallk=0).cpu()
    assert float(((C[:, :N] - C0[:, :N]).abs().max(1).values.double() / den).max()) < 2e-6


@pytest.mark.parametrize("shape", [(4099, 1544, 76), (1000, 68, 76), (77, 100, 44), (300, 60, 80), (40, 12, 16)])
def test_smallk_zero_low_plane(shape):
    """0 / 1 rows (layer 1's atom features: fp16-exact, so the low plane is zero and the kernel
    skips the h_b l_a products for the block) mixed with random rows in some 16-row blocks:
    every row within 1e-5 of float64 and agreeing with the tile path."""
    M, N, K = shape
    g = torch.Generator().manual_seed(21 + K)
    A = (torch.rand(M, K, generator=g) < 0.15).float()
    mixed = torch.arange(M) % 97 == 5  # a few random rows: their blocks take the full product
    A[mixed] = torch.randn(int(mixed.sum()), K, generator=g)
    B = torch.randn(N, K, generator=g).float()
    ref = A.double() @ B.double().t()
    C = _run(A, B, M, N, K).double().cpu()
    den = ref.abs().max(1).values.clamp_min(1e-30)
    assert float(((C - ref).abs().max(1).values / den).max()) < TOL
    C0 = _run(A, B, M, N, K, smallk=0).double().cpu()
    assert float(((C - C0).abs().max(1).values / den).max()) < 2e-6


@pytest.mark.parametrize("shape", [(4099, 1544, 76), (1000, 68, 76), (40, 12, 76)])
def test_smallk_b_in_lds_bitwise(shape):
    """The default kernel (B planes in LDS, a workgroup per slab) against the register-B build
    (option smallk 10): the same fragments and products, so bitwise equal outputs."""
    M, N, K = shape
    A, B = _inputs(M, N, K, 17)
    assert torch.equal(_run(A, B, M, N, K, smallk=1), _run(A, B, M, N, K, smallk=10))
