"""mvml_gemm_f16x2_amax_colsum: a GAT layer's weight gradient gY^T X and its bias gradient (column
sums of gY's residual columns) from one call.  On the skinny 128x128 split-fp16 plan (layer 1,
N = 76) the column sums come out of the product's own fragment reads (gemm_f32_kernel RS); the
product itself must stay BITWISE the plain mvml_gemm_f16x2_amax, and the sums within fp32
rounding of float64.  On other plans the entry is the product then mvml_colsum_f32: bitwise both.
Shapes: split-K and not, M and K off the tile sizes, a row pitch past M, sum ranges inside M."""
import pytest
import torch

from mvml_gat import _lib
from mvml_gat import functional as Fn
from mvml_gat._lib import call, ptr, stream_ptr

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _case(M, N, K, lda, sum_off, sum_n, alpha, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    A = torch.randn((K, lda), device=DEV, generator=g) * 0.3  # gY: K atoms x M gradient columns
    A[:, :M] += torch.randn((1, M), device=DEV, generator=g)  # column means that do not cancel
    B = torch.randn((K, N), device=DEV, generator=g)          # X: K atoms x N features
    amx = torch.zeros(2, dtype=torch.int32, device=DEV)
    Fn.absmax(A, K, M, lda, amx, 0)
    Fn.absmax(B, K, N, N, amx, 1)
    return A, B, amx


@pytest.mark.parametrize("M,N,K,lda,sum_off,sum_n,alpha", [
    (1552, 76, 60000, 1600, 768, 768, 1.0),   # layer 1 shape at a split-K size
    (777, 20, 4133, 800, 100, 333, 0.25),     # ragged M and K, a sum range inside M
    (300, 76, 1000, 320, 0, 300, 1.0),        # K < 2048: no split-K
    (1928, 768, 20000, 1984, 1536, 384, 0.25),  # the wide plan (layer 2): product + column sums
])
def test_dw_colsum_matches_separate_calls(M, N, K, lda, sum_off, sum_n, alpha):
    A, B, amx = _case(M, N, K, lda, sum_off, sum_n, alpha, seed=M + N + K)
    L = _lib.lib()
    fused = bool(L.mvml_gemm_colsum_fused(M, N, K))
    assert fused == (N <= 96)
    st = stream_ptr()
    C1 = torch.full((M, N), float("nan"), device=DEV)
    s1 = torch.full((sum_n,), float("nan"), device=DEV)
    wp, wn = _lib.ws_ptr_size(L.mvml_gemm_colsum_workspace_size(M, N, K, sum_n), DEV)
    call("mvml_gemm_f16x2_amax_colsum", M, N, K, ptr(A), lda, ptr(B), N, Fn.slot(amx, 0), Fn.slot(amx, 1),
         ptr(C1), N, sum_off, sum_n, alpha, ptr(s1), wp, wn, st)
    # the two calls it replaces
    C0 = torch.empty((M, N), device=DEV)
    wp, wn = _lib.ws_ptr_size(L.mvml_gemm_workspace_size(M, N, K), DEV)
    call("mvml_gemm_f16x2_amax", 1, 1, M, N, K, ptr(A), lda, ptr(B), N, Fn.slot(amx, 0), Fn.slot(amx, 1),
         None, 0.0, 0, ptr(C0), N, wp, wn, st)
    s0 = torch.empty(sum_n, device=DEV)
    Fn.colsum(A, K, sum_n, lda, s0, offset=sum_off, alpha=alpha)
    assert torch.equal(C1, C0)
    if not fused:
        assert torch.equal(s1, s0)
    ref = alpha * A[:, sum_off:sum_off + sum_n].double().sum(0)
    err = ((s1.double() - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-6, err
    # deterministic: a second call gives the same bits
    s2 = torch.empty_like(s1)
    wp, wn = _lib.ws_ptr_size(L.mvml_gemm_colsum_workspace_size(M, N, K, sum_n), DEV)
    call("mvml_gemm_f16x2_amax_colsum", M, N, K, ptr(A), lda, ptr(B), N, Fn.slot(amx, 0), Fn.slot(amx, 1),
         ptr(C1), N, sum_off, sum_n, alpha, ptr(s2), wp, wn, st)
    assert torch.equal(s1, s2)
