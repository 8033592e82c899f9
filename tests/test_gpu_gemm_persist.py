"""The persistent tile loop of the 256x256 split-fp16 GEMMs (option gemm_persist, default 256:
one workgroup per CU walking its XCD's tile range) against one workgroup per tile
(gemm_persist = 0): BITWISE equal outputs, row maxima and output maxima.

Each case has more than 256 tiles and a tile count that is not a multiple of 8, ragged M and N
(partial edge tiles), so a workgroup walks several tiles — re-initialising the per-tile row
shifts / row maxima in LDS — and the XCD partition has uneven ranges.  A cap below 8 is rounded
up to 8 by the host (every XCD gets a workgroup), which the last case checks too.
"""
import pytest
import torch

from mvml_gat._lib import call, lib, option, ptr, stream_ptr, ws_ptr_size
from mvml_gat.functional import absmax, absmax_rows, slot

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
M, N, K = 256 * 37 + 45, 256 * 9 + 72, 384  # 38 x 10 = 380 tiles (not a multiple of 8)


def _inputs(seed, m=M, n=N, k=K, batch=1):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(batch, m, k, generator=g)
    A *= torch.pow(2.0, -torch.randint(0, 20, (batch, m, 1), generator=g).float())  # row dynamic range
    B = torch.randn(batch, n, k, generator=g)
    return A.to(DEV), B.to(DEV)


def _run(fn, caps=(0, 256, 5)):
    outs = []
    for cap in caps:
        with option("gemm_persist", cap):
            outs.append([t.clone() for t in fn()])
    torch.cuda.synchronize()
    for cap, o in zip(caps[1:], outs[1:]):
        for i, (a, b) in enumerate(zip(outs[0], o)):
            assert torch.equal(a, b), (cap, i, (a.double() - b.double()).abs().max().item())


@pytest.mark.parametrize("il4", [0, 1])
def test_persist_rows(il4):
    """mvml_gemm_f16x2_rows: per-row A scales (rsh re-initialised per tile), B as fp32 or as its
    interleaved-by-4 image, bias + ReLU epilogue."""
    A, B = _inputs(1)
    A, B = A[0], B[0]
    st = stream_ptr()
    bmx = torch.zeros(1, dtype=torch.int32, device=DEV)
    absmax(B, N, K, K, bmx, 0)
    rows = absmax_rows(A, M, K, K)
    img = None
    if il4:
        img = torch.empty_like(B)
        call("mvml_split_f16x2_il4", N, K, ptr(B), K, slot(bmx, 0), ptr(img), st)
    bias = torch.randn(N, device=DEV)
    wp, wn = ws_ptr_size(lib().mvml_gemm_workspace_size(M, N, K), DEV)

    def fn():
        C = torch.full((M, N), float("nan"), device=DEV)
        call("mvml_gemm_f16x2_rows", M, N, K, ptr(A), K, ptr(B), K, 0, ptr(img), ptr(rows), slot(bmx, 0),
             ptr(bias), 0.0, 1, ptr(C), N, wp, wn, st)
        return [C]
    _run(fn)


def test_persist_amax_and_bsplit():
    """mvml_gemm_f16x2_amax (operand-wide scales) and mvml_gemm_f16x2_bsplit (B from its
    interleaved split image)."""
    A, B = _inputs(2)
    A, B = A[0], B[0]
    st = stream_ptr()
    mx = torch.zeros(2, dtype=torch.int32, device=DEV)
    absmax(A, M, K, K, mx, 0)
    absmax(B, N, K, K, mx, 1)
    img = torch.empty_like(B)
    call("mvml_split_f16x2_il4", N, K, ptr(B), K, slot(mx, 1), ptr(img), st)
    wp, wn = ws_ptr_size(lib().mvml_gemm_workspace_size(M, N, K), DEV)

    def fn():
        C1 = torch.full((M, N), float("nan"), device=DEV)
        C2 = torch.full((M, N), float("nan"), device=DEV)
        call("mvml_gemm_f16x2_amax", 0, 0, M, N, K, ptr(A), K, ptr(B), K, slot(mx, 0), slot(mx, 1), None,
             0.0, 0, ptr(C1), N, wp, wn, st)
        call("mvml_gemm_f16x2_bsplit", 0, 0, M, N, K, ptr(A), K, ptr(B), K, ptr(img), 0,
             slot(mx, 0), slot(mx, 1), None, 0.0, 0, ptr(C2), N, wp, wn, st)
        return [C1, C2]
    _run(fn)


def test_persist_batched():
    """mvml_gemm_f16x2_batched: grid z = product, the tile loop per product."""
    Ab, Bb = _inputs(3, m=256 * 17 + 9, n=256 * 5 + 40, batch=3)
    m, n = Ab.shape[1], Bb.shape[1]
    st = stream_ptr()
    mx = torch.zeros(2, dtype=torch.int32, device=DEV)
    absmax(Ab.view(-1, K), 3 * m, K, K, mx, 0)
    absmax(Bb.view(-1, K), 3 * n, K, K, mx, 1)

    def fn():
        C = torch.full((3, m, n), float("nan"), device=DEV)
        call("mvml_gemm_f16x2_batched", 0, 0, m, n, K, 3, ptr(Ab), K, m * K, ptr(Bb), K, n * K,
             slot(mx, 0), slot(mx, 1), ptr(C), n, m * n, st)
        return [C]
    _run(fn)


@pytest.mark.parametrize("act", [2, 3])
def test_persist_ex_epilogues(act):
    """mvml_gemm_f16x2_ex with the output's maxima: act 2 (bias + ELU) with per-row output
    maxima c_rows and the output max c_amax (s_rmax re-initialised per tile; the EX row-max
    atomics), act 3 (x ELU'(aux))."""
    if not hasattr(lib(), "mvml_gemm_f16x2_ex"):
        pytest.skip("mvml_gemm_f16x2_ex not exported")
    A, B = _inputs(4)
    A, B = A[0], B[0]
    st = stream_ptr()
    bmx = torch.zeros(1, dtype=torch.int32, device=DEV)
    absmax(B, N, K, K, bmx, 0)
    rows = absmax_rows(A, M, K, K)
    bias = torch.randn(N, device=DEV)
    aux = torch.randn(M, N, device=DEV)

    def fn():
        C = torch.full((M, N), float("nan"), device=DEV)
        camax = torch.zeros(1, dtype=torch.int32, device=DEV)
        crows = torch.zeros(M, dtype=torch.int32, device=DEV)
        if act == 2:
            call("mvml_gemm_f16x2_ex", M, N, K, 1, ptr(A), K, 0, ptr(B), K, 0, None, 0, ptr(rows), 0,
                 slot(bmx, 0), ptr(bias), 0, 2, ptr(C), N, 0, None, 0, ptr(camax), ptr(crows), 0, 0, 0, st)
        else:
            call("mvml_gemm_f16x2_ex", M, N, K, 1, ptr(A), K, 0, ptr(B), K, 0, None, 0, ptr(rows), 0,
                 slot(bmx, 0), None, 0, 3, ptr(C), N, 0, ptr(aux), N, ptr(camax), None, 0, 0, 0, st)
        return [C, camax, crows]
    _run(fn)
