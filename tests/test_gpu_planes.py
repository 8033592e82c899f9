"""The LDS-DMA split-fp16 tile (csrc/gemm_planes.hip, mvml_gemm_f16x2_planes; a measured
experiment, not in the training step: DESIGN.md "Round 6") is BITWISE the register-staged tile
(mvml_gemm_f16x2_rows) on the same operands — fp32 A split in the loop or A as its il8 image,
per-row or operand-wide A scales, 16- and 32-deep stages and the ping-pong wave groups — and
the A-image form equals the fp32-A form (K <= 96 products run the small-K kernel behind
mvml_gemm_f16x2_rows: there only the float64 bar)."""
import pytest
import torch

from mvml_gat.functional import absmax, absmax_rows, gemm, gemm_planes, slot, split_il4, split_il8

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("M,N,K", [(1000, 300, 200), (2600, 520, 768), (777, 1544, 76)])
@pytest.mark.parametrize("variant", [dict(BK="32", PP="0"), dict(BK="16", PP="0"), dict(BK="16", PP="1")])
def test_planes_bitwise_rows_tile(M, N, K, variant, monkeypatch):
    for k, v in variant.items():
        monkeypatch.setenv(f"MVML_PLANES_{k}", v)
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    A = torch.randn((M, K), device=DEV, generator=g) * torch.exp2(
        torch.randint(-8, 9, (M, 1), device=DEV, generator=g).float())
    Bm = torch.randn((N, K), device=DEV, generator=g)
    mx = torch.zeros(2, dtype=torch.int32, device=DEV)
    absmax(Bm, N, K, K, mx, 1)
    rows = absmax_rows(A, M, K, K)
    il4 = split_il4(Bm, N, K, K, slot(mx, 1))
    il8 = split_il8(Bm, N, K, K, amax_ptr=slot(mx, 1))
    kp = il8.shape[1]
    assert kp % 32 == 0 and kp >= K
    ref = torch.empty((M, N), device=DEV)
    gemm(A, Bm, M, N, K, 0, 0, K, K, ref, N, amax=(None, slot(mx, 1)), arows=rows, bil4=il4)
    out = torch.empty((M, N), device=DEV)
    gemm_planes(A, M, N, K, K, il8, kp, out, N, slot(mx, 1), arows=rows)
    torch.cuda.synchronize()
    if K > 96:  # (K <= 96: mvml_gemm_f16x2_rows runs the small-K memory kernel, not the tile)
        assert torch.equal(out, ref)
    aimg = split_il8(A, M, K, K, rows_max=rows)
    out2 = torch.empty((M, N), device=DEV)
    gemm_planes(aimg, M, N, K, kp, il8, kp, out2, N, slot(mx, 1), arows=rows, a_image=True)
    torch.cuda.synchronize()
    assert torch.equal(out2, out)
    # against float64: each row within 1e-5 of its own max
    r64 = A.double() @ Bm.double().T
    err = ((out.double() - r64).abs().amax(dim=1) / r64.abs().amax(dim=1).clamp_min(1e-300)).max().item()
    assert err < 1e-5, err
