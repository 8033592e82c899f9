"""bf16 projection on MFMA (BASELINE.json config 4; north_star accuracy bar 2e-2 for bf16).

* mvml_gemm_bf16 against fp64 products of the bf16-ROUNDED operands: bf16 x bf16 products are
  exact in fp32, so the only error left is fp32 accumulation (bar 1e-5, TOL_EXACT) — this
  pins the kernel's operand rounding (round-to-nearest-even) and layouts exactly;
* the same products against fp64 of the unrounded operands within 2e-2 (TOL_BF16);
* GNNModule(proj_dtype=torch.bfloat16) output within 2e-2 of the float64 oracle (the fp32
  reference semantics); gradients by norm-wise error (GRAD_FRO) and cosine (GRAD_COS)."""
import pytest
import torch

from _util import batch_of_sizes, graph_dict, model_pair
from conftest import rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL_EXACT = 1e-5
TOL_BF16 = 2e-2
GRAD_FRO = 0.15    # norm-wise relative error of every parameter gradient (worst measured: 0.13, L2 attn_r)
GRAD_COS = 0.99    # cosine similarity with the fp64 gradient (worst measured: 0.9917, L2 attn_r)
# The attention vectors' gradients sum d el / d er over atoms, and d er is the edge softmax
# backward a (g_a - sum a g_a): a difference of near-equal dots of bf16-rounded Z rows, so the
# bf16 representation error comes back amplified by that cancellation.  Measured on the MVP step
# with the restated fingerprints' upstream gradient: L2 attn_r 0.206 / 0.9885 (attn_l 0.079).
GRAD_FRO_ATTN, GRAD_COS_ATTN = 0.3, 0.98


def grad_ok(name, fro, cos):
    if name.endswith(("attn_l", "attn_r")):
        return fro < GRAD_FRO_ATTN and cos > GRAD_COS_ATTN
    return fro < GRAD_FRO and cos > GRAD_COS


def _bf(x):
    return x.float().bfloat16().double()


@pytest.mark.parametrize("ak,bk", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (130, 70, 74), (257, 300, 768), (1000, 1928, 768),
                                   (512, 384, 65536 + 17)])
def test_gemm_bf16_layouts(ak, bk, M, N, K):
    from mvml_gat.functional import gemm
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    B = torch.randn(K, N, generator=g, dtype=torch.float64)
    bias = torch.randn(N, generator=g, dtype=torch.float64)
    C0 = torch.randn(M, N, generator=g, dtype=torch.float64)
    Ad = (A.t() if ak else A).contiguous().float().to(DEV)
    Bd = (B if bk else B.t()).contiguous().float().to(DEV)
    C = C0.float().to(DEV)
    gemm(Ad, Bd, M, N, K, ak, bk, M if ak else K, N if bk else K, C, N,
         bias=bias.float().to(DEV), beta=0.5, act=1, algo="bf16")
    exact = torch.relu(_bf(A) @ _bf(B) + bias.float().double() + 0.5 * C0.float().double())
    assert rel_err(C, exact) < TOL_EXACT
    assert rel_err(C, torch.relu(A @ B + bias + 0.5 * C0)) < TOL_BF16


def test_gnn_module_bf16_projection():
    sb = batch_of_sizes([25, 11, 40, 23, 17, 3, 1, 60, 33], seed=11)
    prod, ref = model_pair(seed=3)
    prod.set_projection_dtype(torch.bfloat16)
    prod.eval()
    ref64 = ref.double().eval()
    out_r = ref64(graph_dict(sb), torch.as_tensor(sb.feats, dtype=torch.float64))
    gout = torch.randn_like(out_r)
    out_r.backward(gout)
    prod = prod.to(DEV)
    g = sb.to_graph().to(DEV)
    out_p = prod(g, g.ndata["h"])
    out_p.backward(gout.float().to(DEV))
    err_out = rel_err(out_p, out_r)
    print(f"bf16 projection: output rel err {err_out:.1e}")
    assert 1e-6 < err_out < TOL_BF16           # the bf16 path really ran, within the bar
    # Gradients: the 2e-2 bar is on outputs (north_star).  A bf16-perturbed pre-activation that
    # crosses a ReLU / leaky-ReLU kink flips single gradient entries by O(1), so gradients are
    # held to a norm-wise (Frobenius) relative error and direction (cosine) instead.
    pr = dict(ref64.named_parameters())
    worst = {}
    for n, p in prod.named_parameters():
        a, b = p.grad.double().cpu().flatten(), pr[n].grad.flatten()
        fro = ((a - b).norm() / b.norm()).item()
        cos = (a @ b / (a.norm() * b.norm())).item()
        worst[n] = (round(fro, 4), round(cos, 5))
    print("bf16 projection grads (frobenius rel err, cosine):", worst)
    bad = {n: v for n, v in worst.items() if not grad_ok(n, *v)}
    assert not bad, bad
