"""Debug: per-stage comparison of the fusion backward against float64 torch."""
import sys, os, math
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "mvml-mpi_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch
from conftest import rel_err
from oracle.fusion_ref import MVFusionRef
from mvml_gat import MVFusion
from mvml_gat import fusion as FU
DEV = "cuda"
for B in (5, 64, 65, 130):
    torch.manual_seed(B)
    ref = MVFusionRef().double().eval()
    mod = MVFusion().to(DEV).eval()
    mod.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    g = torch.Generator().manual_seed(B + 1)
    xs = [torch.randn(B, 384, generator=g, dtype=torch.float64) for _ in range(3)]
    # reference intermediates
    ln = ref.norm_layer_module
    X = torch.stack(xs, 1).reshape(3 * B, 384).requires_grad_(True)
    Xn = ln(X)
    Xn.retain_grad()
    W = torch.cat([ref.linear_q.weight, ref.linear_k.weight, ref.linear_v.weight])
    QKV = Xn @ W.t()
    QKV.retain_grad()
    q, k, v = QKV.view(B, 3, 3, 12, 384).unbind(2)
    q, k, v = (t.transpose(1, 2) for t in (q, k, v))
    att = torch.softmax(q @ k.transpose(2, 3) / math.sqrt(384), -1) @ v
    att.retain_grad()
    out = torch.relu(torch.nn.functional.conv2d(att, ref.conv[0].weight, ref.conv[0].bias)).view(B, -1)
    gup = torch.randn(out.shape, generator=g, dtype=torch.float64)
    (out * gup).sum().backward()
    # device path
    xd = [x.float().to(DEV).requires_grad_(True) for x in xs]
    o = FU.FusionAttnConvFunction.apply(*xd, mod.norm_layer_module.weight, mod.norm_layer_module.bias,
                                        mod.linear_q.weight, mod.linear_k.weight, mod.linear_v.weight,
                                        mod.conv[0].weight, mod.conv[0].bias, 1e-5)
    print(B, "out", rel_err(o, out))
    saved = {}
    orig = FU.gemm
    def spy(A, Bm, M, N, K, *a, **kw):
        orig(A, Bm, M, N, K, *a, **kw)
        saved.setdefault("calls", []).append((M, N, K))
    FU.gemm = spy
    (o * gup.float().to(DEV)).sum().backward()
    FU.gemm = orig
    gX = torch.stack([x.grad for x in xd], 1).reshape(3 * B, 384)
    print(B, "gX", rel_err(gX, X.grad), "calls", saved.get("calls"))
    d = (gX.double().cpu() - X.grad).abs()
    idx = d.argmax()
    print("   worst row", int(idx // 384), "col", int(idx % 384), float(d.max()), float(X.grad.abs().max()))
    print("   per-row max err (first 8 bad rows):", [(int(r), float(d[r].max())) for r in torch.nonzero(d.max(1).values > 1e-6 * float(X.grad.abs().max())).flatten()[:8]])
