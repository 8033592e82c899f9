import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "mvml-mpi_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch
from conftest import rel_err
from mvml_gat.fusion import LinearFunction
from mvml_gat.functional import LinearReLUFunction
DEV = "cuda"
for B in (5, 64, 65):
    g = torch.Generator().manual_seed(B)
    x = torch.randn(B, 4584, generator=g, dtype=torch.float64)
    w1 = torch.randn(1024, 4584, generator=g, dtype=torch.float64) * 0.01
    b1 = torch.randn(1024, generator=g, dtype=torch.float64) * 0.1
    w2 = torch.randn(11, 1024, generator=g, dtype=torch.float64) * 0.03
    b2 = torch.randn(11, generator=g, dtype=torch.float64) * 0.1
    up = torch.randn(B, 11, generator=g, dtype=torch.float64)
    R = [t.clone().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    h = torch.relu(R[0] @ R[1].t() + R[2])
    z = h @ R[3].t() + R[4]
    (z * up).sum().backward()
    D = [t.float().to(DEV).requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    hd = LinearReLUFunction.apply(D[0], D[1], D[2])
    zd = LinearFunction.apply(hd, D[3], D[4])
    (zd * up.float().to(DEV)).sum().backward()
    print(B, "h", rel_err(hd, h), "z", rel_err(zd, z), "grads", [f"{rel_err(a.grad, b.grad):.2e}" for a, b in zip(D, R)])
