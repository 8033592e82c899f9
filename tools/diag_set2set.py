"""Diagnostics: Set2Set backward on config-3 molecules, with random and with real GAT node
features, against the float64 / float32 oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mvml-mpi_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from _util import graph_dict, model_pair  # noqa: E402
from conftest import rel_err  # noqa: E402
from mvml_gat import synth  # noqa: E402
from oracle import gnn_ref  # noqa: E402

DEV = "cuda:0"
sb = synth.config3(192, seed=11)
gd = graph_dict(sb, group_size=64)
prod, ref = model_pair(seed=7)
ref64 = ref.double().eval()
X = torch.as_tensor(sb.feats, dtype=torch.float64)
with torch.no_grad():
    node_x = gnn_ref.gat_ref(gd["src"], gd["dst"], X, ref64.layer_params(), ref64.hidden_feats)
print("node_x absmax", node_x.abs().max().item(), "rms", node_x.pow(2).mean().sqrt().item())
g = sb.to_graph(group_size=64).to(DEV)
from mvml_gat.nn import Set2Set  # noqa: E402
for name, Xn in (("random", torch.randn_like(node_x)), ("gat", node_x)):
    torch.manual_seed(0)
    s2s = Set2Set(384, 6, 3)
    lstm64 = torch.nn.LSTM(768, 384, 3).double()
    lstm64.load_state_dict({k: v.double() for k, v in s2s.lstm.state_dict().items()})
    lstm32 = torch.nn.LSTM(768, 384, 3)
    lstm32.load_state_dict(s2s.lstm.state_dict())
    Xr = Xn.clone().requires_grad_()
    out_r = gnn_ref.set2set_ref(gd["node_offsets"], Xr, lstm64, 6)
    gout = torch.randn(out_r.shape, generator=torch.Generator().manual_seed(1), dtype=torch.float64)
    out_r.backward(gout)
    X32 = Xn.float().clone().requires_grad_()
    o32 = gnn_ref.set2set_ref(gd["node_offsets"], X32, lstm32, 6)
    o32.backward(gout.float())
    s2s = s2s.to(DEV)
    Xp = Xn.float().to(DEV).requires_grad_()
    out_p = s2s(g, Xp)
    out_p.backward(gout.float().to(DEV))
    print(f"{name}: out {rel_err(out_p, out_r):.2e} (fp32 oracle {rel_err(o32, out_r):.2e}) "
          f"gX {rel_err(Xp.grad, Xr.grad):.2e} (fp32 oracle {rel_err(X32.grad, Xr.grad):.2e})")
    for (n, p), (n2, p2), (n3, p3) in zip(s2s.lstm.named_parameters(), lstm64.named_parameters(), lstm32.named_parameters()):
        print(f"   {n:16s} {rel_err(p.grad, p2.grad):.2e} (fp32 oracle {rel_err(p3.grad, p2.grad):.2e})")
