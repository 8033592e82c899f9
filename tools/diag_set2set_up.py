"""Diagnostics: Set2Set backward with the module's real upstream gradient (GraphNorm -> fc),
GEMM algorithm from MVML_GEMM_ALGO (x3 / f32)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mvml-mpi_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from _util import graph_dict, model_pair  # noqa: E402
from conftest import rel_err  # noqa: E402
from mvml_gat import synth  # noqa: E402
from mvml_gat.nn import Set2Set  # noqa: E402
from oracle import gnn_ref  # noqa: E402

DEV = "cuda:0"
sb = synth.config3(192, seed=11)
gd = graph_dict(sb, group_size=64)
prod, ref = model_pair(seed=7)
ref64 = ref.double().eval()
X = torch.as_tensor(sb.feats, dtype=torch.float64)
with torch.no_grad():
    node_x = gnn_ref.gat_ref(gd["src"], gd["dst"], X, ref64.layer_params(), ref64.hidden_feats)
s_in = node_x.clone().requires_grad_()
s = gnn_ref.set2set_ref(gd["node_offsets"], s_in, ref64.readout.lstm, 6)
sd = s.detach().requires_grad_()
y = gnn_ref.graphnorm_ref(sd, ref64.norm.weight, ref64.norm.bias, ref64.norm.mean_scale, 1e-5, gd["group_offsets"])
o = ref64.fc(y)
gout = torch.randn(o.shape, generator=torch.Generator().manual_seed(7), dtype=torch.float64)
o.backward(gout)
g_s = sd.grad.clone()
print("upstream g_s: absmax", g_s.abs().max().item(), "column-sum / column-abs-sum (median)",
      (g_s.sum(0).abs() / g_s.abs().sum(0)).median().item())
g = sb.to_graph(group_size=64).to(DEV)
s2s = prod.readout
lstm64 = ref64.readout.lstm
lstm32 = torch.nn.LSTM(768, 384, 3)
lstm32.load_state_dict({k: v.float() for k, v in lstm64.state_dict().items()})
Xr = node_x.clone().requires_grad_()
out_r = gnn_ref.set2set_ref(gd["node_offsets"], Xr, lstm64, 6)
out_r.backward(g_s)
X32 = node_x.float().clone().requires_grad_()
gnn_ref.set2set_ref(gd["node_offsets"], X32, lstm32, 6).backward(g_s.float())
s2s = s2s.to(DEV)
Xp = node_x.float().to(DEV).requires_grad_()
s2s(g, Xp).backward(g_s.float().to(DEV))
print(f"gX {rel_err(Xp.grad, Xr.grad):.2e} (fp32 oracle {rel_err(X32.grad, Xr.grad):.2e})")
for (n, p), (n2, p2), (n3, p3) in zip(s2s.lstm.named_parameters(), lstm64.named_parameters(), lstm32.named_parameters()):
    print(f"   {n:16s} {rel_err(p.grad, p2.grad):.2e} (fp32 oracle {rel_err(p3.grad, p2.grad):.2e})")
