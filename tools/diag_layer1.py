"""Diagnostics: layer-1 (mean) backward intermediates (d el, d er) on config-3 molecules with
the module's real upstream gradient, per node group."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mvml-mpi_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from _util import graph_dict, model_pair  # noqa: E402
from mvml_gat import functional as Fn, synth  # noqa: E402
from oracle import gnn_ref  # noqa: E402

DEV = "cuda:0"
sb = synth.config3(192, seed=11)
gd = graph_dict(sb, group_size=64)
prod, ref = model_pair(seed=7)
ref64 = ref.double().eval()
X = torch.as_tensor(sb.feats, dtype=torch.float64)
lp = ref64.layer_params()
h1 = gnn_ref.gat_layer_ref(gd["src"], gd["dst"], X, lp[0], 4, 192, "flatten", F.elu).detach()
h1.requires_grad_()
# oracle layer 1 with explicit el / er
p = {k: v.detach().clone().requires_grad_() for k, v in lp[1].items()}
src = torch.as_tensor(np.asarray(gd["src"]), dtype=torch.long)
dst = torch.as_tensor(np.asarray(gd["dst"]), dtype=torch.long)
N = h1.shape[0]
H, Fo = 4, 384
Z = (h1 @ p["fc.weight"].t()).view(N, H, Fo); Z.retain_grad()
el = (Z * p["attn_l"]).sum(-1); el.retain_grad()
er = (Z * p["attn_r"]).sum(-1); er.retain_grad()
e = F.leaky_relu(el[src] + er[dst], 0.2)
a = gnn_ref.edge_softmax_ref(e, dst, N)
rst = torch.zeros((N, H, Fo), dtype=torch.float64).index_add(0, dst, a.unsqueeze(-1) * Z[src])
rst = rst + (h1 @ p["res_fc.weight"].t()).view(N, H, Fo) + p["bias"].view(1, H, Fo)
h2 = rst.mean(1)
# the module's upstream gradient at h2 (Set2Set -> GraphNorm -> fc)
h2d = h2.detach().requires_grad_()
s = gnn_ref.set2set_ref(gd["node_offsets"], h2d, ref64.readout.lstm, 6)
y = gnn_ref.graphnorm_ref(s, ref64.norm.weight, ref64.norm.bias, ref64.norm.mean_scale, 1e-5, gd["group_offsets"])
o = ref64.fc(y)
gout = torch.randn(o.shape, generator=torch.Generator().manual_seed(7), dtype=torch.float64)
o.backward(gout)
g_h2 = h2d.grad.clone()
h2.backward(g_h2)
print("g_h2 per-molecule structure: rms", g_h2.pow(2).mean().sqrt().item())
print("d el absmax", el.grad.abs().max().item(), "d er absmax", er.grad.abs().max().item(),
      "dZ absmax", Z.grad.abs().max().item())

c = prod.conv.gnn_layers[1].to(DEV)
g = sb.to_graph(group_size=64).to(DEV)
cap = {}
Fn.DEBUG_CAPTURE = cap
h1p = h1.detach().float().to(DEV).requires_grad_()
out = c(g, h1p)
out.backward(g_h2.float().to(DEV))
gelr = cap["gelr"].double().cpu()
d_el, d_er = gelr[:, :H], gelr[:, H:2 * H]
attn = cap["attn"].double().cpu()
print("attn (in-CSR order) vs oracle: first check skipped")
err_l = (d_el - el.grad).abs()
err_r = (d_er - er.grad).abs()
print("d el err max", err_l.max().item(), "rel", err_l.max().item() / el.grad.abs().max().item())
print("d er err max", err_r.max().item(), "rel", err_r.max().item() / er.grad.abs().max().item())
G = g.num_node_groups
plan = g.node_groups.cpu().numpy()
starts = plan[:G + 1]
worst = []
for gi in range(G):
    a0, a1 = starts[gi], starts[gi + 1]
    if a1 > a0:
        worst.append((err_r[a0:a1].max().item(), gi, a1 - a0))
worst.sort(reverse=True)
print("worst groups (err, group, atoms):", worst[:8])
print("best groups:", worst[-4:])
v = int(err_r.max(1).values.argmax())
print("worst atom", v, "ours", d_er[v].tolist(), "oracle", er.grad[v].tolist())
