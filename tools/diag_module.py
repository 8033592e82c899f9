"""Diagnostics: gradient error at every stage boundary of GNNModule on config-3 molecules."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mvml-mpi_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from _util import graph_dict, model_pair  # noqa: E402
from conftest import rel_err  # noqa: E402
from mvml_gat import functional as Fn, synth  # noqa: E402
from oracle import gnn_ref  # noqa: E402

DEV = "cuda:0"
n = int(sys.argv[1]) if len(sys.argv) > 1 else 192
sb = synth.config3(n, seed=11)
gd = graph_dict(sb, group_size=64)
prod, ref = model_pair(seed=7)
prod.eval(); ref.eval()


def run_ref(m, X):
    t = {}
    lp = m.layer_params()
    h1 = gnn_ref.gat_layer_ref(gd["src"], gd["dst"], X, lp[0], 4, 192, "flatten", torch.nn.functional.elu)
    h2 = gnn_ref.gat_layer_ref(gd["src"], gd["dst"], h1, lp[1], 4, 384, "mean", None)
    s = gnn_ref.set2set_ref(gd["node_offsets"], h2, m.readout.lstm, 6)
    y = gnn_ref.graphnorm_ref(s, m.norm.weight, m.norm.bias, m.norm.mean_scale, 1e-5, gd["group_offsets"])
    o = m.fc(y)
    for k, v in (("h1", h1), ("h2", h2), ("s2s", s), ("gn", y)):
        v.retain_grad(); t[k] = v
    return o, t


ref32 = type(ref)(74, [192, 384], 0.5, 6, 3).eval()
ref32.load_state_dict(ref.state_dict())
ref64 = ref.double()
X = torch.as_tensor(sb.feats, dtype=torch.float64)
o64, t64 = run_ref(ref64, X)
gout = torch.randn(o64.shape, generator=torch.Generator().manual_seed(7), dtype=torch.float64)
o64.backward(gout)
o32, t32 = run_ref(ref32, X.float())
o32.backward(gout.float())

prod = prod.to(DEV)
g = sb.to_graph(group_size=64).to(DEV)
h1 = prod.conv.gnn_layers[0](g, g.ndata["h"]); h1.retain_grad()
h2 = prod.conv.gnn_layers[1](g, h1); h2.retain_grad()
s = prod.readout(g, h2); s.retain_grad()
y = prod.norm(s, group_offsets=g.group_offsets_rows()); y.retain_grad()
o = Fn.LinearReLUFunction.apply(y, prod.fc[0].weight, prod.fc[0].bias)
o.backward(gout.float().to(DEV))
tp = {"h1": h1, "h2": h2, "s2s": s, "gn": y}
for k in ("gn", "s2s", "h2", "h1"):
    print(f"{k:4s} value {rel_err(tp[k], t64[k]):.2e} (fp32 {rel_err(t32[k].detach(), t64[k].detach()):.2e})  "
          f"grad {rel_err(tp[k].grad, t64[k].grad):.2e} (fp32 {rel_err(t32[k].grad, t64[k].grad):.2e})")
p64 = dict(ref64.named_parameters()); p32 = dict(ref32.named_parameters())
for nme, p in prod.named_parameters():
    if "gnn_layers" in nme:
        print(f"  {nme:45s} {rel_err(p.grad, p64[nme].grad):.2e} (fp32 {rel_err(p32[nme].grad, p64[nme].grad):.2e})")
# layer-1 alone with the module's own upstream gradient (oracle g of h2) and inputs (oracle h1)
c = prod.conv.gnn_layers[1].to(DEV)
c.zero_grad()
h1r = t64["h1"].detach().float().to(DEV).requires_grad_()
h2p = c(g, h1r)
h2p.backward(t64["h2"].grad.float().to(DEV))
print("layer1 with exact inputs: out", f"{rel_err(h2p, t64['h2']):.2e}", "dX", f"{rel_err(h1r.grad, t64['h1'].grad):.2e}")
for nme, p in c.named_parameters():
    print(f"  {nme:30s} {rel_err(p.grad, p64['conv.gnn_layers.1.' + nme].grad):.2e}")
