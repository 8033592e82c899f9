"""Diagnostics for the config-3 (GraphNorm groups of 64) parity failure: per-parameter errors of
the whole module, then each GAT layer alone on the same graph."""
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
sb = synth.config3(int(sys.argv[1]) if len(sys.argv) > 1 else 192, seed=11)
gs = int(sys.argv[2]) if len(sys.argv) > 2 else 64
prod, ref = model_pair(seed=7)
prod.eval(); ref.eval()
ref64 = ref.double()
gd = graph_dict(sb, group_size=gs)
X = torch.as_tensor(sb.feats, dtype=torch.float64)
out_r = ref64(gd, X)
gout = torch.randn(out_r.shape, generator=torch.Generator().manual_seed(7), dtype=torch.float64)
out_r.backward(gout)
prod = prod.to(DEV)
g = sb.to_graph(group_size=gs).to(DEV)
plan = g.node_groups.cpu().numpy()
G = g.num_node_groups
print("groups", G, "kinds", {int(k): int((plan[G + 1:2 * G + 1] == k).sum()) for k in set(plan[G + 1:2 * G + 1].tolist())},
      "fallback fwd/bwd", plan[2 * G + 1], plan[2 * G + 2])
out_p = prod(g, g.ndata["h"])
out_p.backward(gout.float().to(DEV))
print("module out", rel_err(out_p, out_r))
p64 = dict(ref64.named_parameters())
for n, p in prod.named_parameters():
    print(f"  {n:45s} {rel_err(p.grad, p64[n].grad):.2e}")

for layer in (0, 1):
    prod, ref = model_pair(seed=layer)
    conv_p = prod.conv.gnn_layers[layer].to(DEV)
    conv_r = ref.conv.gnn_layers[layer].gat_conv
    n = int(sb.num_nodes.sum())
    gen = torch.Generator().manual_seed(layer)
    Xl = torch.as_tensor(sb.feats, dtype=torch.float64) if layer == 0 else torch.randn(n, 768, generator=gen, dtype=torch.float64)
    params = {"fc.weight": conv_r.fc.weight, "res_fc.weight": conv_r.res_fc.weight,
              "attn_l": conv_r.attn_l, "attn_r": conv_r.attn_r, "bias": conv_r.bias}
    pp = {k: v.detach().double().requires_grad_() for k, v in params.items()}
    Xr = Xl.clone().requires_grad_()
    o_r = gnn_ref.gat_layer_ref(gd["src"], gd["dst"], Xr, pp, 4, 192 if layer == 0 else 384,
                                "flatten" if layer == 0 else "mean",
                                torch.nn.functional.elu if layer == 0 else None)
    go = torch.randn(o_r.shape, generator=gen, dtype=torch.float64)
    o_r.backward(go)
    Xp = Xl.float().to(DEV).requires_grad_()
    o_p = conv_p(g, Xp)
    o_p.backward(go.float().to(DEV))
    c = conv_p.gat_conv
    print(f"layer {layer}: out {rel_err(o_p, o_r):.2e} dX {rel_err(Xp.grad, Xr.grad):.2e} " +
          " ".join(f"{k} {rel_err(getattr(c, k.split('.')[0]).weight.grad if '.' in k else getattr(c, k).grad, pp[k].grad):.2e}"
                   for k in pp))
