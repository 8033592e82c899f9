"""Per-layer error budget on the golden fixture: for each GAT layer, feed the float64 oracle's
layer input and upstream gradient to (a) the HIP GATLayerFunction (fp32) and (b) the fp32 CPU
oracle, and report relative errors of outputs, el/er, attention, d el/d er and parameter
gradients against the float64 oracle.  Diagnostic only (imports the oracle as the checker)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mvml-mpi_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle.gnn_ref import edge_softmax_ref  # noqa: E402


def rel(a, b):
    a = np.asarray(torch.as_tensor(a).detach().cpu().double())
    b = np.asarray(torch.as_tensor(b).detach().cpu().double())
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def layer_ref(src, dst, X, p, H, Fo, mean, dtype):
    """gatconv_ref + GATLayer agg with el/er/a retained for inspection."""
    src = torch.as_tensor(src, dtype=torch.long)
    dst = torch.as_tensor(dst, dtype=torch.long)
    X = X.to(dtype).detach().requires_grad_()
    q = {k: v.to(dtype).detach().requires_grad_() for k, v in p.items()}
    n = X.shape[0]
    Z = (X @ q["fc.weight"].t()).view(n, H, Fo)
    el = (Z * q["attn_l"]).sum(-1)
    er = (Z * q["attn_r"]).sum(-1)
    el.retain_grad()
    er.retain_grad()
    e = F.leaky_relu(el[src] + er[dst], 0.2)
    a = edge_softmax_ref(e, dst, n)
    rst = torch.zeros((n, H, Fo), dtype=dtype).index_add(0, dst, a.unsqueeze(-1) * Z[src])
    rst = rst + (X @ q["res_fc.weight"].t()).view(n, H, Fo) + q["bias"].view(1, H, Fo)
    out = rst.mean(1) if mean else F.elu(rst.flatten(1))
    return X, q, el, er, a, out


def main():
    from mvml_gat import from_arrays
    from mvml_gat import functional as Fn
    gold = dict(np.load(os.path.join(ROOT, "tests", "golden", "gnn_small.npz")))
    bg = from_arrays(gold["num_nodes"], gold["num_edges"], gold["src_local"], gold["dst_local"],
                     group_size=int(gold["group_size"])).to("cuda")
    src, dst = gold["batch_src"], gold["batch_dst"]
    H = 4
    feats = [16, 24]
    h = torch.as_tensor(gold["X"])
    torch.manual_seed(0)
    for li, Fo in enumerate(feats):
        mean = li == len(feats) - 1
        pre = f"param:conv.gnn_layers.{li}.gat_conv."
        p = {k: torch.as_tensor(gold[pre + k]) for k in ("fc.weight", "res_fc.weight", "attn_l", "attn_r", "bias")}
        X64, q64, el64, er64, a64, out64 = layer_ref(src, dst, h, p, H, Fo, mean, torch.float64)
        g = torch.randn(out64.shape, dtype=torch.float64)
        out64.backward(g)
        X32, q32, el32, er32, a32, out32 = layer_ref(src, dst, h, p, H, Fo, mean, torch.float32)
        out32.backward(g.float())
        # HIP
        Xc = h.float().cuda().requires_grad_()
        pc = {k: v.float().cuda().requires_grad_() for k, v in p.items()}
        mode = Fn.MODE_MEAN if mean else Fn.MODE_FLATTEN_ELU
        outc = Fn.GATLayerFunction.apply(Xc, pc["fc.weight"], pc["res_fc.weight"], pc["attn_l"],
                                         pc["attn_r"], pc["bias"], bg, H, Fo, 0.2, mode)
        Fn.DEBUG_CAPTURE = {}
        outc.backward(g.float().cuda())
        cap, Fn.DEBUG_CAPTURE = Fn.DEBUG_CAPTURE, None
        eid = bg.in_eid.long().cpu()
        print(f"layer {li} ({'mean' if mean else 'flatten+elu'}, F={Fo})   hip     fp32-cpu")
        print(f"  out        {rel(outc, out64):.2e}  {rel(out32, out64):.2e}")
        print(f"  gX         {rel(Xc.grad, X64.grad):.2e}  {rel(X32.grad, X64.grad):.2e}")
        for k in p:
            print(f"  g {k:14s}{rel(pc[k].grad, q64[k].grad):.2e}  {rel(q32[k].grad, q64[k].grad):.2e}")
        print(f"  el         {rel(cap['elr'][:, :H], el64):.2e}  {rel(el32, el64):.2e}")
        print(f"  er         {rel(cap['elr'][:, H:], er64):.2e}  {rel(er32, er64):.2e}")
        print(f"  attention  {rel(cap['attn'].cpu(), a64[eid]):.2e}  {rel(a32, a64):.2e}")
        print(f"  d el       {rel(cap['gelr'][:, :H], el64.grad):.2e}  {rel(el32.grad, el64.grad):.2e}")
        print(f"  d er       {rel(cap['gelr'][:, H:], er64.grad):.2e}  {rel(er32.grad, er64.grad):.2e}")
        print(f"  d el (cpu32) {rel(el32.grad, el64.grad):.2e}   d er (cpu32) {rel(er32.grad, er64.grad):.2e}")
        h = out64.detach()


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def model_stages():
    """Whole-model stage-by-stage error budget on the golden fixture (HIP vs fp32-CPU)."""
    from mvml_gat import GNNModule, from_arrays
    from oracle.gnn_ref import GNNModuleRef, gat_ref, graphnorm_ref, set2set_ref
    gold = dict(np.load(os.path.join(ROOT, "tests", "golden", "gnn_small.npz")))
    bg = from_arrays(gold["num_nodes"], gold["num_edges"], gold["src_local"], gold["dst_local"],
                     group_size=int(gold["group_size"])).to("cuda")
    sd = {k[6:]: torch.as_tensor(v) for k, v in gold.items() if k.startswith("param:")}
    offs = np.concatenate([[0], np.cumsum(gold["num_nodes"])])
    B = len(gold["num_nodes"])
    gs = int(gold["group_size"])
    groups = list(range(0, B, gs)) + [B]

    def run_ref(dtype):
        m = GNNModuleRef(74, [16, 24], 0.5, 3, 2).to(dtype).eval()
        m.load_state_dict({k: v.to(dtype) for k, v in sd.items()})
        X = torch.as_tensor(gold["X"]).to(dtype).requires_grad_()
        nx = gat_ref(gold["batch_src"], gold["batch_dst"], X, m.layer_params(), m.hidden_feats)
        gx = set2set_ref(offs, nx, m.readout.lstm, m.readout.n_iters)
        no = graphnorm_ref(gx, m.norm.weight, m.norm.bias, m.norm.mean_scale, m.norm.eps, groups)
        out = m.fc(no)
        for t in (nx, gx, no):
            t.retain_grad()
        out.backward(torch.as_tensor(gold["g_out"]).to(dtype))
        return m, X, nx, gx, no, out

    def run_hip():
        m = GNNModule(74, [16, 24], 0.5, 3, 2)
        m.load_state_dict({k: v.float() for k, v in sd.items()})
        m = m.cuda().eval()
        X = torch.as_tensor(gold["X"]).float().cuda().requires_grad_()
        nx = m.conv(bg, X)
        gx = m.readout(bg, nx)
        no = m.norm(gx, group_offsets=bg.group_offsets_rows())
        from mvml_gat import functional as Fn
        out = Fn.LinearReLUFunction.apply(no, m.fc[0].weight, m.fc[0].bias)
        for t in (nx, gx, no):
            t.retain_grad()
        out.backward(torch.as_tensor(gold["g_out"]).float().cuda())
        return m, X, nx, gx, no, out

    r64, r32, hp = run_ref(torch.float64), run_ref(torch.float32), run_hip()
    names = ["X", "node_x", "graph_x", "norm_out", "out"]
    print("stage          fwd hip  fwd cpu32  grad hip  grad cpu32")
    for i, n in enumerate(names):
        a64, a32, ah = r64[i + 1], r32[i + 1], hp[i + 1]
        gf = lambda t: t.grad if t.grad is not None else torch.zeros(1)
        print(f"  {n:12s} {rel(ah, a64):.2e}  {rel(a32, a64):.2e}  "
              f"{rel(gf(ah), gf(a64)) if i < 4 else 0:.2e}  {rel(gf(a32), gf(a64)) if i < 4 else 0:.2e}")
    p64 = dict(r64[0].named_parameters())
    p32 = dict(r32[0].named_parameters())
    for k, p in hp[0].named_parameters():
        print(f"  g {k:45s} {rel(p.grad, p64[k].grad):.2e}  {rel(p32[k].grad, p64[k].grad):.2e}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "model":
    model_stages()
