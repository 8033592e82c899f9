"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on identical inputs.

Bars (BASELINE.json north_star): bit-exact for batching/CSR indices; fp32 outputs and
gradients within 1e-5 norm-wise relative error of the float64 oracle.
"""
import numpy as np
import pytest
import torch

from _util import batch_of_sizes, graph_dict, model_pair
from conftest import rel_err
from oracle import gnn_ref, graph_ref

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 1e-5


def _to_dev(sb, group_size=None):
    return sb.to_graph(group_size=group_size).to(DEV)


# ------------------------------------------------------------------ batching / CSR (bit-exact)
@pytest.mark.parametrize("sizes,hubs", [
    ([25] * 37, False),
    ([11, 23, 80, 5, 1, 40, 23], False),
    ([150, 300, 220], True),
    ([1] * 5, False),
    # one wave per molecule up to 256 atoms / 1024 edges, a workgroup for the rest, in one batch
    ([25, 300, 255, 257, 1, 64, 90, 256], True),
    ([256, 255, 257, 2, 3], False),
])
def test_build_csr_bit_exact(sizes, hubs):
    sb = batch_of_sizes(sizes, seed=3, hubs=hubs)
    g = _to_dev(sb)
    ref = graph_ref.batch_ref(sb.num_nodes, sb.src_local, sb.dst_local, sb.num_edges)
    csr = graph_ref.csr_ref(ref["src"], ref["dst"], ref["node_offsets"][-1])
    for k in ("node_offsets", "edge_offsets", "src", "dst", "node_graph"):
        np.testing.assert_array_equal(getattr(g, k).cpu().numpy(), ref[k], err_msg=k)
    for k in ("in_rowptr", "in_src", "in_eid", "out_rowptr", "out_dst", "out_inslot"):
        np.testing.assert_array_equal(getattr(g, k).cpu().numpy(), csr[k], err_msg=k)
    assert g.has_zero_in_degree is False


@pytest.mark.parametrize("sizes,hubs", [
    ([25] * 37, False),
    ([11, 23, 80, 5, 1, 40, 23, 130, 64, 64, 2], False),
    ([150, 300, 220, 7, 9], True),
    ([1] * 5, False),
    ([200, 30, 1, 90] * 300, False),  # > 1024 groups: several chunks of the list scan
])
def test_node_group_plan_bit_exact(sizes, hubs):
    sb = batch_of_sizes(sizes, seed=5, hubs=hubs)
    g = _to_dev(sb)
    G = g.num_node_groups
    plan = g.node_groups.cpu().numpy()
    starts, kinds, fwd, bwd = graph_ref.node_group_plan_ref(g.node_offsets.cpu().numpy(),
                                                            g.in_rowptr.cpu().numpy())
    assert G == len(kinds) and plan.size == 4 * G + 3
    np.testing.assert_array_equal(plan[:G + 1], starts)
    np.testing.assert_array_equal(plan[G + 1:2 * G + 1], kinds)
    nf, nb = int(plan[2 * G + 1]), int(plan[2 * G + 2])
    # the fallback lists come in group order (XCD-contiguous walks, gat_agg.hip list_block)
    assert plan[2 * G + 3:2 * G + 3 + nf].tolist() == sorted(fwd)
    assert plan[3 * G + 3:3 * G + 3 + nb].tolist() == sorted(bwd)


def test_build_csr_edge_cases():
    from mvml_gat import batching as G
    graphs = [
        G.bigraph_from_bonds(3, [(0, 1), (1, 2)]),
        G.MolGraph(0, [], []),                                      # empty molecule
        G.graph(([0, 1, 2, 2], [1, 2, 0, 1]), num_nodes=4),         # node 3 has no in-edge
        G.bigraph_from_bonds(5000, [(i, i + 1) for i in range(4999)]),  # > LDS histogram path
    ]
    bg = G.batch(graphs).to(DEV)
    src, dst = bg.edges()
    ref = graph_ref.batch_ref(bg._bnn, bg.src_local, bg.dst_local, bg._bne)
    csr = graph_ref.csr_ref(ref["src"], ref["dst"], ref["node_offsets"][-1])
    np.testing.assert_array_equal(src.cpu().numpy(), ref["src"])
    for k in ("in_rowptr", "in_src", "in_eid", "out_rowptr", "out_dst", "out_inslot"):
        np.testing.assert_array_equal(getattr(bg, k).cpu().numpy(), csr[k], err_msg=k)
    assert bg.has_zero_in_degree is True and csr["zero_in_degree"] == 1


def test_recollate_reproduces_indices():
    """BatchedMolGraph.recollate() (bench.py's per-step device collation) rebuilds every index
    and the node-group plan into the same buffers, bitwise equal to the first build."""
    sb = batch_of_sizes([11, 23, 80, 5, 1, 40, 23, 130, 64, 300, 150], seed=6, hubs=True)
    g = _to_dev(sb)
    keys = ("node_offsets", "edge_offsets", "src", "dst", "node_graph", "in_rowptr", "in_src",
            "in_eid", "out_rowptr", "out_dst", "out_inslot", "node_groups")
    first = {k: getattr(g, k).clone() for k in keys}
    for k in keys:
        getattr(g, k).fill_(-7)
    g.recollate()
    torch.cuda.synchronize()
    for k in keys[:-1]:
        assert torch.equal(getattr(g, k), first[k]), k
    G = g.num_node_groups
    a, b = first["node_groups"].cpu().numpy(), g.node_groups.cpu().numpy()
    np.testing.assert_array_equal(a[:2 * G + 3], b[:2 * G + 3])  # starts, kinds, list counts
    nf, nb = int(a[2 * G + 1]), int(a[2 * G + 2])
    np.testing.assert_array_equal(a[2 * G + 3:2 * G + 3 + nf], b[2 * G + 3:2 * G + 3 + nf])
    np.testing.assert_array_equal(a[3 * G + 3:3 * G + 3 + nb], b[3 * G + 3:3 * G + 3 + nb])


def test_build_csr_rejects_bad_ids():
    from mvml_gat import batching as G
    bad = G.MolGraph(2, [0, 5], [1, 0])
    with pytest.raises(ValueError):
        G.batch([bad]).to(DEV)


# ------------------------------------------------------------------ GEMM
import contextlib  # noqa: E402
import os  # noqa: E402


@contextlib.contextmanager
def _x3_tile(algo):
    """'x3-128' / 'x3-256' / 'f16x2-256' force the tile size (option gemm_tile, C ABI)."""
    from mvml_gat._lib import option
    with option("gemm_tile", int(algo.split("-")[1]) if "-" in algo else 0):
        yield algo.split("-")[0]


@pytest.mark.parametrize("algo", ["f32", "x3", "x3-128", "x3-256", "f16x2", "f16x2-256"])
@pytest.mark.parametrize("ak,bk", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (130, 70, 74), (257, 300, 768), (96, 40, 20000),
                                   (256, 384, 1000), (640, 512, 4000), (1000, 1928, 768),
                                   (512, 384, 65536 + 17),
                                   (49152, 384, 100), (6144, 384, 20000)])  # N = 256 + 128 splits
def test_gemm_layouts(ak, bk, M, N, K, algo):
    from mvml_gat.functional import gemm
    if K > 50000 and algo in ("f32", "x3-128"):
        pytest.skip("long-K case targets the 256x256 split-K path")
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    B = torch.randn(K, N, generator=g, dtype=torch.float64)
    bias = torch.randn(N, generator=g, dtype=torch.float64)
    C0 = torch.randn(M, N, generator=g, dtype=torch.float64)
    Ad = (A.t() if ak else A).contiguous().float().to(DEV)
    Bd = (B if bk else B.t()).contiguous().float().to(DEV)
    C = C0.float().to(DEV)
    with _x3_tile(algo) as a:
        gemm(Ad, Bd, M, N, K, ak, bk, M if ak else K, N if bk else K, C, N,
             bias=bias.float().to(DEV), beta=0.5, act=1, algo=a)
    ref = torch.relu(A @ B + bias + 0.5 * C0)
    assert rel_err(C, ref) < TOL


@pytest.mark.parametrize("K", [768, 20000])
def test_gemm_x3_error_matches_fp32(K):
    """The split-bf16 GEMM is as accurate as an fp32 GEMM: its error against fp64 stays within
    2x the error of the f32-input MFMA GEMM (and of torch's fp32 CPU matmul) on the same data,
    elementwise-max and RMS, including a wide dynamic range of magnitudes."""
    from mvml_gat.functional import gemm
    g = torch.Generator().manual_seed(K)
    M, N = 512, 384
    A = torch.randn(M, K, generator=g, dtype=torch.float64) * torch.exp(2 * torch.randn(M, 1, generator=g, dtype=torch.float64))
    B = torch.randn(K, N, generator=g, dtype=torch.float64)
    ref = A @ B
    errs = {}
    for algo in ("f32", "x3", "x3-256", "f16x2-256"):
        C = torch.zeros(M, N, device=DEV)
        with _x3_tile(algo) as a:
            gemm(A.float().to(DEV), B.t().contiguous().float().to(DEV), M, N, K, 0, 0, K, K, C, N, algo=a)
        d = (C.double().cpu() - ref)
        errs[algo] = (d.abs().max().item(), d.pow(2).mean().sqrt().item())
    cpu = (A.float() @ B.float()).double() - ref
    errs["cpu"] = (cpu.abs().max().item(), cpu.pow(2).mean().sqrt().item())
    base = max(errs["f32"][0], errs["cpu"][0]), max(errs["f32"][1], errs["cpu"][1])
    for algo in ("x3", "x3-256", "f16x2-256"):
        assert errs[algo][0] <= 2 * base[0] and errs[algo][1] <= 2 * base[1], errs


@pytest.mark.parametrize("sa,sb", [(1e-30, 1e25), (1e30, 1e-32), (3e-8, 1.0), (0.0, 1.0)])
def test_gemm_f16x2_scales(sa, sb):
    """Split-fp16 operand scaling: operands far outside fp16 range (either direction), a zero
    operand, plus a product through caller-supplied maxima (mvml_gemm_f16x2_amax) and the
    mvml_absmax_f32 pass itself (bits of max |x|)."""
    from mvml_gat import _lib
    from mvml_gat.functional import absmax, gemm, ptr, slot, _stream
    g = torch.Generator().manual_seed(5)
    M, N, K = 700, 520, 300
    A = torch.randn(M, K, generator=g, dtype=torch.float64) * sa
    B = torch.randn(K, N, generator=g, dtype=torch.float64) * sb
    ref = A @ B
    Ad, Bd = A.float().to(DEV), B.t().contiguous().float().to(DEV)
    C = torch.zeros(M, N, device=DEV)
    with _x3_tile("f16x2-256") as a:
        gemm(Ad, Bd, M, N, K, 0, 0, K, K, C, N, algo=a)
    if sa == 0.0:
        assert torch.count_nonzero(C).item() == 0
    else:
        assert rel_err(C, ref) < TOL
    amx = torch.zeros(2, dtype=torch.int32, device=DEV)
    absmax(Ad, M, K, K, amx, 0)
    absmax(Bd, N, K, K, amx, 1)
    got = amx.cpu().view(torch.float32)
    assert got[0].item() == Ad.abs().max().item() and got[1].item() == Bd.abs().max().item()
    C2 = torch.zeros(M, N, device=DEV)
    L = _lib.lib()
    wsz = L.mvml_gemm_workspace_size(M, N, K)
    wp, wn = _lib.ws_ptr_size(wsz, DEV)
    with _x3_tile("f16x2-256"):
        _lib.call("mvml_gemm_f16x2_amax", 0, 0, M, N, K, ptr(Ad), K, ptr(Bd), K, slot(amx, 0),
                  slot(amx, 1), None, 0.0, 0, ptr(C2), N, wp, wn, _stream(C2.device))
    assert torch.equal(C, C2)


@pytest.mark.parametrize("ak,bk", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(1000, 1928, 768), (257, 300, 74), (4100, 768, 1928),
                                   (512, 384, 65536 + 17), (6144, 520, 40), (300, 260, 16)])
def test_gemm_f16x2_256_layouts(ak, bk, M, N, K):
    """The split-fp16 256x256 tile on every operand layout — K tails (K % 16 != 0), ragged M / N
    edges, split-K, the N = 256 q + r split, bias / beta / ReLU epilogue — within the fp32 bar
    of float64.  (Rounds 3-5 ran it against the LDS-DMA ring kernel too; the ring was removed in
    round 6.)"""
    from mvml_gat.functional import gemm
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K + ak + 2 * bk)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    B = torch.randn(K, N, generator=g, dtype=torch.float64)
    bias = torch.randn(N, generator=g, dtype=torch.float64)
    C0 = torch.randn(M, N, generator=g, dtype=torch.float64)
    Ad = (A.t() if ak else A).contiguous().float().to(DEV)
    Bd = (B if bk else B.t()).contiguous().float().to(DEV)
    C = C0.float().to(DEV)
    with _x3_tile("f16x2-256") as a:
        gemm(Ad, Bd, M, N, K, ak, bk, M if ak else K, N if bk else K, C, N,
             bias=bias.float().to(DEV), beta=0.5, act=1, algo=a)
    assert rel_err(C, torch.relu(A @ B + bias + 0.5 * C0)) < TOL


@pytest.mark.parametrize("ak,bk", [(1, 1), (0, 1), (0, 0), (1, 0)])
@pytest.mark.parametrize("M,N,K,batch", [(384, 384, 384, 12), (100, 70, 36, 3), (300, 260, 520, 2)])
def test_gemm_batched(ak, bk, M, N, K, batch):
    """mvml_gemm_f32x3_batched: product z at operand strides, C blocks side by side in one wide
    matrix (column stride, as the fusion head's [M_1 .. M_H] panel), beta onto C."""
    from mvml_gat.functional import gemm_batched
    g = torch.Generator().manual_seed(M + N + K + batch)
    A = torch.randn(batch, M, K, generator=g, dtype=torch.float64)
    B = torch.randn(batch, K, N, generator=g, dtype=torch.float64)
    Np = ((N + 3) // 4) * 4
    C0 = torch.randn(M, batch * Np, generator=g, dtype=torch.float64)
    Ad = (A.transpose(1, 2) if ak else A).contiguous().float().to(DEV)
    Bd = (B if bk else B.transpose(1, 2)).contiguous().float().to(DEV)
    C = C0.float().to(DEV)
    gemm_batched(Ad, Bd, M, N, K, ak, bk, M if ak else K, N if bk else K, C, batch * Np, batch,
                 M * K, K * N, Np, beta=0.5)
    ref = C0.clone()
    for z in range(batch):
        ref[:, z * Np:z * Np + N] = A[z] @ B[z] + 0.5 * C0[:, z * Np:z * Np + N]
    assert rel_err(C, ref) < TOL


def test_gemm_two_streams_concurrent():
    """Split-K GEMMs (which use workspace slabs) enqueued on two streams at once: each stream
    has its own scratch, so neither result is corrupted by the other's partial sums."""
    from mvml_gat import _lib
    from mvml_gat.functional import gemm
    g = torch.Generator().manual_seed(9)
    M, N, K = 384, 76, 200000  # long K: split-K with slabs in the workspace
    As = [torch.randn(K, M, generator=g) for _ in range(2)]
    Bs = [torch.randn(K, N, generator=g) for _ in range(2)]
    refs = [(a.double().t() @ b.double()) for a, b in zip(As, Bs)]
    Ad = [a.to(DEV) for a in As]
    Bd = [b.to(DEV) for b in Bs]
    Cs = [torch.zeros(M, N, device=DEV) for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    for rep in range(3):
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                gemm(Ad[i], Bd[i], M, N, K, 1, 1, M, N, Cs[i], N)
    torch.cuda.synchronize()
    keys = {k for k in _lib._ws if k[1] in (s.cuda_stream for s in streams)}
    assert len(keys) == 2, keys
    for C, ref in zip(Cs, refs):
        assert rel_err(C, ref) < TOL


def test_colsum():
    from mvml_gat.functional import colsum
    X = torch.randn(5000, 37, dtype=torch.float64)
    out = torch.ones(37, dtype=torch.float32, device=DEV)
    colsum(X.float().to(DEV), 5000, 37, 37, out, beta=1.0)
    assert rel_err(out, X.sum(0) + 1) < TOL
    # tall: ~1 K row partials per column (the final pass's 16 stripes x 4 accumulators), a
    # column count that is not a multiple of 16, alpha scaling
    X = torch.randn(200003, 517, dtype=torch.float64)
    out = torch.empty(517, dtype=torch.float32, device=DEV)
    colsum(X.float().to(DEV), 200003, 517, 517, out, alpha=0.5)
    assert rel_err(out, 0.5 * X.sum(0)) < TOL


# ------------------------------------------------------------------ GAT layers
def _gat_case(layer, sb, seed=0):
    torch.manual_seed(seed)
    prod, ref = model_pair(seed=seed)
    conv_p = prod.conv.gnn_layers[layer]
    conv_r = ref.conv.gnn_layers[layer].gat_conv
    Fin = 74 if layer == 0 else 768
    X = torch.randn(int(sb.num_nodes.sum()), Fin, dtype=torch.float64)
    if layer == 0:
        X = torch.as_tensor(sb.feats, dtype=torch.float64) + 0.1 * X
    gd = graph_dict(sb)
    H, Fo = 4, (192 if layer == 0 else 384)
    params = {"fc.weight": conv_r.fc.weight, "res_fc.weight": conv_r.res_fc.weight,
              "attn_l": conv_r.attn_l, "attn_r": conv_r.attn_r, "bias": conv_r.bias}
    params64 = {k: v.detach().double().requires_grad_() for k, v in params.items()}
    Xr = X.clone().requires_grad_()
    out_r = gnn_ref.gat_layer_ref(gd["src"], gd["dst"], Xr, params64, H, Fo,
                                  "flatten" if layer == 0 else "mean",
                                  torch.nn.functional.elu if layer == 0 else None)
    gout = torch.randn_like(out_r)
    out_r.backward(gout)

    conv_p = conv_p.to(DEV)
    g = _to_dev(sb)
    Xp = X.float().to(DEV).requires_grad_()
    out_p = conv_p(g, Xp)
    out_p.backward(gout.float().to(DEV))
    assert rel_err(out_p, out_r) < TOL, "forward"
    assert rel_err(Xp.grad, Xr.grad) < TOL, "dX"
    c = conv_p.gat_conv
    for name, pp in (("fc.weight", c.fc.weight), ("res_fc.weight", c.res_fc.weight),
                     ("attn_l", c.attn_l), ("attn_r", c.attn_r), ("bias", c.bias)):
        assert rel_err(pp.grad, params64[name].grad) < TOL, name


@pytest.mark.parametrize("layer", [0, 1])
def test_gat_layer_parity(layer):
    _gat_case(layer, batch_of_sizes([25, 11, 40, 23, 17, 3, 1], seed=5))


def test_gat_layer_hubs_parity():
    # in-degree > 64 exercises the multi-chunk softmax / backward paths
    _gat_case(1, batch_of_sizes([150, 90], seed=7, hubs=True))


# ------------------------------------------------------------------ readout / norm
def test_set2set_parity():
    from mvml_gat.nn import Set2Set
    sb = batch_of_sizes([25, 1, 40, 7, 23], seed=9)
    gd = graph_dict(sb)
    torch.manual_seed(0)
    s2s = Set2Set(384, 6, 3)
    X = torch.randn(int(sb.num_nodes.sum()), 384, dtype=torch.float64)
    lstm64 = torch.nn.LSTM(768, 384, 3).double()
    lstm64.load_state_dict({k: v.double() for k, v in s2s.lstm.state_dict().items()})
    Xr = X.clone().requires_grad_()
    out_r = gnn_ref.set2set_ref(gd["node_offsets"], Xr, lstm64, 6)
    gout = torch.randn_like(out_r)
    out_r.backward(gout)
    s2s = s2s.to(DEV)
    Xp = X.float().to(DEV).requires_grad_()
    out_p = s2s(_to_dev(sb), Xp)
    out_p.backward(gout.float().to(DEV))
    assert rel_err(out_p, out_r) < TOL
    assert rel_err(Xp.grad, Xr.grad) < TOL
    for (n, p), (n2, p2) in zip(s2s.lstm.named_parameters(), lstm64.named_parameters()):
        assert rel_err(p.grad, p2.grad) < TOL, n


@pytest.mark.parametrize("tile", [0, 128])
def test_set2set_cell_epilogue_bitwise(tile):
    """Set2Set at a width where the gates GEMM takes the 256x256 plan (16,384 molecules): the
    fused gates + LSTM-cell epilogue (mvml_lstm_gates_cell_fwd) equals the GEMM + cell kernel
    path bit for bit (same MFMA accumulation per element, same cell arithmetic), forward and
    backward, on the 256x256 split-fp16 kernel and on the 128x128 one (tile = 128: option
    lstm_tile); the unfused path is the one pinned to the float64 oracle above."""
    import mvml_gat.functional as fn
    from mvml_gat import _lib
    from mvml_gat._lib import option
    opt_t = option("lstm_tile", tile)
    opt_t.__enter__()
    from mvml_gat.nn import Set2Set
    sb = batch_of_sizes([3, 5, 2, 7] * 4096, seed=4)
    assert _lib.lib().mvml_lstm_gates_cell_plan_ok(16384, 384, 1152)
    g = _to_dev(sb)
    torch.manual_seed(1)
    s2s = Set2Set(384, 6, 3).to(DEV)
    X = torch.randn(int(sb.num_nodes.sum()), 384, device=DEV)
    gout = torch.randn(16384, 768, device=DEV)
    res = []
    for fused in (True, False):
        old = fn.CELL_EPI
        fn.CELL_EPI = fused
        try:
            s2s.zero_grad()
            Xp = X.clone().requires_grad_()
            out = s2s(g, Xp)
            out.backward(gout)
            res.append([out.detach().clone(), Xp.grad.clone()] + [p.grad.clone() for p in s2s.parameters()])
        finally:
            fn.CELL_EPI = old
    opt_t.__exit__(None, None, None)
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_graphnorm_parity():
    from mvml_gat.nn import GraphNorm
    x = torch.randn(164, 768, dtype=torch.float64) * 3 + 1
    gn = GraphNorm(768)
    with torch.no_grad():
        gn.weight.add_(torch.randn(768) * 0.1)
        gn.bias.add_(torch.randn(768) * 0.1)
        gn.mean_scale.add_(torch.randn(768) * 0.1)
    offs = [0, 64, 128, 164]
    w, b, ms = (p.detach().double().requires_grad_() for p in (gn.weight, gn.bias, gn.mean_scale))
    xr = x.clone().requires_grad_()
    yr = gnn_ref.graphnorm_ref(xr, w, b, ms, 1e-5, offs)
    gy = torch.randn_like(yr)
    yr.backward(gy)
    gn = gn.to(DEV)
    xp = x.float().to(DEV).requires_grad_()
    yp = gn(xp, group_offsets=torch.tensor(offs, device=DEV))
    yp.backward(gy.float().to(DEV))
    assert rel_err(yp, yr) < TOL
    assert rel_err(xp.grad, xr.grad) < TOL
    for a, r in ((gn.weight, w), (gn.bias, b), (gn.mean_scale, ms)):
        assert rel_err(a.grad, r.grad) < TOL


@pytest.mark.parametrize("G,D,big", [(1000, 100, False), (37, 768, False), (1, 20, False), (6, 300, True)])
def test_graphnorm_param_reduce_many_groups(G, D, big):
    """The parameter gradients' reduction over G group partials (16 stripes per column, a fixed
    tree) at group counts around its stripe / unroll boundaries and a column count that is not a
    multiple of 16, against float64.  big: groups of 63-130 rows, on both sides of the kernels'
    64-row register path (longer groups re-read their rows)."""
    from mvml_gat.nn import GraphNorm
    gen = torch.Generator().manual_seed(G + D)
    sizes = torch.randint(63, 131, (G,), generator=gen) if big else torch.randint(1, 6, (G,), generator=gen)
    if big:
        sizes[:3] = torch.tensor([64, 65, 63])
    offs = [0] + torch.cumsum(sizes, 0).tolist()
    x = torch.randn(offs[-1], D, dtype=torch.float64, generator=gen) * 2 + 0.5
    gn = GraphNorm(D)
    with torch.no_grad():
        gn.weight.add_(torch.randn(D, generator=gen) * 0.1)
        gn.mean_scale.add_(torch.randn(D, generator=gen) * 0.1)
    w, b, ms = (p.detach().double().requires_grad_() for p in (gn.weight, gn.bias, gn.mean_scale))
    xr = x.clone().requires_grad_()
    yr = gnn_ref.graphnorm_ref(xr, w, b, ms, 1e-5, offs)
    gy = torch.randn(yr.shape, dtype=torch.float64, generator=gen)
    yr.backward(gy)
    gn = gn.to(DEV)
    xp = x.float().to(DEV).requires_grad_()
    yp = gn(xp, group_offsets=torch.tensor(offs, device=DEV))
    yp.backward(gy.float().to(DEV))
    assert rel_err(yp, yr) < TOL
    assert rel_err(xp.grad, xr.grad) < TOL
    for a, r in ((gn.weight, w), (gn.bias, b), (gn.mean_scale, ms)):
        assert rel_err(a.grad, r.grad) < TOL


# ------------------------------------------------------------------ full GNNModule
def test_gnn_module_parity_eval_and_grads():
    sb = batch_of_sizes([25, 11, 40, 23, 17, 3, 1, 60, 33], seed=11)
    prod, ref = model_pair(seed=3)
    prod.eval()
    ref.eval()
    ref64 = ref.double()
    gd = graph_dict(sb)
    X = torch.as_tensor(sb.feats, dtype=torch.float64)
    out_r = ref64(gd, X)
    gout = torch.randn_like(out_r)
    out_r.backward(gout)
    prod = prod.to(DEV)
    g = _to_dev(sb)
    out_p = prod(g, g.ndata["h"])
    out_p.backward(gout.float().to(DEV))
    assert rel_err(out_p, out_r) < TOL
    pr = dict(ref64.named_parameters())
    for n, p in prod.named_parameters():
        assert rel_err(p.grad, pr[n].grad) < TOL, n


def test_gnn_module_groups_equal_separate_batches():
    """GraphNorm groups in one launch == the reference run batch by batch."""
    sb = batch_of_sizes([20] * 5 + [30] * 4, seed=2)
    prod, _ = model_pair(seed=4)
    prod = prod.to(DEV).eval()
    with torch.no_grad():
        g = _to_dev(sb, group_size=5)
        y_all = prod(g, g.ndata["h"])
        from mvml_gat import from_arrays
        ys = []
        for lo, hi in ((0, 5), (5, 9)):
            e0, e1 = int(sb.num_edges[:lo].sum()), int(sb.num_edges[:hi].sum())
            n0, n1 = int(sb.num_nodes[:lo].sum()), int(sb.num_nodes[:hi].sum())
            gi = from_arrays(sb.num_nodes[lo:hi], sb.num_edges[lo:hi], sb.src_local[e0:e1],
                             sb.dst_local[e0:e1], sb.feats[n0:n1]).to(DEV)
            ys.append(prod(gi, gi.ndata["h"]))
    assert rel_err(y_all, torch.cat(ys)) < TOL


def test_deterministic_bitwise():
    sb = batch_of_sizes([25, 11, 40, 23], seed=1)
    prod, _ = model_pair(seed=5)
    prod = prod.to(DEV).eval()
    res = []
    for _ in range(2):
        prod.zero_grad()
        g = _to_dev(sb)
        y = prod(g, g.ndata["h"])
        y.sum().backward()
        res.append([y.detach().clone()] + [p.grad.clone() for p in prod.parameters()])
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_zero_in_degree_raises():
    from mvml_gat import batching as G
    prod, _ = model_pair(seed=0)
    prod = prod.to(DEV)
    g = G.graph(([0], [1]), num_nodes=2, ndata={"h": torch.randn(2, 74)})
    bg = G.batch([g]).to(DEV)
    with pytest.raises(RuntimeError, match="0-in-degree"):
        prod(bg, bg.ndata["h"])


@pytest.mark.parametrize("kmajor", [0, 1])
def test_gemm_f16x2_row_dynamic_range(kmajor):
    """the split-fp16 scale is one power of two per operand (from its |max|), so its
    accuracy is norm-wise; rows far below the operand's max lose relative precision once their
    low fp16 plane goes subnormal (~2^17 below the max).  Rows of A are scaled 2^0, 2^-8 ...
    2^-28; the per-row relative error max_j |C_ij - C64_ij| / max_j |C64_ij| is measured for
    the split-fp16 and the f32-input MFMA GEMMs and written to the margins directory; the test
    holds split-fp16 rows within 2^-20 of the max to the fp32 bar (1e-5) — the documented
    guarantee (GEMM) — and every row to the norm-wise bar."""
    import json
    import os
    from mvml_gat.functional import gemm
    g = torch.Generator().manual_seed(11 + kmajor)
    M, N, K = 1024, 384, 768
    exps = torch.tensor([0, 8, 12, 16, 18, 20, 22, 24, 28], dtype=torch.float64)
    row_exp = exps[torch.arange(M) % len(exps)]
    A = torch.randn(M, K, generator=g, dtype=torch.float64) * torch.pow(2.0, -row_exp).unsqueeze(1)
    A = A.float().double()
    B = torch.randn(K, N, generator=g, dtype=torch.float64).float().double()
    ref = A @ B
    Bd = B.t().contiguous().float().to(DEV)
    res = {}
    for algo, tile in (("f16x2", "f16x2-256"), ("f32", "f32")):
        C = torch.zeros(M, N, device=DEV)
        with _x3_tile(tile) as a:
            if kmajor:
                gemm(A.t().contiguous().float().to(DEV), Bd, M, N, K, 1, 0, M, K, C, N, algo=a)
            else:
                gemm(A.float().to(DEV), Bd, M, N, K, 0, 0, K, K, C, N, algo=a)
        d = (C.double().cpu() - ref).abs().max(1).values / ref.abs().max(1).values
        res[algo] = {int(e): d[row_exp == e].max().item() for e in exps.tolist()}
        res[algo]["normwise"] = rel_err(C, ref)
    out = os.environ.get("MVML_MARGINS_DIR", os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "gpurun_out", "parity_margins"))
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, f"gemm_row_dynamic_range_k{kmajor}.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(res)
    assert res["f16x2"]["normwise"] < TOL
    for e in exps.tolist():
        if e <= 20:
            assert res["f16x2"][int(e)] < TOL, (e, res)
