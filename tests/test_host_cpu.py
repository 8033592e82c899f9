"""CPU tests of the host side: graph construction/batching logic, the synthetic generators, the
C-ABI library (loads, exports every header symbol, validates arguments without a GPU) and the
no-CPU-fallback guarantee."""
import ctypes
import re

import numpy as np
import pytest
import torch

import mvml_gat
from mvml_gat import _lib, batching, synth
from oracle import graph_ref


# ------------------------------------------------------------------ graphs / batching
def test_bigraph_matches_oracle():
    bonds = [(0, 1), (1, 2), (2, 0), (2, 3)]
    g = batching.bigraph_from_bonds(4, bonds)
    s, d = graph_ref.bigraph_edges(4, bonds)
    np.testing.assert_array_equal(g.src, s)
    np.testing.assert_array_equal(g.dst, d)


def test_host_batch_edges_match_dgl_batch_semantics():
    sb = synth.config3(50, seed=3)
    bg = sb.to_graph()
    ref = graph_ref.batch_ref(sb.num_nodes, sb.src_local, sb.dst_local, sb.num_edges)
    s, d = bg.edges()
    np.testing.assert_array_equal(s.numpy(), ref["src"])
    np.testing.assert_array_equal(d.numpy(), ref["dst"])
    assert bg.batch_size == 50 and bg.num_nodes() == int(sb.num_nodes.sum())
    assert torch.equal(bg.batch_num_nodes(), torch.as_tensor(sb.num_nodes))


def test_csr_oracle_invariants():
    sb = synth.config3(20, seed=1)
    ref = graph_ref.batch_ref(sb.num_nodes, sb.src_local, sb.dst_local, sb.num_edges)
    N = int(ref["node_offsets"][-1])
    c = graph_ref.csr_ref(ref["src"], ref["dst"], N)
    for v in range(N):
        row = c["in_eid"][c["in_rowptr"][v]:c["in_rowptr"][v + 1]]
        assert np.all(np.diff(row) > 0)
        assert np.all(ref["dst"][row] == v)
        orow = slice(c["out_rowptr"][v], c["out_rowptr"][v + 1])
        eids = c["in_eid"][c["out_inslot"][orow]]
        assert np.all(ref["src"][eids] == v) and np.all(np.diff(eids) > 0)
    assert c["zero_in_degree"] == 0


def test_group_offsets():
    sb = synth.config2(130, seed=0)
    bg = sb.to_graph(group_size=64)
    assert list(bg.group_offsets_host()) == [0, 64, 128, 130]
    assert list(sb.to_graph().group_offsets_host()) == [0, 130]


# ------------------------------------------------------------------ synthetic data
def _check_onehots(X):
    blocks = [(0, 43), (43, 54), (54, 61), (63, 68), (69, 74)]
    for a, b in blocks:
        assert np.all(X[:, a:b].sum(1) == 1), (a, b)


def test_config2_shapes():
    sb = synth.config2(256, seed=0)
    assert np.all(sb.num_nodes == 25) and np.all(sb.num_edges == 79)
    _check_onehots(sb.feats)
    ref = graph_ref.batch_ref(sb.num_nodes, sb.src_local, sb.dst_local, sb.num_edges)
    deg = np.bincount(ref["dst"], minlength=int(sb.num_nodes.sum())) - 1  # minus self-loop
    assert deg.max() <= 4
    assert np.all((sb.feats[:, 43:54].argmax(1)) == deg)


def test_config3_size_distribution():
    sb = synth.config3(4000, seed=0)
    assert sb.num_nodes.min() >= 11 and sb.num_nodes.max() <= 80
    assert 21 <= np.median(sb.num_nodes) <= 25
    _check_onehots(sb.feats)


def test_config5_hubs():
    sb = synth.config5(6, seed=1)
    assert sb.num_nodes.min() >= 150 and sb.num_nodes.max() <= 400
    ref = graph_ref.batch_ref(sb.num_nodes, sb.src_local, sb.dst_local, sb.num_edges)
    indeg = np.bincount(ref["dst"])
    assert indeg.max() >= 33


# ------------------------------------------------------------------ C ABI
def test_library_exports_every_header_symbol():
    text = open(_lib.HEADER_PATH).read()
    declared = set(re.findall(r"\b(mvml_\w+)\s*\(", re.sub(r"/\*.*?\*/", "", text, flags=re.S)))
    assert len(declared) >= 20
    L = _lib.lib()
    for name in declared:
        assert hasattr(L, name), name
    assert set(_lib.exported_symbols()) == declared
    assert L.mvml_version().startswith(b"mvml_gat")


def test_abi_argument_validation_without_gpu():
    L = _lib.lib()
    rc = L.mvml_gemm_f32(0, 0, -1, 4, 4, None, 4, None, 4, None, 0.0, 0, None, 4, None, 0, None)
    assert rc == 1 and b"negative" in L.mvml_last_error()
    rc = L.mvml_gat_agg_fwd(10, None, 1, None, None, None, 3 * 8 * 2, 3, 8, None, None, 0.2, 0, None, None, None,
                            None, None)
    assert rc == 1 and b"num_heads" in L.mvml_last_error()
    rc = L.mvml_build_csr(None, None, None, None, 1, 1 << 31, 5, *([None] * 12), None, 0, None)
    assert rc == 1 and b"overflow" in L.mvml_last_error()
    assert L.mvml_gemm_workspace_size(3080, 768, 1_000_000) > 0
    assert L.mvml_gemm_workspace_size(100000, 3080, 768) == 256  # the split-fp16 maxima only
    rc = L.mvml_gemm_f16x2_amax(0, 0, 4, 4, 4, None, 4, None, 4, None, None, None, 0.0, 0, None, 4, None, 0, None)
    assert rc == 1 and b"amax" in L.mvml_last_error()
    rc = L.mvml_absmax_f32(-1, 4, None, 4, None, 0, None)
    assert rc == 1 and b"absmax" in L.mvml_last_error()


def test_no_cpu_fallback():
    model = mvml_gat.GNNModule(74, [192, 384], 0.5, 6, 3)
    sb = synth.config2(4, seed=0)
    bg = sb.to_graph()
    with pytest.raises(RuntimeError):
        model(bg, bg.ndata["h"])


def test_state_dict_layout_matches_reference():
    from oracle.gnn_ref import GNNModuleRef
    prod = mvml_gat.GNNModule(74, [192, 384], 0.5, 6, 3)
    ref = GNNModuleRef(74, [192, 384], 0.5, 6, 3)
    ps, rs = prod.state_dict(), ref.state_dict()
    assert list(ps.keys()) == list(rs.keys())
    assert all(ps[k].shape == rs[k].shape for k in ps)
    assert sum(p.numel() for p in prod.parameters()) == 6_915_456
    keys = list(ps.keys())
    assert keys[:5] == ["conv.gnn_layers.0.gat_conv.attn_l", "conv.gnn_layers.0.gat_conv.attn_r",
                        "conv.gnn_layers.0.gat_conv.bias", "conv.gnn_layers.0.gat_conv.fc.weight",
                        "conv.gnn_layers.0.gat_conv.res_fc.weight"]


@pytest.mark.parametrize("which", ["gnn", "mvp"])
def test_state_dict_accepts_folded_residual_bias(which):
    """both DGL GATConv layouts load with strict=True — the explicit
    ``gat_conv.bias`` (dgl 0.9.1, what state_dict() writes) and the later releases' bias folded
    into the projecting residual (``gat_conv.res_fc.bias``, no ``bias``); the arithmetic is the
    same, so the folded tensor becomes ``bias``."""
    from mvml_gat.mvp import MVP
    torch.manual_seed(0)
    make = (lambda: mvml_gat.GNNModule(74, [192, 384], 0.5, 6, 3)) if which == "gnn" else \
        (lambda: MVP(11, 74, [192, 384], 6, 3, 128, 384, 2, 512, 12, 0.5))
    src, dst = make(), make()
    for p in src.parameters():
        p.data.uniform_(-1, 1)
    sd = src.state_dict()
    folded = {}
    for k, v in sd.items():
        if k.endswith("gat_conv.bias"):
            folded[k[:-len("bias")] + "res_fc.bias"] = v.clone()
        else:
            folded[k] = v.clone()
    assert not any(k.endswith("gat_conv.bias") for k in folded)
    dst.load_state_dict(folded, strict=True)
    for (k, a), (k2, b) in zip(src.state_dict().items(), dst.state_dict().items()):
        assert k == k2 and torch.equal(a, b), k
    dst.load_state_dict(sd, strict=True)  # and the explicit layout still loads


# ------------------------------------------------------------------ fusion head / node groups
def test_fusion_state_dict_matches_reference_layout():
    """MVFusion carries MVP's fusion parameters under MVP's names and shapes (model.py:23-45)."""
    from oracle.fusion_ref import MVFusionRef
    ref, mod = MVFusionRef(), mvml_gat.MVFusion()
    assert {k: tuple(v.shape) for k, v in ref.state_dict().items()} == \
           {k: tuple(v.shape) for k, v in mod.state_dict().items()}
    assert tuple(mod.linear_q.weight.shape) == (4608, 384) and mod.mlp[3].out_features == 11


def test_node_group_plan_oracle_invariants():
    """Every group is a run of whole molecules, groups tile the atoms, and the kinds route
    exactly the groups that exceed the LDS kernels' caps to the fallback lists."""
    sb = synth.config5(12, seed=2)  # 150-400-atom molecules with hubs: fallback groups too
    ref = graph_ref.batch_ref(sb.num_nodes, sb.src_local, sb.dst_local, sb.num_edges)
    N = int(ref["node_offsets"][-1])
    csr = graph_ref.csr_ref(ref["src"], ref["dst"], N)
    starts, kinds, fwd, bwd = graph_ref.node_group_plan_ref(ref["node_offsets"], csr["in_rowptr"])
    mol_starts = set(int(x) for x in ref["node_offsets"])
    assert starts[0] == 0 and starts[-1] == N and np.all(np.diff(starts) >= 0)
    assert all(int(s) in mol_starts for s in starts)
    rp = csr["in_rowptr"]
    for g in range(len(kinds)):
        a0, a1 = int(starts[g]), int(starts[g + 1])
        if a1 == a0:
            assert kinds[g] == 0 and g not in fwd and g not in bwd
            continue
        # edges stay inside the group (molecule-closed)
        srcs = csr["in_src"][rp[a0]:rp[a1]]
        assert srcs.min() >= a0 and srcs.max() < a1
        fits = a1 - a0 <= 128 and rp[a1] - rp[a0] <= 512
        assert bool(kinds[g] & 2) == fits and (g in bwd) == (not fits)
        assert bool(kinds[g] & 1) == (fits and np.max(np.diff(rp[a0:a1 + 1])) <= 5)
