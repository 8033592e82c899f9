"""Oracle: molecule bigraph construction, batching and CSR indices (numpy, integer-exact).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Restates:

* a1  dgllife 0.3.0 ``construct_bigraph_from_mol`` as called by ``mol_to_bigraph(mol,
      add_self_loop=True, ...)`` at dataset.py:34-35: for bond i (bond-index order) append
      (u_i -> v_i), (v_i -> u_i); then one self-loop per atom 0..n-1; ids int32.
* a3  dgl 0.9.1 ``dgl.batch`` as called by ``collate`` at dataset.py:54: node offsets are
      the exclusive cumsum of per-graph node counts, edges are concatenated in graph order
      with src/dst shifted by the graph's node offset; ``batch_num_nodes/edges`` are int64.
* a4  the in-CSR DGL builds for ``update_all`` / ``edge_softmax`` (rows = dst, stable
      counting sort, so a row lists its in-edges in ascending edge id) and the matching
      out-CSR (rows = src) used by the atomic-free backward.
"""
import numpy as np


def bigraph_edges(num_atoms, bonds):
    """Edges of one molecule in mol_to_bigraph order (dataset.py:34, a1)."""
    bonds = np.asarray(bonds, dtype=np.int64).reshape(-1, 2)
    nb = bonds.shape[0]
    src = np.empty(2 * nb + num_atoms, dtype=np.int32)
    dst = np.empty(2 * nb + num_atoms, dtype=np.int32)
    src[0:2 * nb:2] = bonds[:, 0]
    dst[0:2 * nb:2] = bonds[:, 1]
    src[1:2 * nb:2] = bonds[:, 1]
    dst[1:2 * nb:2] = bonds[:, 0]
    src[2 * nb:] = np.arange(num_atoms, dtype=np.int32)
    dst[2 * nb:] = np.arange(num_atoms, dtype=np.int32)
    return src, dst


def batch_ref(num_nodes, src_local, dst_local, num_edges):
    """dgl.batch restated (dataset.py:54, a3).

    num_nodes, num_edges: int64[B]; src_local/dst_local: int32[E] = per-graph local ids
    concatenated in graph order.  Returns a dict of numpy arrays.
    """
    num_nodes = np.asarray(num_nodes, dtype=np.int64)
    num_edges = np.asarray(num_edges, dtype=np.int64)
    node_off = np.zeros(len(num_nodes) + 1, dtype=np.int64)
    edge_off = np.zeros(len(num_edges) + 1, dtype=np.int64)
    np.cumsum(num_nodes, out=node_off[1:])
    np.cumsum(num_edges, out=edge_off[1:])
    edge_graph = np.repeat(np.arange(len(num_edges)), num_edges)
    shift = node_off[:-1][edge_graph]
    src = (np.asarray(src_local, dtype=np.int64) + shift).astype(np.int32)
    dst = (np.asarray(dst_local, dtype=np.int64) + shift).astype(np.int32)
    node_graph = np.repeat(np.arange(len(num_nodes)), num_nodes).astype(np.int32)
    return dict(node_offsets=node_off, edge_offsets=edge_off, src=src, dst=dst,
                node_graph=node_graph, batch_num_nodes=num_nodes, batch_num_edges=num_edges)


def csr_ref(src, dst, num_nodes_total):
    """In-CSR (rows = dst) and out-CSR (rows = src), both stable in edge id (a4).

    Returns in_rowptr[N+1], in_src[E], in_eid[E], out_rowptr[N+1], out_dst[E],
    out_inslot[E] (the in-CSR slot of each out-CSR edge), all int32, plus the
    number of zero in-degree nodes (GATConv raises on those unless
    allow_zero_in_degree, dgl 0.9.1 GATConv.forward).
    """
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    n = int(num_nodes_total)
    in_eid = np.argsort(dst, kind="stable")
    in_deg = np.bincount(dst, minlength=n)
    in_rowptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(in_deg, out=in_rowptr[1:])
    in_src = src[in_eid]
    inslot_of_eid = np.empty_like(in_eid)
    inslot_of_eid[in_eid] = np.arange(len(in_eid))
    out_eid = np.argsort(src, kind="stable")
    out_deg = np.bincount(src, minlength=n)
    out_rowptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(out_deg, out=out_rowptr[1:])
    out_dst = dst[out_eid]
    out_inslot = inslot_of_eid[out_eid]
    zero_in = int((in_deg == 0).sum())
    i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)
    return dict(in_rowptr=i32(in_rowptr), in_src=i32(in_src), in_eid=i32(in_eid),
                out_rowptr=i32(out_rowptr), out_dst=i32(out_dst), out_inslot=i32(out_inslot),
                zero_in_degree=zero_in)


def node_group_plan_ref(node_offsets, in_rowptr, group_atoms=64, win_atoms=128, edge_cap=512,
                        deg_cap=5, big_atoms=512, big_edge_cap=2432):
    """Node-group plan of mvml_build_node_groups (launch geometry; no reference counterpart):
    group g starts at the first atom of the molecule containing atom group_atoms*g; kind bit 0
    = forward LDS kernel (atom, edge and in-degree caps), bit 1 = backward LDS kernel (atom and
    edge caps).  Returns (starts [G+1], kinds [G], fwd fallback set, bwd fallback set)."""
    node_offsets = np.asarray(node_offsets, dtype=np.int64)
    rp = np.asarray(in_rowptr, dtype=np.int64)
    N = int(node_offsets[-1])
    G = -(-N // group_atoms) if N > 0 else 0
    starts = np.empty(G + 1, dtype=np.int32)
    for g in range(G):
        m = np.searchsorted(node_offsets, g * group_atoms, side="right") - 1
        starts[g] = node_offsets[m]
    starts[G] = N
    kinds = np.zeros(G, dtype=np.int32)
    fwd, bwd = set(), set()
    for g in range(G):
        a0, a1 = int(starts[g]), int(starts[g + 1])
        if a1 <= a0:
            continue
        fits = a1 - a0 <= win_atoms and rp[a1] - rp[a0] <= edge_cap
        dmax = int(np.max(rp[a0 + 1:a1 + 1] - rp[a0:a1]))
        big = a1 - a0 <= big_atoms and rp[a1] - rp[a0] <= big_edge_cap
        kinds[g] = (1 if fits and dmax <= deg_cap else 0) | (2 if fits else 0) | (4 if big else 0)
        if not kinds[g] & 1:
            fwd.add(g)
        if not kinds[g] & 2:
            bwd.add(g)
    return starts, kinds, fwd, bwd
