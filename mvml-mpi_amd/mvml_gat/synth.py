"""Seeded synthetic drug-like molecule batches (BASELINE.json configs 2, 3 and 5).

No RDKit / no network: molecules are random chemical-looking graphs, vectorised over many
molecules at once.  Every molecule is emitted exactly as mol_to_bigraph(add_self_loop=True)
would lay it out (dataset.py:34): bond i -> edges (u_i, v_i), (v_i, u_i); then one self-loop
per atom.  Atom features are valid 74-d CanonicalAtomFeaturizer vectors (dgllife 0.3.0):
  [0,43) atom type one-hot | [43,54) degree | [54,61) implicit valence | 61 formal charge |
  62 radical electrons | [63,68) hybridisation SP..SP3D2 | 68 aromatic | [69,74) total H.

* config2(n_mols)  25 atoms, 27 bonds (tree + 3 ring closures, degree <= 4)      seed 0
* config3(n_mols)  KEGG-like sizes: median 23 atoms, clipped to 11-80, ~2.4 rings  seed 0
* config5(n_mols)  150-400 atoms + 1-4 hub atoms with 32-128 extra bonds each       seed 1
"""
import numpy as np

FEAT_DIM = 74
# C, N, O, S, F, Si, P, Cl, Br, I  (indices into dgllife's 43-symbol list)
_TYPE_IDX = np.array([0, 1, 2, 3, 4, 5, 6, 7, 8, 15])
_TYPE_P = np.array([0.70, 0.12, 0.13, 0.015, 0.01, 0.002, 0.01, 0.008, 0.003, 0.002])
_VALENCE = np.array([4, 3, 2, 2, 1, 4, 3, 1, 1, 1])


def _tree_and_rings(rng, M, n, n_rings):
    """Bonds (M, n-1+max_rings) int32 with -1 padding, and the number of bonds per molecule."""
    deg = np.zeros((M, n), dtype=np.int32)
    rows = np.arange(M)
    R = int(n_rings.max()) if M else 0
    bonds = np.full((M, n - 1 + R, 2), -1, dtype=np.int32)
    for i in range(1, n):
        cand = i - 1 - rng.integers(0, 3, size=M)
        cand = np.maximum(cand, 0)
        full = deg[rows, cand] >= 4
        cand = np.where(full, i - 1, cand)
        bonds[:, i - 1, 0] = cand
        bonds[:, i - 1, 1] = i
        deg[rows, cand] += 1
        deg[:, i] += 1
    nb = np.full(M, n - 1, dtype=np.int64)
    for r in range(R):
        need = n_rings > r
        done = ~need
        for _ in range(64):
            if done.all():
                break
            a = rng.integers(0, max(n - 4, 1), size=M)
            b = a + rng.integers(4, 8, size=M)
            ok = (~done) & (b < n)
            bb = np.minimum(b, n - 1)
            ok &= (deg[rows, a] < 4) & (deg[rows, bb] < 4)
            # no duplicate ring bond
            for rr in range(r):
                ok &= ~((bonds[:, n - 1 + rr, 0] == a) & (bonds[:, n - 1 + rr, 1] == bb))
            bonds[ok, n - 1 + r, 0] = a[ok]
            bonds[ok, n - 1 + r, 1] = bb[ok]
            deg[rows[ok], a[ok]] += 1
            deg[rows[ok], bb[ok]] += 1
            nb[ok] += 1
            done |= ok
    # compact: valid bonds first (stable), so bonds[:, :nb] are the molecule's bonds in order
    order = np.argsort(bonds[:, :, 0] < 0, axis=1, kind="stable")
    bonds = np.take_along_axis(bonds, order[:, :, None], axis=1)
    return bonds, nb, deg


def _features(rng, M, n, deg, in_ring):
    X = np.zeros((M, n, FEAT_DIM), dtype=np.float32)
    t = rng.choice(len(_TYPE_IDX), size=(M, n), p=_TYPE_P)
    mi, ai = np.meshgrid(np.arange(M), np.arange(n), indexing="ij")
    X[mi, ai, _TYPE_IDX[t]] = 1.0
    d = np.minimum(deg, 10)
    X[mi, ai, 43 + d] = 1.0
    h = np.clip(_VALENCE[t] - deg, 0, 4)
    X[mi, ai, 54 + np.minimum(h, 6)] = 1.0
    charged = rng.random((M, n)) < 0.01
    X[mi, ai, 61] = np.where(charged, rng.choice([-1.0, 1.0], size=(M, n)), 0.0)
    u = rng.random((M, n))
    hyb = np.where(u < 0.58, 2, np.where(u < 0.98, 1, 0))  # SP3, SP2, SP
    X[mi, ai, 63 + hyb] = 1.0
    X[mi, ai, 68] = ((hyb == 1) & in_ring & (rng.random((M, n)) < 0.8)).astype(np.float32)
    X[mi, ai, 69 + h] = 1.0
    return X


class SynthBatch:
    """Concatenated per-molecule arrays in molecule order (what mvml_gat.from_arrays takes)."""

    def __init__(self, num_nodes, num_edges, src_local, dst_local, feats):
        self.num_nodes = num_nodes
        self.num_edges = num_edges
        self.src_local = src_local
        self.dst_local = dst_local
        self.feats = feats

    @property
    def batch_size(self):
        return int(self.num_nodes.shape[0])

    def to_graph(self, group_size=None):
        from .batching import from_arrays
        return from_arrays(self.num_nodes, self.num_edges, self.src_local, self.dst_local,
                           self.feats, group_size=group_size)


def _assemble(sizes, per_size):
    """per_size[n] = (mol_ids, bonds (M,nbmax,2), nb (M,), feats (M,n,74), extra_edges list)."""
    B = len(sizes)
    num_nodes = sizes.astype(np.int64)
    nb_all = np.zeros(B, dtype=np.int64)
    for n, (ids, bonds, nb, feats) in per_size.items():
        nb_all[ids] = nb
    num_edges = 2 * nb_all + num_nodes
    eoff = np.concatenate([[0], np.cumsum(num_edges)])
    noff = np.concatenate([[0], np.cumsum(num_nodes)])
    E, N = int(eoff[-1]), int(noff[-1])
    src = np.empty(E, dtype=np.int32)
    dst = np.empty(E, dtype=np.int32)
    feats_all = np.empty((N, FEAT_DIM), dtype=np.float32)
    for n, (ids, bonds, nb, feats) in per_size.items():
        M, nbmax = bonds.shape[0], bonds.shape[1]
        j = np.arange(nbmax)
        valid = j[None, :] < nb[:, None]
        base = eoff[ids][:, None] + 2 * j[None, :]
        src[base[valid]] = bonds[:, :, 0][valid]
        dst[base[valid]] = bonds[:, :, 1][valid]
        src[base[valid] + 1] = bonds[:, :, 1][valid]
        dst[base[valid] + 1] = bonds[:, :, 0][valid]
        sl = eoff[ids][:, None] + 2 * nb[:, None] + np.arange(n)[None, :]
        src[sl] = np.arange(n, dtype=np.int32)[None, :]
        dst[sl] = np.arange(n, dtype=np.int32)[None, :]
        rowsel = noff[ids][:, None] + np.arange(n)[None, :]
        feats_all[rowsel.reshape(-1)] = feats.reshape(-1, FEAT_DIM)
    return SynthBatch(num_nodes, num_edges, src, dst, feats_all)


def _gen_sizes(rng, sizes, ring_sampler, hubs=None):
    per = {}
    for n in np.unique(sizes):
        ids = np.nonzero(sizes == n)[0]
        M = len(ids)
        rings = ring_sampler(M, n)
        bonds, nb, deg = _tree_and_rings(rng, M, int(n), rings)
        if hubs is not None:
            bonds, nb, deg = hubs(M, int(n), bonds, nb, deg)
        in_ring = np.zeros((M, int(n)), dtype=bool)
        feats = _features(rng, M, int(n), deg, in_ring | (rng.random((M, int(n))) < 0.3))
        per[int(n)] = (ids, bonds, nb, feats)
    return _assemble(sizes, per)


def config2(n_mols=65536, seed=0):
    """BASELINE config 2: 25 atoms, 27 bonds -> 79 edges per molecule incl. self-loops."""
    rng = np.random.default_rng(seed)
    sizes = np.full(n_mols, 25, dtype=np.int64)
    return _gen_sizes(rng, sizes, lambda M, n: np.full(M, 3, dtype=np.int64))


def kegg_like_sizes(rng, n_mols):
    """Log-normal atom counts with median 23, mean ~28, clipped to 11-80."""
    s = np.exp(rng.normal(np.log(23.0), 0.55, size=n_mols))
    return np.clip(np.rint(s), 11, 80).astype(np.int64)


def config3(n_mols=65536, seed=0):
    """BASELINE config 3 molecules (KEGG-like size distribution)."""
    rng = np.random.default_rng(seed)
    sizes = kegg_like_sizes(rng, n_mols)
    return _gen_sizes(rng, sizes,
                      lambda M, n: np.minimum(rng.poisson(2.4, size=M), max(n // 5, 1)))


class Config3Set:
    """The ONE global config-3 molecule set (BASELINE.json config 3: 1M molecules) as a cheap
    global plan — every molecule's atom count and requested ring closures, drawn up front — from
    which any contiguous range of molecules is generated on demand, identically whatever range
    asks for it: the structures / features of chunk c (molecules [c*chunk, (c+1)*chunk)) come
    from their own seeded stream, so a rank generating only its shard gets exactly the rows of
    the single-process set.

    group_costs(group_size): the expected edge count of each GraphNorm group (2 (n-1+rings) + n
    per molecule; a ring closure that fails its 64 attempts makes the real count lower), the
    cost mvml_gat.dist.shard_groups balances."""

    def __init__(self, n_mols=1_000_000, seed=0, chunk=65536):
        self.n_mols, self.seed, self.chunk = int(n_mols), int(seed), int(chunk)
        rng = np.random.default_rng([self.seed, 0x5EED])
        self.sizes = kegg_like_sizes(rng, self.n_mols)
        self.rings = np.minimum(rng.poisson(2.4, size=self.n_mols), np.maximum(self.sizes // 5, 1))

    def group_costs(self, group_size):
        e = 2 * (self.sizes - 1 + self.rings) + self.sizes
        G = -(-self.n_mols // group_size)
        pad = np.zeros(G * group_size, dtype=np.int64)
        pad[:self.n_mols] = e
        return pad.reshape(G, group_size).sum(1)

    def _chunk(self, c):
        lo, hi = c * self.chunk, min(self.n_mols, (c + 1) * self.chunk)
        sizes, rings = self.sizes[lo:hi], self.rings[lo:hi]
        rng = np.random.default_rng([self.seed, c])
        return _gen_sizes(rng, sizes, lambda M, n: rings[sizes == n])

    def molecules(self, lo, hi):
        """SynthBatch of molecules [lo, hi) of the global set."""
        lo, hi = max(0, int(lo)), min(self.n_mols, int(hi))
        parts = []
        for c in range(lo // self.chunk, -(-hi // self.chunk)):
            sb = self._chunk(c)
            c0 = c * self.chunk
            parts.append(slice_batch(sb, max(lo, c0) - c0, min(hi, c0 + sb.batch_size) - c0))
        return concat_batches(parts)


def slice_batch(sb, lo, hi):
    """Molecules [lo, hi) of a SynthBatch."""
    e0, e1 = int(sb.num_edges[:lo].sum()), int(sb.num_edges[:hi].sum())
    n0, n1 = int(sb.num_nodes[:lo].sum()), int(sb.num_nodes[:hi].sum())
    return SynthBatch(sb.num_nodes[lo:hi], sb.num_edges[lo:hi], sb.src_local[e0:e1],
                      sb.dst_local[e0:e1], sb.feats[n0:n1])


def concat_batches(parts):
    if len(parts) == 1:
        return parts[0]
    return SynthBatch(np.concatenate([p.num_nodes for p in parts]),
                      np.concatenate([p.num_edges for p in parts]),
                      np.concatenate([p.src_local for p in parts]),
                      np.concatenate([p.dst_local for p in parts]),
                      np.concatenate([p.feats for p in parts]))


def config5(n_mols=4096, seed=1):
    """BASELINE config 5: 150-400 atoms plus 1-4 hubs with 32-128 extra bonds (non-chemical)."""
    rng = np.random.default_rng(seed)
    sizes = rng.integers(150, 401, size=n_mols).astype(np.int64)

    def hubs(M, n, bonds, nb, deg):
        k = rng.integers(1, 5, size=M)
        m = rng.integers(32, 129, size=(M, 4))
        extra_max = int((m * (np.arange(4)[None, :] < k[:, None])).sum(1).max())
        out = np.full((M, bonds.shape[1] + extra_max, 2), -1, dtype=np.int32)
        out[:, :bonds.shape[1]] = bonds
        nb2 = nb.copy()
        for i in range(M):
            pos = int(nb[i])
            # compact the ring slots that failed (-1) out of the way
            row = bonds[i][bonds[i, :, 0] >= 0]
            out[i, :len(row)] = row
            pos = len(row)
            hub_ids = rng.choice(n, size=int(k[i]), replace=False)
            for j, h in enumerate(hub_ids):
                partners = rng.choice(np.setdiff1d(np.arange(n), [h]), size=int(m[i, j]), replace=False)
                out[i, pos:pos + len(partners), 0] = h
                out[i, pos:pos + len(partners), 1] = partners
                deg[i, h] += len(partners)
                deg[i, partners] += 1
                pos += len(partners)
            nb2[i] = pos
        return out, nb2, deg

    return _gen_sizes(rng, sizes, lambda M, n: rng.poisson(n / 10.0, size=M), hubs=hubs)
