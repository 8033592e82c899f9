"""SMILES -> graph featurisation: mvml_gat.featurize against
hand-derived RDKit/dgllife known answers, and the KEGG test split (config 1) fixture.

Agreement with RDKit itself is unpinned (RDKit is absent here); every expected tuple below is
what RDKit 2022.09 + dgllife 0.3.0 CanonicalAtomFeaturizer give for that molecule, derived by
hand from their documented rules: (symbol, aromatic, degree, implicit valence, hybridisation,
total H, formal charge)."""
import os

import numpy as np
import pytest

from mvml_gat import featurize as fz

HERE = os.path.dirname(os.path.abspath(__file__))
KEGG = os.path.join(HERE, "golden", "kegg_test_split.csv")
SP, SP2, SP3 = fz.HYB_SP, fz.HYB_SP2, fz.HYB_SP3


def _atoms(smi):
    m = fz.mol_from_smiles(smi)
    return [(m.sym[i], bool(m.arom[i]), m.degree(i), m.implicit_h[i], m.hyb[i], m.total_h(i),
             m.charge[i]) for i in range(m.num_atoms)]


KAT = {
    # benzene: aromatic CH, sp2
    "c1ccccc1": [("C", True, 2, 1, SP2, 1, 0)] * 6,
    # kekule input is perceived aromatic
    "C1=CC=CC=C1": [("C", True, 2, 1, SP2, 1, 0)] * 6,
    "CCO": [("C", False, 1, 3, SP3, 3, 0), ("C", False, 2, 2, SP3, 2, 0),
            ("O", False, 1, 1, SP3, 1, 0)],
    # acid OH is conjugated with C=O -> sp2 (RDKit "second O in O=CO")
    "CC(=O)O": [("C", False, 1, 3, SP3, 3, 0), ("C", False, 3, 0, SP2, 0, 0),
                ("O", False, 1, 0, SP2, 0, 0), ("O", False, 1, 1, SP2, 1, 0)],
    # pyrrole: bracket [nH] -> implicit valence 0, one explicit H
    "c1cc[nH]c1": [("C", True, 2, 1, SP2, 1, 0)] * 3 + [("N", True, 2, 0, SP2, 1, 0),
                                                       ("C", True, 2, 1, SP2, 1, 0)],
    "CC#N": [("C", False, 1, 3, SP3, 3, 0), ("C", False, 2, 0, SP, 0, 0),
             ("N", False, 1, 0, SP, 0, 0)],
    "C[N+](=O)[O-]": [("C", False, 1, 3, SP3, 3, 0), ("N", False, 3, 0, SP2, 0, 1),
                      ("O", False, 1, 0, SP2, 0, 0), ("O", False, 1, 0, SP2, 0, -1)],
    "OP(=O)(O)O": [("O", False, 1, 1, SP3, 1, 0), ("P", False, 4, 0, SP3, 0, 0),
                   ("O", False, 1, 0, SP2, 0, 0), ("O", False, 1, 1, SP3, 1, 0),
                   ("O", False, 1, 1, SP3, 1, 0)],
    # furan O: two lone pairs, one in the pi system -> sp2
    "o1cccc1": [("O", True, 2, 0, SP2, 0, 0)] + [("C", True, 2, 1, SP2, 1, 0)] * 4,
    # aniline N conjugated with the ring -> sp2
    "Nc1ccccc1": [("N", False, 1, 2, SP2, 2, 0), ("C", True, 3, 0, SP2, 0, 0)] +
                 [("C", True, 2, 1, SP2, 1, 0)] * 5,
    # cyclopentadiene (CH2 is sp3) and p-benzoquinone are not aromatic
    "C1=CCC=C1": [("C", False, 2, 1, SP2, 1, 0)] * 2 + [("C", False, 2, 2, SP3, 2, 0)] +
                 [("C", False, 2, 1, SP2, 1, 0)] * 2,
    "C1CCCCC1": [("C", False, 2, 2, SP3, 2, 0)] * 6,
    # pyrylium
    "c1cc[o+]cc1": [("C", True, 2, 1, SP2, 1, 0)] * 3 + [("O", True, 2, 0, SP2, 0, 1)] +
                   [("C", True, 2, 1, SP2, 1, 0)] * 2,
}


@pytest.mark.parametrize("smi", sorted(KAT))
def test_known_answers(smi):
    assert _atoms(smi) == KAT[smi]


@pytest.mark.parametrize("smi,n_arom", [
    ("c1ccc2ccccc2c1", 10),                      # naphthalene
    ("c1ccc2cccc2cc1", 10),                      # azulene (5+7 fused, 10 pi electrons)
    ("Cn1cnc2c1c(=O)n(C)c(=O)n2C", 9),           # caffeine: both rings (C=O carbons vacant)
    ("O=C1NC(=O)C=CN1", 6),                      # kekule uracil perceived aromatic
    ("O=C1C=CC(=O)C=C1", 0),                     # p-benzoquinone
    ("C=C1C=CC=C1", 0),                          # fulvene
    ("c1ccc2c(c1)[nH]c1ccccc12", 13),            # carbazole
    ("Nc1ncnc2[nH]cnc12", 9),                    # adenine
])
def test_aromaticity(smi, n_arom):
    assert sum(fz.mol_from_smiles(smi).arom) == n_arom


def test_feature_layout_and_bigraph():
    """74-d layout of CanonicalAtomFeaturizer and mol_to_bigraph edge order (a1)."""
    g = fz.smiles_to_bigraph("CC(=O)[O-]", canonical_atom_order=False)
    f = g.ndata["h"].numpy()
    assert f.shape == (4, fz.FEAT_SIZE)
    assert f[0, 0] == 1 and f[2, 2] == 1                  # C, O one-hot
    assert f[1, 43 + 3] == 1 and f[0, 43 + 1] == 1        # degree block
    assert f[0, 54 + 3] == 1 and f[1, 54 + 0] == 1        # implicit valence block
    assert f[3, 61] == -1                                 # formal charge
    assert f[0, 63 + SP3] == 1 and f[1, 63 + SP2] == 1    # hybridisation
    assert f[0, 69 + 3] == 1                              # total H block
    src, dst = g.edges()
    assert list(src) == [0, 1, 1, 2, 1, 3, 0, 1, 2, 3]
    assert list(dst) == [1, 0, 2, 1, 3, 1, 0, 1, 2, 3]


def test_unknown_element_and_dummy():
    f = fz.atom_features(fz.mol_from_smiles("[*]C[Mo]"))
    assert f[0, :43].sum() == 0 and f[2, :43].sum() == 0  # '*' and Mo: not in the 43 types
    assert f[1, 0] == 1


def test_kegg_test_split_fixture():
    """Config 1 input: all 420 test-split SMILES featurise; feature blocks are one-hot."""
    ds = fz.MolDataSet(KEGG)
    assert len(ds) == 420
    n_atoms = 0
    for i in range(len(ds)):
        g, y = ds[i]
        f = g.ndata["h"].numpy()
        n_atoms += g.num_nodes()
        assert f.shape[1] == 74 and y.sum() >= 1
        assert np.all(f[:, 43:54].sum(1) == 1)            # degree <= 10
        assert np.all(f[:, 69:74].sum(1) <= 1)
        src, dst = g.edges()
        indeg = np.bincount(dst, minlength=g.num_nodes())
        assert indeg.min() >= 1                           # self-loops: no zero in-degree
        nb = (g.num_edges() - g.num_nodes()) // 2
        assert np.all(src[0:2 * nb:2] == dst[1:2 * nb:2])  # rev(e) = e ^ 1
    assert 10_000 < n_atoms < 14_000                      # ~11.7k atoms


def test_canonical_ranks_ethanol_and_dgllife_renumbering():
    """CCO: base invariants (degree, Z, isotope, total H, charge) already separate the atoms —
    C0 (1, 6, 0, 3, 0) < O2 (1, 8, 0, 1, 0) < C1 (2, 6, 0, 2, 0) — so the ranks are [0, 2, 1].
    dgllife passes the rank list to RenumberAtoms as newOrder (mol_to_graph,
    canonical_atom_order=True): new atom k is old atom rank[k], bonds keep order and
    orientation: bond (0, 1) -> (0, 2), bond (1, 2) -> (2, 1)."""
    m = fz.mol_from_smiles("CCO")
    assert fz.canonical_ranks(m) == [0, 2, 1]
    g = fz.smiles_to_bigraph("CCO", add_self_loop=False)
    src, dst = g.edges()
    assert list(src) == [0, 2, 2, 1] and list(dst) == [2, 0, 1, 2]
    f = g.ndata["h"].numpy()
    assert f[0, 0] == 1 and f[1, 2] == 1 and f[2, 0] == 1           # C, O, C
    assert f[0, 69 + 3] == 1 and f[2, 69 + 2] == 1                 # CH3 first, CH2 last


@pytest.mark.parametrize("a,b", [
    ("OCC(N)C", "CC(N)CO"),
    ("CC(=O)Oc1ccccc1C(=O)O", "OC(=O)c1ccccc1OC(C)=O"),          # aspirin, two writings
])
def test_canonical_ranks_are_writing_independent(a, b):
    """The ranks themselves are canonical: an atom's rank does not depend on how the SMILES was
    written (matched through each writing's rank-sorted feature rows and neighbour ranks)."""
    def signature(smi):
        m = fz.mol_from_smiles(smi)
        r = fz.canonical_ranks(m)
        f = fz.atom_features(m)
        by_rank = sorted(range(m.num_atoms), key=lambda i: r[i])
        return [(tuple(f[i]), tuple(sorted(r[j] for (j, _) in m.nbrs(i)))) for i in by_rank]
    assert signature(a) == signature(b)


@pytest.mark.parametrize("smi", ["c1ccccc1", "C1CCCCC1", "CC(C)(C)C", "OC(=O)CC(O)(CC(=O)O)C(=O)O"])
def test_canonical_ranks_symmetric(smi):
    """Symmetric molecules: ties broken to a permutation of 0..n-1; the ranked graph is the
    molecule (same degree sequence, bigraph invariants kept)."""
    m = fz.mol_from_smiles(smi)
    r = fz.canonical_ranks(m)
    assert sorted(r) == list(range(m.num_atoms))
    g = fz.smiles_to_bigraph(smi)
    src, dst = g.edges()
    nb = (g.num_edges() - g.num_nodes()) // 2
    assert np.all(src[0:2 * nb:2] == dst[1:2 * nb:2])
    deg = np.bincount(dst[:2 * nb], minlength=g.num_nodes())
    assert sorted(deg.tolist()) == sorted(m.degree(i) for i in range(m.num_atoms))
