"""Known answers for the restated fingerprints of the reference's fingerprint view (dataset.py:37-45;
mvml_gat/fingerprints.py).  RDKit cannot run here, so agreement with it is unpinned; these pin
the restatement:

* MACCS: RDKit's own doctest vectors for CNO and CCC (MACCSkeys.py; the reference copies them
  into pubchemfp.py:788-793) and hand-derived ring / count keys;
* PubChem: the ring-count block (pubchemfp.py:815-1511) on benzene, pyridine and cyclohexane
  worked by hand, the quirk that saturated rings count in every func_2-func_4 class, and
  element / H-count keys of the substructure table on ethane;
* Morgan: the number of distinct environments of symmetric molecules (methane 1, ethane 2,
  benzene 3 bits) and invariance to atom order;
* ErG: phenol's two property-point pairs at reduced-graph distance 1 with the 0.3 fuzz.
"""
import numpy as np
import pytest

from mvml_gat import featurize as fz
from mvml_gat import fingerprints as fp


def _on(bits):
    return tuple(int(i) for i in np.nonzero(bits)[0])


@pytest.mark.parametrize("smi,want", [
    ("CNO", (24, 68, 69, 71, 93, 94, 102, 124, 131, 139, 151, 158, 160, 161, 164)),
    ("CCC", (74, 114, 149, 155, 160)),
])
def test_maccs_rdkit_doctest_vectors(smi, want):
    assert _on(fp.maccs_keys(fz.mol_from_smiles(smi))) == want


def test_maccs_rings_and_counts():
    b = fp.maccs_keys(fz.mol_from_smiles("c1ccccc1-c1ccccc1"))  # biphenyl
    assert b[125] == 1 and b[162] == 1 and b[163] == 1 and b[145] == 1 and b[165] == 1
    b = fp.maccs_keys(fz.mol_from_smiles("c1ccccc1"))
    assert b[125] == 0 and b[145] == 0 and b[163] == 1
    b = fp.maccs_keys(fz.mol_from_smiles("C1CC1.C"))  # 3-ring + a second fragment
    assert b[22] == 1 and b[166] == 1 and b[162] == 0
    b = fp.maccs_keys(fz.mol_from_smiles("OCC(O)CO"))  # glycerol: O > 2, O > 1, O > 0
    assert b[164] == b[159] == b[146] == 1 and b[140] == 0


def _pc_ring(smi):
    return set(_on(fp.pubchem_fp(fz.mol_from_smiles(smi))[115:263]))


def test_pubchem_ring_counts():
    # columns: 0 any ring, 1 sat./aromatic C-only, 2 sat./aromatic N, 3 sat./aromatic hetero,
    # 4-6 unsaturated non-aromatic C / N / hetero; a 6-ring's first threshold is slot 9 (63+c)
    assert _pc_ring("c1ccccc1") == {63, 64, 140}
    assert _pc_ring("c1ccncc1") == {63, 65, 66, 140, 141}
    assert _pc_ring("C1CCCCC1") == {63, 64, 65, 66}      # saturated: every func_2-func_4 class
    assert _pc_ring("C1=CCCCC1") == {63, 67}             # unsaturated non-aromatic carbon ring
    assert _pc_ring("c1ccccc1-c1ccccc1") == {63, 64, 70, 71, 140, 142}  # two: second threshold


def test_pubchem_substructure_keys():
    b = fp.pubchem_fp(fz.mol_from_smiles("CC"))         # 6 H atoms, 2 C
    on = set(_on(b))
    assert 0 in on and 1 not in on                      # [H] > 3, not > 7
    assert 9 in on and 10 not in on                     # [C] > 1, not > 3
    assert b.shape == (881,)
    b = fp.pubchem_fp(fz.mol_from_smiles("[Li]C"))
    assert 4 in set(_on(b))                             # [Li] present


def test_morgan_environments():
    n = lambda s: int(fp.morgan_fp(fz.mol_from_smiles(s)).sum())
    assert n("C") == 1
    assert n("CC") == 2
    assert n("c1ccccc1") == 3
    a = fp.morgan_fp(fz.mol_from_smiles("OCC(N)C"))
    b = fp.morgan_fp(fz.mol_from_smiles("CC(N)CO"))     # same molecule, other atom order
    assert np.array_equal(a, b)


def test_erg_phenol():
    e = fp.erg_fp(fz.mol_from_smiles("Oc1ccccc1"))
    assert e.shape == (441,)
    # ring node {aromatic} and the OH node {donor, acceptor} at distance 1 (bin 0, fuzz into bin 1)
    for a in (0, 1):
        base = fp._pair_index(a, 5) * 21
        assert e[base] == pytest.approx(1.0) and e[base + 1] == pytest.approx(0.3)
    assert e.sum() == pytest.approx(2.6)
    assert fp.erg_fp(fz.mol_from_smiles("c1ccccc1")).sum() == 0


def test_fingerprint_layout():
    v = fp.fingerprints(["CNO", "c1ccncc1"])
    assert v.shape == (2, 2513) and v.dtype == np.float32
    assert np.array_equal(v[0, :167], fp.maccs_keys(fz.mol_from_smiles("CNO")))


def test_kegg_pool_matches_fingerprints():
    """The packed pool bench.py's MVP workload reads holds exactly what fingerprints() computes
    for those molecules (a sample of rows recomputed here)."""
    import csv
    import os
    from mvml_gat.fingerprints import FP_SIZE, fingerprints, kegg_pool
    pool = kegg_pool()
    assert pool.shape == (420, FP_SIZE) and pool.dtype == np.float32
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "golden", "kegg_test_split.csv"), newline="") as f:
        smiles = [r["smiles"] for r in csv.DictReader(f)]
    idx = [0, 1, 57, 200, 419]
    assert np.array_equal(pool[idx], fingerprints([smiles[i] for i in idx]))
