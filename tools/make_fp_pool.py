"""Regenerate mvml-mpi_amd/mvml_gat/data/kegg_fp_pool.npz: the 2,513-value fingerprint view
(dataset.py:37-45: MACCS 167 | ErG 441 | PubChem 881 | Morgan r2 1024, restated in
mvml_gat/fingerprints.py, RDKit agreement unpinned) of the 420 KEGG test-split molecules of
tests/golden/kegg_test_split.csv, bit-packed.  bench.py's MVP workload cycles these real bit
vectors over its synthetic molecules (computing them per molecule costs ~70 ms of host time, so
the bench reads this pool instead).  ErG's fuzzy values are not bits: they are kept as float32.

    python tools/make_fp_pool.py
"""
import csv
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mvml-mpi_amd")]
from mvml_gat.fingerprints import ERG_BITS, FP_SIZE, MACCS_BITS, fingerprints  # noqa: E402

OUT = os.path.join(ROOT, "mvml-mpi_amd", "mvml_gat", "data", "kegg_fp_pool.npz")


def main():
    with open(os.path.join(ROOT, "tests", "golden", "kegg_test_split.csv"), newline="") as f:
        smiles = [r["smiles"] for r in csv.DictReader(f)]
    fp = np.asarray(fingerprints(smiles), dtype=np.float32)
    assert fp.shape == (len(smiles), FP_SIZE)
    erg = fp[:, MACCS_BITS:MACCS_BITS + ERG_BITS]
    bits = np.concatenate([fp[:, :MACCS_BITS], fp[:, MACCS_BITS + ERG_BITS:]], axis=1)
    assert set(np.unique(bits).tolist()) <= {0.0, 1.0}
    np.savez_compressed(OUT, bits=np.packbits(bits.astype(np.uint8), axis=1), nbits=bits.shape[1],
                        erg=erg)
    print(f"wrote {len(smiles)} fingerprints to {OUT}: {bits.mean():.3f} of the bits set")


if __name__ == "__main__":
    main()
