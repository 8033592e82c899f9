"""Regenerate mvml-mpi_amd/mvml_gat/data/pubchem_smarts.json: the 733 PubChem substructure keys
(SMARTS, count threshold) of the reference's fingerprint view — the public PubChem fingerprint
specification (ftp.ncbi.nlm.nih.gov/pubchem/specifications/pubchem_fingerprints.txt) as the
reference carries it in /root/reference/pubchemfp.py:28-733 (`smartsPatts`, keys 1-115 and
264-881 of the 881-bit fingerprint).  Only the table is taken, as data (parsed with ast, never
imported or executed); the ring-count bits 116-263 and the bit assembly are restated in
mvml_gat/fingerprints.py.  Run in this container (the GPU box has no /root/reference):

    python tools/make_pubchem_table.py
"""
import ast
import json
import os

SRC = "/root/reference/pubchemfp.py"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mvml-mpi_amd",
                   "mvml_gat", "data", "pubchem_smarts.json")


def main():
    text = open(SRC).read()
    i = text.index("smartsPatts = {")
    j = text.index("PubchemKeys = None")
    table = ast.literal_eval(text[i + len("smartsPatts = "):j].strip())
    keys = sorted(table)
    assert keys == list(range(1, 734)), "expected keys 1..733"
    rows = [[table[k][0], int(table[k][1])] for k in keys]
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    src = ("PubChem substructure fingerprint keys as listed in the reference's pubchemfp.py:28-733 "
           "(public PubChem specification); [SMARTS, count]: bit set when the number of unique "
           "matches exceeds count (0: any match)")
    with open(OUT, "w") as f:
        f.write('{"source": %s,\n "keys": [\n' % json.dumps(src))
        f.write(",\n".join("  " + json.dumps(r) for r in rows))
        f.write("\n]}\n")
    json.load(open(OUT))
    print(f"wrote {len(rows)} keys to {OUT}")


if __name__ == "__main__":
    main()
