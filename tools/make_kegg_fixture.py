"""Write tests/golden/kegg_test_split.csv: the KEGG test split.

Data, not code: the rows of /root/reference/data/kegg_dataset.csv (smiles, label) whose
indices are listed on line 3 of /root/reference/data/data_index.txt (main.py:68-77 reads it
the same way: line 1 train, line 2 validate, line 3 test), kept in the listed order, so the
GPU box (which has no /root/reference) can run config 1.  Run once here:
    python tools/make_kegg_fixture.py
"""
import ast
import csv
import os

REF = "/root/reference/data"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "kegg_test_split.csv")


def main():
    rows = list(csv.DictReader(open(os.path.join(REF, "kegg_dataset.csv"))))
    lines = [l for l in open(os.path.join(REF, "data_index.txt")).read().splitlines() if l.strip()]
    test_idx = ast.literal_eval(lines[2])
    with open(OUT, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["index", "smiles", "label"])
        for i in test_idx:
            w.writerow([i, rows[i]["smiles"], rows[i]["label"]])
    print(f"wrote {len(test_idx)} rows to {OUT}")


if __name__ == "__main__":
    main()
