"""SMILES BiLSTM view (RNNModule, model.py:98-135) throughput on the KEGG test split's SMILES
(tests/golden/kegg_test_split.csv, 420 molecules, reference batches of 64, MVP sizes E=128,
H=384, 2 layers, out 384): fwd+bwd molecules/s with HIP events, plus the float32 CPU restatement
(oracle/smiles_ref.py, torch nn.LSTM on the host) for a baseline.

    python tools/smiles_bench.py [--steps 5] [--cpu]
"""
import argparse
import csv
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mvml-mpi_amd")]
from mvml_gat.smiles import RNNModule, collate_smiles, tokens_struct  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args()
    with open(os.path.join(ROOT, "tests", "golden", "kegg_test_split.csv")) as f:
        smiles = [r["smiles"] for r in csv.DictReader(f)]
    vocab = tokens_struct()
    batches = [collate_smiles(smiles[i:i + 64], vocab) for i in range(0, len(smiles), 64)]
    torch.manual_seed(0)
    mod = RNNModule(vocab, 128, 384, 2, 384, 0.2).cuda().train()
    dev_b = [{"smiles": b["smiles"].cuda(), "seq_len": b["seq_len"]} for b in batches]
    up = torch.randn(64, 384, device="cuda")

    def epoch():
        for b in dev_b:
            z = mod(b)
            (z * up[:z.shape[0]]).sum().backward()

    epoch()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    s.record()
    for _ in range(a.steps):
        epoch()
    e.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    n = a.steps * len(smiles)
    res = {"metric": "SMILES BiLSTM view fwd+bwd molecules/s (KEGG test split, batch 64)",
           "value": round(n / (s.elapsed_time(e) / 1e3), 1), "unit": "molecules/s",
           "ms_per_epoch": round(s.elapsed_time(e) / a.steps, 3), "wall_s": round(wall, 3),
           "max_len": max(max(b["seq_len"]) for b in batches),
           "mean_len": round(sum(sum(b["seq_len"]) for b in batches) / len(smiles), 1)}
    if a.cpu:
        from oracle.smiles_ref import RNNModuleRef
        torch.set_num_threads(min(16, os.cpu_count()))
        ref = RNNModuleRef(39, 128, 384, 2, 384, 0.2).train()
        t0 = time.perf_counter()
        for b in batches:
            z = ref(b)
            z.sum().backward()
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(len(smiles) / dt, 1), "unit": "molecules/s",
                               "cores": torch.get_num_threads(), "kind": "port",
                               "sample": "one pass over the 420 KEGG test SMILES, fp32 torch nn.LSTM on CPU"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
