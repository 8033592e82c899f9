"""BASELINE config 1: the KEGG test split (420 molecules, data_index.txt line 3
order, batches of 64 = config.py:21, eval mode) through the HIP graph view + fusion head,
compared with the float64 CPU restatement on identical graphs and weights.

Bars: logits within 1e-5 norm-wise relative error (TOL); predicted labels
(sigmoid(logit) >= 0.5, utils.py:127-130) identical; the per-batch-mean test metrics of
main.py:100-110 (acc of utils.py:109-123, sample-averaged precision/recall/F1) identical.

Inputs: graphs from mvml_gat.featurize (RDKit agreement unpinned, see tests/test_featurize.py);
seeded random weights (no trained checkpoint exists here).  The SMILES-BiLSTM and fingerprint
views are out of scope: their two fusion tokens are fixed seeded tensors,
identical on both sides."""
import os

import numpy as np
import pytest
import torch

from _util import randomize_
from conftest import rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 1e-5
HERE = os.path.dirname(os.path.abspath(__file__))


def _metrics(y, z):
    from sklearn.metrics import f1_score, precision_score, recall_score
    pred = (1.0 / (1.0 + np.exp(-z)) >= 0.5).astype(int)
    y = y.astype(int)
    acc = np.mean([np.logical_and(a, b).sum() / np.logical_or(a, b).sum() for a, b in zip(y, pred)])
    return pred, [acc, precision_score(y, pred, average="samples", zero_division=0),
                  recall_score(y, pred, average="samples", zero_division=0),
                  f1_score(y, pred, average="samples", zero_division=0)]


def test_kegg_config1_labels_identical():
    from mvml_gat import GNNModule, MVFusion
    from mvml_gat.featurize import MolDataSet, collate
    from oracle.fusion_ref import MVFusionRef
    from oracle.gnn_ref import GNNModuleRef
    from oracle.graph_ref import batch_ref

    ds = MolDataSet(os.path.join(HERE, "golden", "kegg_test_split.csv"))
    torch.manual_seed(0)
    gnn = GNNModule(74, [192, 384], 0.5, 6, 3)
    randomize_(gnn, 0)
    fus = MVFusion(384, 12, 11, 0.5)      # num_heads = config.py:17 --head default 12
    gnn_ref = GNNModuleRef(74, [192, 384], 0.5, 6, 3).double().eval()
    gnn_ref.load_state_dict({k: v.double() for k, v in gnn.state_dict().items()})
    fus_ref = MVFusionRef(384, 12, 11, 0.5).double().eval()
    fus_ref.load_state_dict({k: v.double() for k, v in fus.state_dict().items()})
    gnn, fus = gnn.to(DEV).eval(), fus.to(DEV).eval()
    g = torch.Generator().manual_seed(11)
    smiles_x = torch.randn(len(ds), 384, generator=g, dtype=torch.float64)
    fp_x = torch.randn(len(ds), 384, generator=g, dtype=torch.float64)

    res_d, res_r, worst, margin = [], [], 0.0, np.inf
    with torch.no_grad():
        for s in range(0, len(ds), 64):
            idx = list(range(s, min(s + 64, len(ds))))
            samples = [ds[i] for i in idx]
            bg, y = collate(samples)
            bgd = bg.to(DEV)
            zd = fus(smiles_x[idx].float().to(DEV), gnn(bgd, bgd.ndata["h"].to(DEV)),
                     fp_x[idx].float().to(DEV)).double().cpu()
            gr = [m for m, _ in samples]
            gd = batch_ref(np.array([m.num_nodes() for m in gr]), np.concatenate([m.src for m in gr]),
                           np.concatenate([m.dst for m in gr]), np.array([m.num_edges() for m in gr]))
            x = torch.cat([m.ndata["h"] for m in gr]).double()
            zr = fus_ref(smiles_x[idx], gnn_ref(gd, x), fp_x[idx])
            worst = max(worst, rel_err(zd, zr))
            margin = min(margin, zr.abs().min().item())
            pd_, md = _metrics(y.numpy(), zd.numpy())
            pr_, mr = _metrics(y.numpy(), zr.numpy())
            assert np.array_equal(pd_, pr_), f"labels differ in batch {s // 64}"
            res_d.append(md)
            res_r.append(mr)
    print(f"config1: logits rel_err {worst:.2e}, min |logit| {margin:.3e}, "
          f"test metrics (acc, prec, rec, f1) {np.mean(res_d, 0)}")
    assert worst < TOL
    assert np.array_equal(np.mean(res_d, 0), np.mean(res_r, 0))


def test_kegg_config1_whole_mvp_real_fingerprints():
    """The whole MVP model in eval mode (model.py:13-75) on the 420 test-split molecules with the
    three real view inputs: SMILES tokens (utils.py:55-96 restated), graphs (featurize) and the
    2,513-value fingerprints of dataset.py:37-45 (mvml_gat.fingerprints; RDKit agreement
    unpinned): logits within 1e-5 of the float64 oracle and predicted labels identical."""
    from mvml_gat.featurize import MolDataSet, collate
    from mvml_gat.fingerprints import FP_SIZE, fingerprints
    from mvml_gat.mvp import MVP
    from mvml_gat.smiles import collate_smiles, tokens_struct
    from oracle.fusion_ref import MVPRef
    from oracle.graph_ref import batch_ref

    ds = MolDataSet(os.path.join(HERE, "golden", "kegg_test_split.csv"))
    fps = torch.as_tensor(fingerprints(ds.smiles))
    assert fps.shape == (len(ds), FP_SIZE) and fps[:, :167].sum() > 0 and fps[:, 1489:].sum() > 0
    torch.manual_seed(0)
    mod = MVP(11, 74, [192, 384], 6, 3, 128, 384, 2, 512, 12, 0.5)
    randomize_(mod.gnn, 0)
    ref = MVPRef().double().eval()
    ref.load_state_dict({k: v.double() for k, v in mod.state_dict().items()})
    mod = mod.to(DEV).eval()
    tok = tokens_struct()
    worst = 0.0
    with torch.no_grad():
        for s in range(0, len(ds), 64):
            idx = list(range(s, min(s + 64, len(ds))))
            samples = [ds[i] for i in idx]
            bg, y = collate(samples)
            sm = collate_smiles([ds.smiles[i] for i in idx], tok)
            g = bg.to(DEV)
            zd = mod({"smiles": sm["smiles"].to(DEV), "seq_len": sm["seq_len"]}, g, g.ndata["h"].to(DEV),
                     fps[idx].to(DEV)).double().cpu()
            gr = [m for m, _ in samples]
            gd = batch_ref(np.array([m.num_nodes() for m in gr]), np.concatenate([m.src for m in gr]),
                           np.concatenate([m.dst for m in gr]), np.array([m.num_edges() for m in gr]))
            x = torch.cat([m.ndata["h"] for m in gr]).double()
            zr = ref(sm, gd, x, fps[idx].double())
            worst = max(worst, rel_err(zd, zr))
            pd_, _ = _metrics(y.numpy(), zd.numpy())
            pr_, _ = _metrics(y.numpy(), zr.numpy())
            assert np.array_equal(pd_, pr_), f"labels differ in batch {s // 64}"
    print(f"config1 whole MVP: logits rel_err {worst:.2e}")
    assert worst < TOL
