"""The whole MVP model (model.py:13-75) on the HIP path — BASELINE config 4's training step
(main.py:24-36): RNNModule + GNNModule + FPNModule (fp_2_dim = 512, config.py:16) + fusion head
+ BCEWithLogits + Adam (lr 1e-3, wd 1e-4, main.py:88) — against the composed float64 oracle
(oracle/fusion_ref.py MVPRef) on one 64-molecule KEGG batch (the first test-split batch,
data_index.txt order, featurised by mvml_gat.featurize; fingerprints are seeded 0/1 bits since
RDKit is absent here).

Bars: logits / loss within 1e-5 of float64; every parameter gradient within 1e-5 or 4x the
fp32 oracle's own error where conditioning makes fp32 lose that much (see
test_gpu_parity_configs.py); after one Adam step the parameters within 1e-5.  The ReLU-fed
fusion biases get the +20 margin of test_gpu_fusion.py (a pre-activation within fp32 rounding
of 0 picks a subgradient), and the GAT LeakyReLU sides come from the product as in
test_gpu_parity_configs.py."""
import os

import numpy as np
import pytest
import torch

from _util import randomize_
from conftest import rel_err
from test_gpu_parity_configs import _branches, _capture

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 1e-5
HERE = os.path.dirname(os.path.abspath(__file__))


def _kegg_batch(n=64, seed=0):
    from mvml_gat.featurize import MolDataSet, collate
    from mvml_gat.smiles import collate_smiles, tokens_struct
    from oracle.graph_ref import batch_ref
    ds = MolDataSet(os.path.join(HERE, "golden", "kegg_test_split.csv"))
    samples = [ds[i] for i in range(n)]
    bg, y = collate(samples)
    gr = [m for m, _ in samples]
    gd = batch_ref(np.array([m.num_nodes() for m in gr]), np.concatenate([m.src for m in gr]),
                   np.concatenate([m.dst for m in gr]), np.array([m.num_edges() for m in gr]))
    x = torch.cat([m.ndata["h"] for m in gr]).double()
    smiles = collate_smiles(ds.smiles[:n], tokens_struct())
    fp = (torch.rand(n, 2513, generator=torch.Generator().manual_seed(seed)) < 0.1).double()
    return bg, gd, x, smiles, fp, y.double()


def _models(seed=0):
    from mvml_gat.mvp import MVP
    from oracle.fusion_ref import MVPRef
    torch.manual_seed(seed)
    mod = MVP(11, 74, [192, 384], 6, 3, 128, 384, 2, 512, 12, 0.5)
    randomize_(mod.gnn, seed)
    with torch.no_grad():
        mod.norm_layer_module.weight.uniform_(0.5, 1.5)
        mod.conv[0].bias += 20.0
        mod.mlp[0].bias += 20.0
    ref64 = MVPRef().double().eval()
    ref64.load_state_dict({k: v.double() for k, v in mod.state_dict().items()})
    ref32 = MVPRef().eval()
    ref32.load_state_dict(mod.state_dict())
    return mod.to(DEV).eval(), ref64, ref32


def test_mvp_train_step_parity():
    from mvml_gat import bce_with_logits
    from oracle.fusion_ref import bce_logits_ref
    bg, gd, x, smiles, fp, y = _kegg_batch()
    mod, ref64, ref32 = _models()
    g = bg.to(DEV)
    sm_d = {"smiles": smiles["smiles"].to(DEV), "seq_len": smiles["seq_len"]}
    opt = torch.optim.Adam(mod.parameters(), lr=1e-3, weight_decay=1e-4)
    opt.zero_grad()
    z_d, elrs = _capture(lambda: mod(sm_d, g, g.ndata["h"].to(DEV), fp.float().to(DEV)))
    br = _branches(gd, elrs)
    loss_d = bce_with_logits(z_d, y.float().to(DEV))
    loss_d.backward()

    z_r = ref64(smiles, gd, x, fp, branches=br)
    loss_r = bce_logits_ref(z_r, y)
    loss_r.backward()
    loss_32 = bce_logits_ref(ref32({"smiles": smiles["smiles"], "seq_len": smiles["seq_len"]}, gd,
                                   x.float(), fp.float(), branches=br), y.float())
    loss_32.backward()
    assert rel_err(z_d, z_r) < TOL
    assert abs(loss_d.item() - loss_r.item()) / abs(loss_r.item()) < TOL
    p64, p32 = dict(ref64.named_parameters()), dict(ref32.named_parameters())
    worst = (0.0, None)
    for n, p in mod.named_parameters():
        if p64[n].grad is None:  # unused LayerNorms (model.py:39, 120): no gradient anywhere
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, n
            continue
        e = rel_err(p.grad, p64[n].grad)
        budget = max(TOL, 4 * rel_err(p32[n].grad, p64[n].grad))
        worst = max(worst, (e / budget, n))
        assert e < budget, (n, e, budget)
    print(f"MVP: logits {rel_err(z_d, z_r):.2e}, loss {loss_d.item():.6f}, worst grad err/budget "
          f"{worst[0]:.2f} ({worst[1]})")
    # one Adam step on both sides (torch's Adam, main.py:88) from the matched gradients
    opt_r = torch.optim.Adam(ref64.parameters(), lr=1e-3, weight_decay=1e-4)
    with torch.no_grad():
        for n, p in mod.named_parameters():  # same gradients on both sides: compare the update
            if p.grad is not None and p64[n].grad is not None:
                p64[n].grad.copy_(p.grad.double().cpu())
    opt.step()
    opt_r.step()
    for n, p in mod.named_parameters():
        assert rel_err(p, p64[n]) < TOL, n


def test_mvp_train_step_dp_reducer_and_dropout_runs():
    """The config-4 step as bench.py runs it (train mode: dropout on) with the flat gradient
    reducer (a no-op on one process) — finite loss, every used parameter gets a gradient."""
    from mvml_gat.dist import FlatGradAllReduce
    from mvml_gat.mvp import train_step
    bg, gd, x, smiles, fp, y = _kegg_batch(32)
    mod, _, _ = _models(1)
    mod.train()
    g = bg.to(DEV)
    opt = torch.optim.Adam(mod.parameters(), lr=1e-3, weight_decay=1e-4)
    batch = ({"smiles": smiles["smiles"].to(DEV), "seq_len": smiles["seq_len"]}, g,
             g.ndata["h"].to(DEV), fp.float().to(DEV), y.float().to(DEV))
    losses = [train_step(mod, opt, batch, FlatGradAllReduce(mod.parameters())).item() for _ in range(3)]
    assert all(np.isfinite(losses)), losses
    used = [n for n, p in mod.named_parameters() if "norm_layer." not in n or n.startswith("norm_layer_module")]
    for n, p in mod.named_parameters():
        if n in used and not n.startswith("rnn.norm_layer"):
            assert p.grad is not None and torch.isfinite(p.grad).all(), n
