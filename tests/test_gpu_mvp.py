"""The whole MVP model (model.py:13-75) on the HIP path — BASELINE config 4's training step
(main.py:24-36): RNNModule + GNNModule + FPNModule (fp_2_dim = 512, config.py:16) + fusion head
+ BCEWithLogits + Adam (lr 1e-3, wd 1e-4, main.py:88) — against the composed float64 oracle
(oracle/fusion_ref.py MVPRef) on one 64-molecule KEGG batch (the first test-split batch,
data_index.txt order, featurised by mvml_gat.featurize; fingerprints from
mvml_gat.fingerprints, the restated MACCS / ErG / PubChem / Morgan of dataset.py:37-45 —
RDKit agreement unpinned, tests/test_fingerprints.py).

Bars: logits / loss within 1e-5 of float64; every parameter gradient within 1e-5 or 4x the
fp32 oracle's own error where conditioning makes fp32 lose that much (see
test_gpu_parity_configs.py); after one Adam step the parameters within 1e-5.  Natural biases
everywhere: the fusion ReLUs' sides (Conv2d, MLP) and the GAT LeakyReLU sides come from the
product's own fp32 outputs and the float64 oracle is evaluated on them (test_gpu_fusion.py,
test_gpu_parity_configs.py) — a pre-activation within fp32 rounding of 0 picks a subgradient."""
import os

import numpy as np
import pytest
import torch

from _util import randomize_
from conftest import rel_err
from test_gpu_parity_configs import _branches

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
    from mvml_gat.fingerprints import fingerprints
    fp = torch.as_tensor(fingerprints(ds.smiles[:n])).double()  # dataset.py:37-45 (restated)
    return bg, gd, x, smiles, fp, y.double()


def _models(seed=0):
    from mvml_gat.mvp import MVP
    from oracle.fusion_ref import MVPRef
    torch.manual_seed(seed)
    mod = MVP(11, 74, [192, 384], 6, 3, 128, 384, 2, 512, 12, 0.5)
    randomize_(mod.gnn, seed)
    with torch.no_grad():
        mod.norm_layer_module.weight.uniform_(0.5, 1.5)
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
    from mvml_gat import functional as Fn
    cap = {}
    Fn.DEBUG_CAPTURE = cap
    try:
        z_d = mod(sm_d, g, g.ndata["h"].to(DEV), fp.float().to(DEV))
    finally:
        Fn.DEBUG_CAPTURE = None
    br = _branches(gd, [e.cpu() for e in cap["elr_fwd"]])
    conv = (cap["conv_out"] > 0).unsqueeze(2).cpu()
    mlp = (cap["relu_out"][-1] > 0).cpu()
    loss_d = bce_with_logits(z_d, y.float().to(DEV))
    loss_d.backward()

    z_r = ref64(smiles, gd, x, fp, branches=br, conv_branch=conv, mlp_branch=mlp)
    loss_r = bce_logits_ref(z_r, y)
    loss_r.backward()
    loss_32 = bce_logits_ref(ref32({"smiles": smiles["smiles"], "seq_len": smiles["seq_len"]}, gd,
                                   x.float(), fp.float(), branches=br, conv_branch=conv,
                                   mlp_branch=mlp), y.float())
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


def test_mvp_train_step_bf16_projection():
    """BASELINE config 4 as written: the MVP training step with the GAT projection GEMMs on bf16
    operands (proj_dtype=torch.bfloat16, fp32 accumulate) against the float64 oracle of the fp32
    reference semantics: logits and loss within north_star's bf16 bar 2e-2; gradients held
    norm-wise (Frobenius) and by direction as test_gpu_bf16.py does (a bf16-perturbed
    pre-activation that crosses a kink flips single gradient entries by O(1)) against the
    bf16-EMULATED float64 oracle (test_gpu_bf16.check_emulated); one Adam step."""
    from mvml_gat import bce_with_logits
    from mvml_gat.mvp import MVP
    from oracle.fusion_ref import MVPRef, bce_logits_ref
    from test_gpu_bf16 import EMU_FRO, TOL_BF16, check_emulated
    bg, gd, x, smiles, fp, y = _kegg_batch()
    _, ref64, _ = _models()
    emu = MVPRef().double().eval()
    emu.load_state_dict(ref64.state_dict())
    emu.gnn.proj = "bf16"
    mod = MVP(11, 74, [192, 384], 6, 3, 128, 384, 2, 512, 12, 0.5, proj_dtype=torch.bfloat16)
    mod.load_state_dict({k: v.float() for k, v in ref64.state_dict().items()})
    mod = mod.to(DEV).eval()
    g = bg.to(DEV)
    sm_d = {"smiles": smiles["smiles"].to(DEV), "seq_len": smiles["seq_len"]}
    opt = torch.optim.Adam(mod.parameters(), lr=1e-3, weight_decay=1e-4)
    opt.zero_grad()
    z_d = mod(sm_d, g, g.ndata["h"].to(DEV), fp.float().to(DEV))
    loss_d = bce_with_logits(z_d, y.float().to(DEV))
    loss_d.backward()
    z_r = ref64(smiles, gd, x, fp)
    loss_r = bce_logits_ref(z_r, y)
    loss_r.backward()
    z_e = emu(smiles, gd, x, fp)
    bce_logits_ref(z_e, y).backward()
    e_z = rel_err(z_d, z_r)
    assert 1e-7 < e_z < TOL_BF16, e_z
    assert rel_err(z_d, z_e) < EMU_FRO
    assert abs(loss_d.item() - loss_r.item()) / abs(loss_r.item()) < TOL_BF16
    rows, bad = check_emulated(mod.named_parameters(), dict(emu.named_parameters()),
                               dict(ref64.named_parameters()))
    print(f"MVP bf16 projection: logits {e_z:.2e}; worst grads (vs emulated, vs exact, emulated vs "
          "exact)", sorted(rows.items(), key=lambda kv: -kv[1][0])[:4])
    assert not bad, bad
    opt.step()
    assert all(torch.isfinite(p).all() for p in mod.parameters())


@pytest.mark.parametrize("n", [64, 600])
def test_mvp_view_streams_bitwise(n):
    """MVP.forward runs the SMILES view on a side stream beside the graph view: logits and every
    parameter gradient are bitwise those of running the views one after the other (64 molecules:
    the narrow BiLSTM path; 600 = the KEGG batch repeated: the wide path)."""
    import mvml_gat.mvp as mvp_mod
    from mvml_gat.featurize import MolDataSet, collate
    from mvml_gat.smiles import collate_smiles, tokens_struct
    ds = MolDataSet(os.path.join(HERE, "golden", "kegg_test_split.csv"))
    idx = [i % 64 for i in range(n)]
    bg, y = collate([ds[i] for i in idx])
    smiles = collate_smiles([ds.smiles[i] for i in idx], tokens_struct())
    fp = (torch.rand(n, 2513, generator=torch.Generator().manual_seed(3)) < 0.1).float()
    mod, _, _ = _models(2)
    g = bg.to(DEV)
    batch = ({"smiles": smiles["smiles"].to(DEV), "seq_len": smiles["seq_len"]}, g, g.ndata["h"].to(DEV),
             fp.to(DEV))
    res = []
    for overlap in (True, False):
        old = mvp_mod.OVERLAP_VIEWS
        mvp_mod.OVERLAP_VIEWS = overlap
        try:
            mod.zero_grad(set_to_none=True)
            z = mod(*batch)
            (z.square().mean()).backward()
            torch.cuda.synchronize()
            res.append([z.detach().clone()] + [p.grad.clone() for p in mod.parameters() if p.grad is not None])
            del z  # drop this pass's autograd graph (its AccumulateGrad nodes carry their stream)
        finally:
            mvp_mod.OVERLAP_VIEWS = old
    assert len(res[0]) == len(res[1])
    for a, b in zip(*res):
        assert torch.equal(a, b)
