"""SMILES BiLSTM view (RNNModule, model.py:98-135): HIP path vs the float64
restatement on torch's nn.LSTM + pack_padded_sequence (oracle/smiles_ref.py)."""
import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-5


def _batch(B, seed, Tmax=60, ragged=True, space=False):
    from mvml_gat.smiles import collate_smiles, tokens_struct
    vocab = tokens_struct()
    rng = np.random.default_rng(seed)
    chars = [t for t in vocab.tokens if len(t) == 1 and t != ' '] + ['X', '%']  # '%','X' -> unk
    if space:  # the pad token ' ' (index 0) inside live positions
        chars += [' '] * 4
    lens = rng.integers(1, Tmax + 1, size=B) if ragged else np.full(B, Tmax)
    smiles = ["".join(rng.choice(chars, size=int(n))) for n in lens]
    return vocab, collate_smiles(smiles, vocab)


@pytest.mark.parametrize("B,Tmax,layers,ragged,space", [(1, 7, 2, True, False), (5, 1, 1, True, False),
                                                         (64, 60, 2, True, False), (33, 40, 3, False, False),
                                                         (24, 30, 2, True, True)])
def test_rnn_module_parity(B, Tmax, layers, ragged, space):
    """The fused step path (mvml_bilstm_seq_fwd / _bwd: B <= SEQ_MAX_B)."""
    _rnn_parity(B, Tmax, layers, ragged, space)


@pytest.mark.parametrize("wide_step", [True, False])
@pytest.mark.parametrize("B,Tmax,layers,ragged,space", [(64, 60, 2, True, False), (24, 30, 2, True, True),
                                                         (700, 25, 2, True, False)])
def test_rnn_module_parity_gemm_path(B, Tmax, layers, ragged, space, wide_step, monkeypatch):
    """The wide-batch paths, forced at small batches: wide_step = one dual launch per time step
    for both directions with the cell fused (mvml_bilstm_wide_step_fwd / _bwd, the default);
    False = a GEMM and a cell kernel per direction and step.  B = 700: three 256-row tiles with
    a ragged last one, and the live-row prefix shrinking across tiles."""
    import mvml_gat.smiles as sm
    monkeypatch.setattr(sm, "SEQ_MAX_B", 0)
    monkeypatch.setattr(sm, "WIDE_STEP", wide_step)
    monkeypatch.setattr(sm, "WIDE_PACK", wide_step)  # the live-row products with the step path
    _rnn_parity(B, Tmax, layers, ragged, space)


@pytest.mark.parametrize("wide_step,wide_pack", [(True, False), (False, True)])
def test_rnn_module_parity_mixed_paths(wide_step, wide_pack, monkeypatch):
    """The two mixed combinations at B = 700: the wide step over time-major gate projections
    (the branch that relies on the zero padding rows of gg), and the packed live-row products
    around the per-step GEMM + cell path."""
    import mvml_gat.smiles as sm
    monkeypatch.setattr(sm, "SEQ_MAX_B", 0)
    monkeypatch.setattr(sm, "WIDE_STEP", wide_step)
    monkeypatch.setattr(sm, "WIDE_PACK", wide_pack)
    _rnn_parity(700, 25, 2, True, False)


@pytest.mark.parametrize("H", [100, 36, 30])
def test_rnn_module_parity_hidden_sizes(H, monkeypatch):
    """Hidden sizes the wide step does not take (H % 8 != 0; 30: H % 4 != 0, so not packed
    either) fall back to the per-step GEMM + cell path instead of raising."""
    import mvml_gat.smiles as sm
    monkeypatch.setattr(sm, "SEQ_MAX_B", 0)
    _rnn_parity(300, 20, 2, True, False, H=H)


@pytest.mark.parametrize("B,Tmax,layers,ragged,space", [(64, 60, 2, True, False), (700, 25, 2, True, False)])
def test_rnn_module_parity_wide_step_tile256(B, Tmax, layers, ragged, space, monkeypatch):
    """The wide step launches on the 256x256 tile (option lstm_tile = 256; the planned tile at
    these row counts is the 128x128 one, which the test above covers)."""
    import mvml_gat.smiles as sm
    from mvml_gat._lib import option
    monkeypatch.setattr(sm, "SEQ_MAX_B", 0)
    with option("lstm_tile", 256):
        _rnn_parity(B, Tmax, layers, ragged, space)


def test_wide_step_plans_bitwise(monkeypatch):
    """The planned wide-step launches (128x128 tile, W_hh pre-split once per layer) and the
    256x256 tile (W_hh split in every workgroup) round identically: the same scales, the same
    split, the same k order — output and every gradient bitwise equal."""
    import mvml_gat.smiles as sm
    from mvml_gat._lib import option
    from mvml_gat.smiles import RNNModule
    monkeypatch.setattr(sm, "SEQ_MAX_B", 0)
    torch.manual_seed(5)
    vocab, batch = _batch(700, 11, 25, True, False)
    mod = RNNModule(vocab, 128, 384, 2, 384, 0.5).to(DEV).eval()
    inp = {"smiles": batch["smiles"].to(DEV), "seq_len": batch["seq_len"]}
    res = []
    for tile in (0, 256):
        with option("lstm_tile", tile):
            mod.zero_grad(set_to_none=True)
            z = mod(inp)
            z.square().sum().backward()
            torch.cuda.synchronize()
            res.append([z.detach().clone()] + [p.grad.clone() for p in mod.parameters() if p.grad is not None])
            del z
    assert len(res[0]) == len(res[1]) > 1
    for a, b in zip(*res):
        assert torch.equal(a, b)


def _rnn_parity(B, Tmax, layers, ragged, space, H=384):
    from mvml_gat.smiles import RNNModule
    from oracle.smiles_ref import RNNModuleRef
    torch.manual_seed(B + layers)
    vocab, batch = _batch(B, B * 7 + Tmax, Tmax, ragged, space)
    if space:
        assert any((row[:n] == 0).any() for row, n in zip(batch["smiles"], batch["seq_len"]))
    ref = RNNModuleRef(39, 128, H, layers, 384, 0.5).double().eval()
    mod = RNNModule(vocab, 128, H, layers, 384, 0.5).to(DEV).eval()
    mod.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    zr = ref(batch)
    zd = mod({"smiles": batch["smiles"].to(DEV), "seq_len": batch["seq_len"]})
    assert zd.shape == (B, 384)
    assert rel_err(zd, zr) < TOL
    g = torch.Generator().manual_seed(B)
    up = torch.randn(zr.shape, generator=g, dtype=torch.float64)
    (zr * up).sum().backward()
    (zd * up.float().to(DEV)).sum().backward()
    pr = dict(ref.named_parameters())
    for name, p in mod.named_parameters():
        if pr[name].grad is None:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, name
            continue
        assert rel_err(p.grad, pr[name].grad) < TOL, name


def test_rnn_module_deterministic():
    from mvml_gat.smiles import RNNModule
    vocab, batch = _batch(16, 3, 30)
    torch.manual_seed(0)
    mod = RNNModule(vocab, 128, 384, 2, 384, 0.5).to(DEV).eval()
    b = {"smiles": batch["smiles"].to(DEV), "seq_len": batch["seq_len"]}
    outs = []
    for _ in range(2):
        mod.zero_grad()
        z = mod(b)
        z.square().sum().backward()
        outs.append((z.detach().clone(), mod.rnn.weight_hh_l0.grad.clone(), mod.embeddings.weight.grad.clone()))
    for a, c in zip(*outs):
        assert torch.equal(a, c)


def test_rnn_module_rejects_empty_sequence():
    from mvml_gat.smiles import RNNModule
    vocab, batch = _batch(4, 1, 10)
    mod = RNNModule(vocab, 128, 384, 1, 384).to(DEV)
    with pytest.raises(RuntimeError):
        mod({"smiles": batch["smiles"].to(DEV), "seq_len": [0] + batch["seq_len"][1:]})


@pytest.mark.timeout(900)
def test_rnn_module_bench_size():
    """the wide BiLSTM at config 4's size — 8,192 molecules per step with the
    bench's token lengths (about 1.8 characters per atom of the config-3 set, 5 .. 462) — output
    and every parameter gradient against the float64 restatement run on the GPU (aten LSTM:
    MIOpen has no float64 RNN), margins to MVML_MARGINS_DIR."""
    import json
    import os
    from mvml_gat import synth
    from mvml_gat.smiles import RNNModule, tokens_struct
    from oracle.smiles_ref import RNNModuleRef
    B = 8192
    sb = synth.Config3Set(1_000_000, seed=0).molecules(0, B)
    rng = np.random.default_rng([0, 77])
    lens = np.clip(np.rint(1.8 * sb.num_nodes * rng.uniform(0.8, 1.2, B)), 5, 462).astype(np.int64)
    T = int(lens.max())
    tok = rng.integers(2, 39, size=(B, T)).astype(np.float32)
    tok[np.arange(T)[None, :] >= lens[:, None]] = 0.0
    batch = {"smiles": torch.from_numpy(tok), "seq_len": lens.tolist()}
    torch.manual_seed(9)
    ref = RNNModuleRef(39, 128, 384, 2, 384, 0.5).double().eval()
    mod = RNNModule(tokens_struct(), 128, 384, 2, 384, 0.5).to(DEV).eval()
    mod.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    up = torch.randn((B, 384), generator=torch.Generator().manual_seed(3), dtype=torch.float64)
    zd = mod({"smiles": batch["smiles"].to(DEV), "seq_len": batch["seq_len"]})
    (zd * up.float().to(DEV)).sum().backward()
    torch.cuda.synchronize()
    ref = ref.to(DEV)
    with torch.backends.cudnn.flags(enabled=False):
        zr = ref({"smiles": batch["smiles"].to(DEV), "seq_len": batch["seq_len"]})
        (zr * up.to(DEV)).sum().backward()
    errs = {"out": rel_err(zd, zr)}
    pr = dict(ref.named_parameters())
    for name, p in mod.named_parameters():
        if pr[name].grad is None:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, name
            continue
        errs[name] = rel_err(p.grad, pr[name].grad)
    out = os.environ.get("MVML_MARGINS_DIR", os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "gpurun_out", "parity_margins"))
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "bilstm_bench_size.json"), "w") as f:
        json.dump({"molecules": B, "T": T, "live_rows": int(lens.sum()), "errors": errs}, f, indent=1)
    print(errs)
    for k, e in errs.items():
        assert e < TOL, (k, e)
