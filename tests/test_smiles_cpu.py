"""Host-side pieces of the SMILES BiLSTM view (no GPU): vocabulary (utils.py:55-88), collate
(dataset.py:47-59), pack_padded_sequence metadata, and the oracle's pack/select semantics."""
import numpy as np
import torch

from mvml_gat.smiles import Packing, RNNModule, collate_smiles, tokens_struct


def test_vocab_matches_reference_indices():
    v = tokens_struct()
    assert v.tokens_length == 39 and v.pad == 0 and v.unk == 1
    enc = v.encode(list("CC(=O)Cl%"))
    assert enc.dtype == np.float32
    assert enc.tolist() == [2, 2, 4, 7, 3, 5, 2, 20, 1]
    assert v.decode([2, 20]) == "Cl"


def test_collate_pads_with_zero():
    b = collate_smiles(["CCO", "C", "c1ccccc1"], tokens_struct())
    assert b["seq_len"] == [3, 1, 8]
    assert b["smiles"].shape == (3, 8)
    assert b["smiles"][1, 1:].abs().sum() == 0


def test_packing_metadata():
    b = collate_smiles(["CCO", "C", "c1ccccc1", "CC"], tokens_struct())
    pk = Packing(b["seq_len"], b["smiles"], 39)
    # pack_padded_sequence's batch_sizes for lengths [3, 1, 8, 2]
    ref = torch.nn.utils.rnn.pack_padded_sequence(torch.zeros(4, 8, 1), b["seq_len"],
                                                  batch_first=True, enforce_sorted=False)
    assert pk.batch_sizes == ref.batch_sizes.tolist()
    assert pk.perm.tolist() == [2, 0, 3, 1]
    assert pk.pos.tolist() == [1, 3, 0, 2]


def test_state_dict_keys_match_oracle():
    from oracle.smiles_ref import RNNModuleRef
    ref = RNNModuleRef(39, 64, 128, 2, 384)
    mod = RNNModule(tokens_struct(), 64, 128, 2, 384)
    rs, ms = ref.state_dict(), mod.state_dict()
    assert list(rs.keys()) == list(ms.keys())
    assert all(rs[k].shape == ms[k].shape for k in rs)


def test_product_path_refuses_cpu_tensors():
    mod = RNNModule(tokens_struct(), 64, 128, 1, 384)
    b = collate_smiles(["CCO"], tokens_struct())
    try:
        mod(b)
    except (RuntimeError, TypeError) as e:
        assert "CPU fallback" in str(e) or "CUDA" in str(e)
    else:
        raise AssertionError("RNNModule ran on CPU tensors")
