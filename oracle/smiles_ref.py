"""Oracle: the SMILES BiLSTM view of MVP (RNNModule) — TEST INFRASTRUCTURE ONLY.

CPU restatement of model.py:98-135 in plain PyTorch (run in float64 for parity), on torch's own
nn.Embedding / nn.LSTM / pack_padded_sequence, the library the reference calls:

    x = Embedding(39, E, padding_idx=0)(smiles.long())                          model.py:127
    packed = pack_padded_sequence(x, seq_len, batch_first=True, enforce_sorted=False)  :128
    output, _ = pad_packed_sequence(LSTM(E, H, L, bidirectional, batch_first)(packed))  :129-130
    fea = [output[b, len_b - 1, :H] | output[b, 0, H:]]                        model.py:131-133
    out = Dropout(ReLU(Linear(2H, out_dim)(fea)))                              model.py:121-134

Parity is pinned to torch's LSTM semantics (the reference's dependency, present here); torch
1.12.1 itself (README.md pin) is not, so versions could differ only in rounding.
"""
import numpy as np
import torch
import torch.nn as nn
from torch.nn.utils.rnn import pack_padded_sequence, pad_packed_sequence


class RNNModuleRef(nn.Module):
    def __init__(self, vocab_size=39, embed_dim=128, blstm_dim=384, num_layers=2, out_dim=384,
                 dropout=0.2, pad=0):
        super().__init__()
        self.blstm_dim = blstm_dim
        self.embeddings = nn.Embedding(vocab_size, embed_dim, padding_idx=pad)
        self.rnn = nn.LSTM(embed_dim, blstm_dim, num_layers=num_layers, bidirectional=True,
                           dropout=dropout, batch_first=True)
        self.drop = nn.Dropout(p=dropout)
        self.norm_layer = nn.LayerNorm(2 * blstm_dim)
        self.fc = nn.Sequential(nn.Linear(2 * blstm_dim, out_dim), nn.ReLU(), nn.Dropout(p=dropout))

    def forward(self, batch):
        smiles, seq_lens = batch["smiles"], batch["seq_len"]
        x = self.embeddings(smiles.long())
        packed = pack_padded_sequence(x, seq_lens, batch_first=True, enforce_sorted=False)
        packed_out, _ = self.rnn(packed)
        output, _ = pad_packed_sequence(packed_out, batch_first=True)
        out_forward = output[range(len(output)), np.array(seq_lens) - 1, :self.blstm_dim]
        out_reverse = output[:, 0, self.blstm_dim:]
        return self.fc(torch.cat((out_forward, out_reverse), 1))
