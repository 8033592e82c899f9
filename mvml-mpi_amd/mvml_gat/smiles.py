"""SMILES BiLSTM view of MVP (RNNModule, /root/reference/model.py:98-135) on
the HIP path, plus the reference's SMILES vocabulary (tokens_struct, utils.py:55-88).

    RNNModule(vocab, embed_dim=128, blstm_dim=384, num_layers=2, out_dim=384, dropout)(batch)

``batch`` is the reference's ``{"smiles": padded tokens [B, T], "seq_len": [len_b]}`` dict
(dataset.py:56-59).  Parameter names / shapes equal the reference's (``embeddings.weight``,
``rnn.weight_ih_l{k}[_reverse]``, ``rnn.weight_hh_…``, ``rnn.bias_{ih,hh}_…``, ``norm_layer.*``,
``fc.0.*``), so a reference state_dict loads unchanged.

Design (not a cuDNN/MIOpen RNN call): the packed sequence of pack_padded_sequence
(enforce_sorted=False) is kept as a time-major [T, B, 2H] buffer with the batch sorted by
descending length, so the sequences alive at step t are a row prefix.  Per layer and direction
one MFMA GEMM projects every position's input at once (layer 0: a [vocab, 4H] table lookup,
mvml_bilstm_gather_rows).  The recurrence then runs in ONE C-ABI call per layer
(mvml_bilstm_seq_fwd / _bwd): one fused launch per time step carries both directions, the
recurrent product and the LSTM cell, with the step loop on the native side (no Python per step).
Batches wider than SEQ_MAX_B rows take the per-step MFMA GEMM (h_prev W_hh^T, beta = 1 onto the
projection, M = the live prefix) + cell-kernel path instead, where the product is FLOP-bound.
Weight gradients are single GEMMs over all positions; the embedding / W_ih_l0 gradient is a
deterministic per-token reduction.  Padded positions stay zero, as pad_packed_sequence's are.
"""
import math

import numpy as np
import torch
import torch.nn as nn

from . import functional as _F
from ._lib import call, lib, ptr, workspace
from .functional import LinearReLUFunction, _c, _check_cuda_f32, _stream, absmax, colsum, gemm, slot


class tokens_struct:
    """The reference's SMILES character vocabulary (utils.py:55-88): 39 tokens, pad ' ' = 0,
    '<unk>' = 1 for characters outside the list."""

    def __init__(self):
        self.tokens = [' ', '<unk>', 'C', 'O', '(', ')', 'c', '=', '1', '2', 'N', '3', 'n', 'P',
                       '4', '[', ']', 'S', 'H', '5', 'l', '-', '*', 'o', '+', '6', '#', 'M', 'F',
                       'g', '7', 'B', 'r', 's', 'I', 'e', 'i', '8', 'Z']
        self.tokens_length = len(self.tokens)
        self.tokens_vocab = dict(zip(self.tokens, range(len(self.tokens))))
        self.reversed_tokens_vocab = {v: k for k, v in self.tokens_vocab.items()}

    @property
    def unk(self):
        return self.tokens_vocab['<unk>']

    @property
    def pad(self):
        return self.tokens_vocab[' ']

    def get_default_tokens(self):
        return self.tokens

    def get_tokens_length(self):
        return self.tokens_length

    def encode(self, char_list):
        """Characters -> float32 indices, unknown -> unk (utils.py:80-88)."""
        return np.array([self.tokens_vocab.get(ch, self.unk) for ch in char_list], dtype=np.float32)

    def decode(self, matrix):
        return "".join(self.reversed_tokens_vocab[int(i)] for i in matrix)


def collate_smiles(smiles_list, vocab):
    """dataset.py:47-59's SMILES half: per-character encode, pad_sequence(batch_first) with 0."""
    enc = [vocab.encode(list(s)) for s in smiles_list]
    seq_len = [e.size for e in enc]
    T = max(seq_len) if enc else 0
    out = np.zeros((len(enc), T), dtype=np.float32)
    for i, e in enumerate(enc):
        out[i, :e.size] = e
    return {"smiles": torch.from_numpy(out), "seq_len": seq_len}


class Packing:
    """Host-side pack_padded_sequence(enforce_sorted=False) metadata (the reference computes it on
    the CPU from the ``seq_len`` list as well): descending-length order, batch_sizes per step."""

    def __init__(self, seq_lens, tokens, vocab_size, pad=None):
        self.pad = pad
        lens = np.asarray(list(seq_lens), dtype=np.int64)
        if lens.ndim != 1 or lens.size == 0:
            raise ValueError("seq_len must be a non-empty list of lengths")
        if tokens.dim() != 2 or tokens.shape[0] != lens.size:
            raise ValueError(f"smiles must be [B, T] with B = len(seq_len), got {tuple(tokens.shape)}")
        if lens.min() < 1 or lens.max() > tokens.shape[1]:
            # pack_padded_sequence: "Length of all samples has to be greater than 0"
            raise RuntimeError("Length of all samples has to be greater than 0 and at most T")
        self.B = int(lens.size)
        self.T = int(lens.max())
        perm = np.argsort(-lens, kind="stable")
        pos = np.empty_like(perm)
        pos[perm] = np.arange(self.B)
        self.batch_sizes = [int((lens > t).sum()) for t in range(self.T)]
        # host int32 copy for the native step loops (mvml_bilstm_seq_*)
        self.batch_sizes_host = torch.tensor(self.batch_sizes, dtype=torch.int32)
        dev = tokens.device
        tok = tokens.to(torch.int64)
        if int(tok.min()) < 0 or int(tok.max()) >= vocab_size:
            raise IndexError("token index out of range of the embedding table")
        self.tokens = tok.to(torch.int32).contiguous()
        self.ldtok = int(tokens.shape[1])
        self.lens = torch.from_numpy(lens.astype(np.int32)).to(dev)
        self.perm = torch.from_numpy(perm.astype(np.int32)).to(dev)
        self.pos = torch.from_numpy(pos.astype(np.int32)).to(dev)
        self._offs = {}

    def packed_tokens(self):
        """Device int32 token of every packed live row (mvml_bilstm_packed_tokens)."""
        if getattr(self, "_ptok", None) is None:
            offs, n = self.live_offsets(0, self.T)
            self._ptok = torch.empty((max(n, 1),), dtype=torch.int32, device=self.lens.device)
            call("mvml_bilstm_packed_tokens", n, self.T, ptr(offs), ptr(self.tokens), self.ldtok,
                 ptr(self.perm), ptr(self._ptok), _stream(self.lens.device))
        return self._ptok

    def live_offsets(self, t0, t1):
        """(device int32 offsets[t1 - t0 + 1], rows): the live rows of steps [t0, t1) packed
        consecutively (mvml_bilstm_pack_rows)."""
        key = (t0, t1)
        if key not in self._offs:
            o = np.concatenate([[0], np.cumsum(self.batch_sizes[t0:t1])]).astype(np.int32)
            self._offs[key] = (torch.from_numpy(o).to(self.lens.device), int(o[-1]))
        return self._offs[key]


SEQ_MAX_B = 512  # fused step path up to this batch width (the GEMM path above)
# wider batches: the products over every position (input projections, weight / input
# gradients) run over the live rows of the packed sequence only (mvml_bilstm_pack_rows);
# False = over all T x B rows (padding rows are zeros)
WIDE_PACK = True
# wider batches: one dual launch per time step (both directions, the LSTM cell in the GEMM
# epilogue / a fused reduce + cell-backward kernel) on the split-fp16 GEMM; False = a GEMM and a
# cell kernel per direction and step (kept, tested)
WIDE_STEP = True
SEQ_H = 384      # the fused step kernels are built for MVP's blstm_dim (config.py)


def _use_seq(pk, H):
    return pk.B <= SEQ_MAX_B and H == SEQ_H


class BiLSTMLayerFunction(torch.autograd.Function):
    """One bidirectional nn.LSTM layer over the packed batch.  ``x`` is the previous layer's
    [T, B, 2H] output, or for layer 0 (``pk_tokens`` = True) the embedding table [V, E]."""

    @staticmethod
    def forward(ctx, x, pk, layer0, *w):
        _check_cuda_f32(x, "x")
        dev = x.device
        st = _stream(dev)
        T, B = pk.T, pk.B
        H = w[1].shape[1]
        G = 4 * H
        x = _c(x)
        In = x.shape[-1]
        out = torch.zeros((T, B, 2 * H), dtype=torch.float32, device=dev)
        saved, gates_d = [], []
        wide_pack = WIDE_PACK and not _use_seq(pk, H) and In % 4 == 0 and H % 4 == 0
        amx = _h_bounds(w, dev) if not _use_seq(pk, H) else None
        # the native wide recurrence (H % 8 == 0) reads a packed input projection directly
        wide_step = WIDE_STEP and amx is not None and _wide_step_ok(H)
        gx_packed = wide_pack and not layer0 and wide_step
        xp = None
        for d in range(2):
            w_ih = _c(w[4 * d])
            if gx_packed:
                xp = _pack(pk, x, In, In) if d == 0 else xp
                gp = torch.empty((xp.shape[0], G), dtype=torch.float32, device=dev)
                gemm(xp, w_ih, xp.shape[0], G, In, 0, 0, In, In, gp, G)
                gates_d.append(gp)
                continue
            gates = torch.empty((T, B, G), dtype=torch.float32, device=dev)
            if layer0:
                V = x.shape[0]
                P = torch.empty((V, G), dtype=torch.float32, device=dev)
                gemm(x, w_ih, V, G, In, 0, 0, In, In, P, G)
                call("mvml_bilstm_gather_rows", T, B, G, ptr(P), ptr(pk.tokens), pk.ldtok,
                     ptr(pk.lens), ptr(pk.perm), ptr(gates), st)
            elif wide_pack:  # only the live rows (a third of T x B for KEGG-like lengths)
                xp = _pack(pk, x, In, In) if d == 0 else xp
                gp = torch.empty((xp.shape[0], G), dtype=torch.float32, device=dev)
                gemm(xp, w_ih, xp.shape[0], G, In, 0, 0, In, In, gp, G)
                _unpack(pk, gp, gates, G, G)
                del gp
            else:
                gemm(x, w_ih, T * B, G, In, 0, 0, In, In, gates, G)
            gates_d.append(gates)
        if _use_seq(pk, H):  # one native call: every step of both directions
            wc = [_c(t) for t in w]
            c = [torch.zeros((T, B, H), dtype=torch.float32, device=dev) for _ in range(2)]
            act = [torch.empty((T, B, G), dtype=torch.float32, device=dev) for _ in range(2)]
            call("mvml_bilstm_seq_fwd", T, B, H, ptr(pk.batch_sizes_host), ptr(gates_d[0]),
                 ptr(gates_d[1]), ptr(wc[1]), ptr(wc[5]), ptr(wc[2]), ptr(wc[3]), ptr(wc[6]),
                 ptr(wc[7]), ptr(out), ptr(c[0]), ptr(c[1]), ptr(act[0]), ptr(act[1]), st)
            saved = [c[0], act[0], c[1], act[1]]
        elif wide_step:
            # wide batches: one launch per time step for both directions, the recurrent product
            # and the LSTM cell fused (mvml_bilstm_wide_step_fwd)
            wperm = [_c(w[4 * d + 1]).view(4, H, H).transpose(0, 1).reshape(G, H).contiguous()
                     for d in range(2)]  # rows 4 j + q = gate q of unit j
            bias = [(_c(w[4 * d + 2]), _c(w[4 * d + 3])) for d in range(2)]
            c = [torch.zeros((T, B, H), dtype=torch.float32, device=dev) for _ in range(2)]
            act = [torch.empty((T, B, G), dtype=torch.float32, device=dev) for _ in range(2)]
            nws = int(lib().mvml_bilstm_wide_fwd_workspace_size(H))
            ws = workspace(nws, dev)
            call("mvml_bilstm_wide_fwd", T, B, H, ptr(pk.batch_sizes_host), ptr(wperm[0]), ptr(wperm[1]),
                 ptr(gates_d[0]), ptr(gates_d[1]), ptr(bias[0][0]), ptr(bias[0][1]), ptr(bias[1][0]),
                 ptr(bias[1][1]), ptr(c[0]), ptr(c[1]), ptr(out), ptr(act[0]), ptr(act[1]), ptr(amx),
                 1 if gx_packed else 0, ptr(ws), nws, st)
            saved = [c[0], act[0], c[1], act[1]]
        else:  # wide batches, other GEMM algorithms: per-step GEMM (beta = 1 onto the projection) + cell kernel
            for d in range(2):
                w_hh, b_ih, b_hh = (_c(t) for t in w[4 * d + 1:4 * d + 4])
                gates = gates_d[d]
                c = torch.zeros((T, B, H), dtype=torch.float32, device=dev)
                act = torch.empty((T, B, G), dtype=torch.float32, device=dev)
                order = range(T) if d == 0 else range(T - 1, -1, -1)
                prev = None
                for t in order:
                    bs = pk.batch_sizes[t]
                    c_prev = None
                    if prev is not None:
                        gemm(out[prev, :, d * H:], w_hh, bs, G, H, 0, 0, 2 * H, H, gates[t], G, beta=1.0,
                             amax=None if amx is None else (slot(amx, 0), slot(amx, 1 + d)))
                        c_prev = c[prev]
                    call("mvml_lstm_cell_fwd", bs, H, ptr(gates[t]), ptr(b_ih), ptr(b_hh), ptr(c_prev),
                         ptr(c[t]), ptr(out[t, :, d * H:]), 2 * H, ptr(act[t]), None, 0, st)
                    prev = t
                saved += [c, act]
        ctx.pk, ctx.layer0, ctx.H = pk, layer0, H
        ctx.xp = xp  # the packed live input rows: the weight gradient reads them again
        ctx.save_for_backward(x, out, *saved, *w)
        return out

    @staticmethod
    def backward(ctx, g_out):
        x, out, c0, a0, c1, a1, *w = ctx.saved_tensors
        pk, layer0, H = ctx.pk, ctx.layer0, ctx.H
        dev = x.device
        st = _stream(dev)
        T, B, G = pk.T, pk.B, 4 * H
        In = x.shape[-1]
        g = g_out.contiguous()
        cs, acts = (c0, c1), (a0, a1)
        g_w = [None] * 8
        g_x = torch.empty_like(x)
        # W_hh^T [H, 4H] once per backward: the recurrent product reads it k-contiguous
        w_hhT = [_c(w[4 * d + 1]).t().contiguous() for d in range(2)]
        seq = _use_seq(pk, H)
        amx = None if seq else _h_bounds(w, dev)
        packed = not seq and WIDE_PACK and In % 4 == 0 and H % 4 == 0
        wide_step = not seq and WIDE_STEP and amx is not None and _wide_step_ok(H)
        # the native wide recurrence writes the gate gradients packed (live rows only: no zero
        # fill of T x B rows, no pack before the weight-gradient products)
        gg_packed = packed and wide_step
        if gg_packed:
            n_live = pk.live_offsets(0, T)[1]
            ggs = [torch.empty((n_live, G), dtype=torch.float32, device=dev) for _ in range(2)]
        else:
            ggs = [torch.zeros((T, B, G), dtype=torch.float32, device=dev) for _ in range(2)]
        if seq:
            carry = torch.zeros((2, B, H), dtype=torch.float32, device=dev)
            call("mvml_bilstm_seq_bwd", T, B, H, ptr(pk.batch_sizes_host), ptr(w_hhT[0]),
                 ptr(w_hhT[1]), ptr(a0), ptr(a1), ptr(c0), ptr(c1), ptr(g), ptr(ggs[0]),
                 ptr(ggs[1]), ptr(carry), st)
        amg = None
        if not seq:
            # running max |dgates| per direction, folded in by mvml_lstm_cell_bwd (a bound for
            # every step already processed, which is all a scale needs)
            amg = torch.zeros(2, dtype=torch.int32, device=dev) if amx is not None else None
        if wide_step:
            # wide batches: one launch per step for both directions (the recurrent product split in
            # two K halves) + one fused reduce / cell-backward launch (mvml_bilstm_wide_step_bwd)
            carry = torch.zeros((2, 2, B, H), dtype=torch.float32, device=dev)
            nws = int(lib().mvml_bilstm_wide_bwd_workspace_size(B, H))
            ws = workspace(nws, dev)
            call("mvml_bilstm_wide_bwd", T, B, H, ptr(pk.batch_sizes_host), ptr(w_hhT[0]), ptr(w_hhT[1]),
                 ptr(g), ptr(acts[0]), ptr(acts[1]), ptr(cs[0]), ptr(cs[1]), ptr(carry), ptr(ggs[0]),
                 ptr(ggs[1]), ptr(amg), ptr(amx), 1 if gg_packed else 0, ptr(ws), nws, st)
        elif not seq:  # wide batches: per-step recurrent GEMM (beta = 1 into g) + cell kernel
            g = g.clone()
            for d in range(2):
                c, act, gg = cs[d], acts[d], ggs[d]
                carry = [torch.zeros((B, H), dtype=torch.float32, device=dev) for _ in range(2)]
                order = range(T - 1, -1, -1) if d == 0 else range(T)
                nxt, k = None, 0
                for t in order:
                    bs = pk.batch_sizes[t]
                    if nxt is not None:  # recurrent gradient from the step this one fed
                        rows = min(bs, pk.batch_sizes[nxt])
                        gemm(gg[nxt], w_hhT[d], rows, H, G, 0, 0, G, G, g[t, :, d * H:], 2 * H, beta=1.0,
                             amax=None if amg is None else (slot(amg, d), slot(amx, 1 + d)))
                    tp = t - 1 if d == 0 else t + 1
                    c_prev = c[tp] if 0 <= tp < T else None
                    g_c = carry[k % 2] if nxt is not None else None
                    call("mvml_lstm_cell_bwd", bs, H, ptr(act[t]), ptr(c[t]), ptr(c_prev),
                         ptr(g[t, :, d * H:]), 2 * H, None, 0, ptr(g_c), ptr(gg[t]), ptr(carry[(k + 1) % 2]),
                         slot(amg, d), None, st)
                    nxt, k = t, k + 1
        # weight / input gradients: GEMMs over every position — on the wide path over the live
        # rows only (packed), else over all T x B rows (the padding rows of gg are zeros)
        if packed:
            offs, n_live = pk.live_offsets(0, T)
            xp = None if layer0 else (ctx.xp if ctx.xp is not None else _pack(pk, x, In, In))
            ctx.xp = None
            gxp = None if layer0 else torch.empty((n_live, In), dtype=torch.float32, device=dev)
            g_x = g_x if layer0 else torch.zeros_like(x)
        for d in range(2):
            w_ih, gg = _c(w[4 * d]), ggs[d]
            gb = torch.empty(G, dtype=torch.float32, device=dev)
            ggp = _pack(pk, gg, G, G) if packed and not gg_packed else gg
            rows = ggp.shape[0] if packed else T * B
            colsum(ggp, rows, G, G, gb)
            g_whh = torch.zeros((G, H), dtype=torch.float32, device=dev)
            if T > 1:
                if packed:  # pairs (gg[t], h[t -+ 1]) of the live rows of gg
                    t0, t1, sh = (1, T, -1) if d == 0 else (0, T - 1, 1)
                    # gg's live rows of steps [t0, t1) are a contiguous slice of ggp (steps
                    # [1, T): all but the first step's rows; [0, T - 1): all but the last's)
                    A = ggp[pk.batch_sizes[0]:] if d == 0 else ggp[:rows - pk.batch_sizes[T - 1]]
                    Bm = _pack(pk, out[:, :, d * H:], H, 2 * H, t0, t1, sh)
                    gemm(A, Bm, G, H, A.shape[0], 1, 1, G, H, g_whh, H,  # Bm = h: |h| < 1
                         amax=None if amg is None else (slot(amg, d), slot(amx, 0)))
                    del A, Bm
                else:
                    A, Bm = (gg[1:], out[:-1, :, d * H:]) if d == 0 else (gg[:-1], out[1:, :, d * H:])
                    gemm(A, Bm, G, H, (T - 1) * B, 1, 1, G, 2 * H, g_whh, H,  # Bm = h: |h| < 1
                         amax=None if amg is None else (slot(amg, d), slot(amx, 0)))
            g_wih = torch.empty((G, In), dtype=torch.float32, device=dev)
            beta = 1.0 if d else 0.0
            if layer0:
                V = x.shape[0]
                Gt = torch.empty((V, G), dtype=torch.float32, device=dev)
                if packed:  # over the live rows only
                    nws = int(lib().mvml_bilstm_token_grad_packed_workspace(rows, G, V))
                    ws = workspace(nws, dev)
                    call("mvml_bilstm_token_grad_packed", rows, G, ptr(ggp), G, ptr(pk.packed_tokens()),
                         V, ptr(Gt), ptr(ws), nws, st)
                else:
                    nws = int(lib().mvml_bilstm_token_grad_workspace(T, B, G, V))
                    ws = workspace(nws, dev)
                    call("mvml_bilstm_token_grad", T, B, G, ptr(gg), ptr(pk.tokens), pk.ldtok,
                         ptr(pk.lens), ptr(pk.perm), V, ptr(Gt), ptr(ws), nws, st)
                gemm(Gt, x, G, In, V, 1, 1, G, In, g_wih, In)
                gemm(Gt, w_ih, V, In, G, 0, 1, G, In, g_x, In, beta=beta)
                if d == 1 and pk.pad is not None:
                    # nn.Embedding(padding_idx=pad) (model.py:113): the padding row never
                    # receives a gradient, even where the pad token occurs inside a sequence
                    g_x[pk.pad].zero_()
            elif packed:
                gemm(ggp, xp, G, In, rows, 1, 1, G, In, g_wih, In)
                gemm(ggp, w_ih, rows, In, G, 0, 1, G, In, gxp, In, beta=beta)
            else:
                gemm(gg, x, G, In, T * B, 1, 1, G, In, g_wih, In)
                gemm(gg, w_ih, T * B, In, G, 0, 1, G, In, g_x, In, beta=beta)
            g_w[4 * d:4 * d + 4] = [g_wih, g_whh, gb, gb.clone()]
            del ggp
        if packed and not layer0:
            _unpack(pk, gxp, g_x, In, In)
        return (g_x, None, None, *g_w)


def _pack(pk, tm, cols, ld, t0=0, t1=None, shift=0, out=None):
    """Live rows (t + shift, p), t in [t0, t1), p < bs_t, of the time-major buffer tm (row
    stride ld, first column at tm's pointer) -> a packed [rows, cols] tensor."""
    t1 = pk.T if t1 is None else t1
    offs, n = pk.live_offsets(t0, t1)
    if out is None:
        out = torch.empty((n, cols), dtype=torch.float32, device=tm.device)
    call("mvml_bilstm_pack_rows", n, t1 - t0, pk.B, cols, ptr(offs), t0, shift, ptr(tm), ld,
         ptr(out), out.stride(0), 0, _stream(tm.device))
    return out


def _unpack(pk, packed, tm, cols, ld):
    offs, n = pk.live_offsets(0, pk.T)
    call("mvml_bilstm_pack_rows", n, pk.T, pk.B, cols, ptr(offs), 0, 0, ptr(tm), ld, ptr(packed),
         packed.stride(0), 1, _stream(tm.device))


def _wide_step_ok(H):
    """mvml_bilstm_wide_fwd / _bwd take H % 8 == 0 (16-B rows of the interleaved W_hh image
    and of the cell epilogue); other hidden sizes run the per-step GEMM + cell kernels."""
    return H % 8 == 0


def _h_bounds(w, dev):
    """Split-fp16 maxima of the wide-batch recurrence: [bits of 1.0 (|h| = |o tanh c| < 1 bounds
    every recurrent operand row), max |W_hh| of the two directions]; None for other algos."""
    from . import functional as _F
    if _F.GEMM_ALGO != "f16x2":
        return None
    amx = torch.full((3,), 0x3F800000, dtype=torch.int32, device=dev)
    for d in range(2):
        wh = _c(w[4 * d + 1])
        absmax(wh, wh.shape[0], wh.shape[1], wh.shape[1], amx, 1 + d)
    return amx


class SelectLastFunction(torch.autograd.Function):
    """text_fea = [output[b, len_b - 1, :H] | output[b, 0, H:]] (model.py:131-133)."""

    @staticmethod
    def forward(ctx, out, pk):
        T, B, H2 = out.shape
        fea = torch.empty((B, H2), dtype=torch.float32, device=out.device)
        call("mvml_bilstm_select_last", B, H2 // 2, ptr(pk.lens), ptr(pk.pos), ptr(out), ptr(fea), 0,
             _stream(out.device))
        ctx.pk, ctx.shape = pk, out.shape
        return fea

    @staticmethod
    def backward(ctx, g_fea):
        T, B, H2 = ctx.shape
        g_out = torch.zeros((T, B, H2), dtype=torch.float32, device=g_fea.device)
        call("mvml_bilstm_select_last", B, H2 // 2, ptr(ctx.pk.lens), ptr(ctx.pk.pos), ptr(g_out),
             ptr(_c(g_fea)), 1, _stream(g_fea.device))
        return g_out, None


class _LSTMParams(nn.Module):
    """Parameter container with nn.LSTM's names and init (uniform +-1/sqrt(H))."""

    def __init__(self, input_size, hidden_size, num_layers, dropout):
        super().__init__()
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.dropout, self.bidirectional, self.batch_first = dropout, True, True
        for l in range(num_layers):
            In = input_size if l == 0 else 2 * hidden_size
            for sfx in ("", "_reverse"):
                self.register_parameter(f"weight_ih_l{l}{sfx}", nn.Parameter(torch.empty(4 * hidden_size, In)))
                self.register_parameter(f"weight_hh_l{l}{sfx}", nn.Parameter(torch.empty(4 * hidden_size, hidden_size)))
                self.register_parameter(f"bias_ih_l{l}{sfx}", nn.Parameter(torch.empty(4 * hidden_size)))
                self.register_parameter(f"bias_hh_l{l}{sfx}", nn.Parameter(torch.empty(4 * hidden_size)))
        stdv = 1.0 / math.sqrt(hidden_size)
        for p in self.parameters():
            nn.init.uniform_(p, -stdv, stdv)

    def layer_weights(self, l):
        return [getattr(self, f"{n}_l{l}{sfx}") for sfx in ("", "_reverse")
                for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]


class RNNModule(nn.Module):
    """model.py:98-135 (bidirectional only, as MVP builds it, model.py:25)."""

    def __init__(self, vocab, embed_dim, blstm_dim, num_layers, out_dim=2, dropout=0.2,
                 bidirectional=True, device='cpu'):
        super().__init__()
        if not bidirectional:
            raise NotImplementedError("MVP builds RNNModule bidirectional (model.py:25)")
        self.vocab, self.embed_dim, self.blstm_dim = vocab, embed_dim, blstm_dim
        self.hidden_size, self.num_layers, self.out_dim = blstm_dim, num_layers, out_dim
        self.bidirectional, self.device, self.num_dir = True, device, 2
        self.embeddings = nn.Embedding(vocab.tokens_length, embed_dim, padding_idx=vocab.pad)
        self.rnn = _LSTMParams(embed_dim, blstm_dim, num_layers, dropout)
        self.drop = nn.Dropout(p=dropout)
        self.norm_layer = nn.LayerNorm(2 * blstm_dim)  # built but unused by forward (model.py:120)
        self.fc = nn.Sequential(nn.Linear(2 * blstm_dim, out_dim), nn.ReLU(), nn.Dropout(p=dropout))

    def forward(self, batch):
        tokens = batch["smiles"]
        dev = self.embeddings.weight.device
        if tokens.device != dev:
            tokens = tokens.to(dev)
        pk = Packing(batch["seq_len"], tokens, self.vocab.tokens_length, self.embeddings.padding_idx)
        x = self.embeddings.weight
        for l in range(self.num_layers):
            x = BiLSTMLayerFunction.apply(x, pk, l == 0, *self.rnn.layer_weights(l))
            if l + 1 < self.num_layers and self.training and self.rnn.dropout > 0:
                x = nn.functional.dropout(x, self.rnn.dropout, True)  # nn.LSTM inter-layer dropout
        fea = SelectLastFunction.apply(x, pk)
        return LinearReLUFunction.apply(fea, self.fc[0].weight, self.fc[0].bias, _F.dropout_p(self.fc[2]))
