"""torch.autograd.Functions over the HIP kernels of libmvml_gat.so.

Each Function owns one stage of GNNModule (model.py:89-95) and calls only the C ABI; there is
no PyTorch math on the hot path besides allocation (and nn.Dropout, which the reference
applies with torch's own RNG, model.py:87).
"""
import contextlib
import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr

MODE_FLATTEN_ELU, MODE_MEAN, MODE_FLATTEN = 0, 1, 2


def _check_cuda_f32(t, name):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA (HIP) tensor: the mvml_gat path has no CPU fallback")
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32, got {t.dtype}")


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def _stream(dev):
    return _lib.stream_ptr(dev)


_UNIT_SEGMENT = {}


def _unit_segment(dev):
    """int64 [0, 1] on `dev` (made once): the offsets of one one-element segment."""
    t = _UNIT_SEGMENT.get(str(dev))
    if t is None:
        t = _UNIT_SEGMENT[str(dev)] = torch.tensor([0, 1], dtype=torch.int64, device=dev)
    return t


def zeros(shape, dtype=torch.float32, device=None):
    """torch.zeros through mvml_fill_zero (hipMemsetAsync): no framework fill kernel in the step."""
    t = torch.empty(shape, dtype=dtype, device=device)
    zero_(t)
    return t


def zero_(t):
    """Zero a contiguous tensor, or a 2-D row-pitched one (unit column stride), in place."""
    es = t.element_size()
    if t.is_contiguous():
        n = t.numel() * es
        call("mvml_fill_zero", ptr(t), 1, n, n, _stream(t.device))
    else:
        if t.dim() != 2 or t.stride(1) != 1:
            raise ValueError("zero_: contiguous or 2-D row-pitched tensors only")
        call("mvml_fill_zero", ptr(t), t.shape[0], t.shape[1] * es, t.stride(0) * es, _stream(t.device))
    return t


def copy2d(dst, src):
    """dst[:] = src for float32 2-D views with unit column stride (1-D: one row); a src row
    stride of 0 (an expanded row) replicates it (mvml_copy_cols)."""
    d2 = dst.view(1, -1) if dst.dim() == 1 else dst
    s2 = src.reshape(1, -1) if src.dim() == 1 else src
    if d2.shape != s2.shape or d2.stride(1) != 1 or (s2.shape[1] > 1 and s2.stride(1) != 1):
        raise ValueError("copy2d: matching 2-D views with unit column stride")
    call("mvml_copy_cols", d2.shape[0], d2.shape[1], ptr(s2), s2.stride(0) if s2.shape[0] > 1 else s2.shape[1],
         ptr(d2), d2.stride(0) if d2.shape[0] > 1 else d2.shape[1], _stream(dst.device))
    return dst


# Diagnostics hook (tools/diag_golden.py, the parity tests' kink-branch capture): when a dict,
# GATLayerFunction.forward appends each layer's el/er to DEBUG_CAPTURE["elr_fwd"] and the
# backward stores its saved el/er, attention and el/er gradients; LinearReLUFunction appends its
# post-ReLU output to ["relu_out"] and the fusion its Conv2d+ReLU output to ["conv_out"].  None
# in normal use.
DEBUG_CAPTURE = None


def _round4(x):
    return (x + 3) // 4 * 4


# Row pitch of the N-row projection / gradient matrices: a multiple of 64 floats, so every row
# starts on a 256-B boundary and the aggregation kernels' 64-column chunks (256-B row segments)
# never straddle an extra cache line (MVML_ROW_PITCH64=0: multiples of 4 floats only)
_PITCH64 = os.environ.get("MVML_ROW_PITCH64", "1") != "0"


def _row_pitch(cols):
    return (cols + 63) // 64 * 64 if _PITCH64 else _round4(cols)


def agg_fwd_bytes(N, E, H, F, out_cols, res_cols):
    """Algorithmic HBM bytes of one mvml_gat_agg_fwd: read Z and R once,
    rowptr, src ids, el/er; write the layer output and the saved attention.  R is the
    head-mean residual (F columns) in mean mode."""
    return 4 * (N * H * F + N * res_cols + 2 * N * H + (N + 1) + E + N * out_cols + E * H)


def agg_bwd_bytes(N, E, H, F, gout_cols, mode):
    """Algorithmic bytes of mvml_gat_agg_bwd: read Z, el/er, g_out (+ out for ELU'), the saved
    attention, both CSRs; write gY = [dZ_agg | dR | d el | d er]."""
    rw = F if mode == MODE_MEAN else H * F
    reads = N * H * F + 2 * N * H + N * gout_cols + (N * H * F if mode == 0 else 0) + E * H
    idx = 2 * (N + 1) + 3 * E
    writes = N * (H * F + rw + 2 * H)
    return 4 * (reads + idx + writes)


# GEMM algorithm for every dense product of the view: "f16x2" = scaled split-fp16 MFMA at fp32
# accuracy (mvml_gemm_f16x2, the default; 3 fp16 MFMAs per product), "x3" = split-bf16
# (mvml_gemm_f32x3, 6 bf16 MFMAs), "f32" = f32-input MFMA (mvml_gemm_f32).  All are parity-
# tested against fp64 at the fp32 bar; override with MVML_GEMM_ALGO=x3 / f32.
GEMM_ALGO = os.environ.get("MVML_GEMM_ALGO", "f16x2")
_GEMM_ENTRY = {"f32": ("mvml_gemm_f32", 0), "x3": ("mvml_gemm_f32x3", 1),
               "bf16": ("mvml_gemm_bf16", 2),  # bf16: the projection option of config 4
               "f16x2": ("mvml_gemm_f16x2", 3)}


def known_amax(X):
    """(int32 tensor, slot) holding max |X| bits if the kernel that produced X folded it into
    its stores, else None.  X._mvml_amax is set by the producer on the exact tensor it wrote;
    the record is trusted only while that tensor is unmodified by torch (same _version) and
    still is the storage the producer wrote (same data pointer, shape and strides) — a view, a
    copy or an in-place update through autograd-visible ops gets a fresh |max| pass instead."""
    rec = getattr(X, "_mvml_amax", None)
    if rec is None or rec[2] != X._version or rec[3] != (X.data_ptr(), tuple(X.shape), X.stride()):
        return None
    return rec[0], rec[1]


# Per-row A maxima (mvml_gemm_f16x2_rows): the split-fp16 products whose A rows are atoms or
# molecules split every row with its own scale — per-row fp32 accuracy, and a row's result
# independent of the batch it is computed in (a shard gives bitwise its slice of the whole
# batch).  MVML_ROW_SCALES=0: one scale per operand (the round-3 path).
ROW_SCALES = os.environ.get("MVML_ROW_SCALES", "1") != "0"


def known_rows(X):
    """Per-row |max| bits of X (int32 [rows]) if its producer recorded them (same rule as
    known_amax), else None."""
    rec = getattr(X, "_mvml_rows", None)
    if rec is None or rec[1] != X._version or rec[2] != (X.data_ptr(), tuple(X.shape), X.stride()):
        return None
    return rec[0]


def zero_padded(X, Fp):
    """The zero-padded [N, Fp] buffer X is the [:, :F] view of (batching.pad_columns: the
    batch's resident atom features), if unchanged since recorded, else None."""
    rec = getattr(X, "_mvml_padded", None)
    if rec is None or rec[1] != X._version or rec[2] != (X.data_ptr(), tuple(X.shape), X.stride()):
        return None
    return rec[0] if rec[0].shape[1] == Fp else None


def fold_rows(out, rows):
    """Record that rows[r] holds max |out[r, :]| bits (written with out by its producer)."""
    out._mvml_rows = (rows, out._version, (out.data_ptr(), tuple(out.shape), out.stride()))


def absmax_rows(P, rows, cols, ld, out=None, offset=0, accumulate=False):
    """out[r] (int32 [rows]) = bits of max_c |P[r, offset + c]| (mvml_absmax_rows_f32)."""
    if out is None:
        out = torch.empty(max(rows, 1), dtype=torch.int32, device=P.device)
    pp = ctypes.c_void_p(ptr(P).value + 4 * offset)
    call("mvml_absmax_rows_f32", rows, cols, pp, ld, ptr(out), int(accumulate), _stream(P.device))
    return out


def row_maxima(X, rows, cols, ld):
    """Per-row |max| bits of a K-contiguous operand: its producer's record, else one pass."""
    r = known_rows(X)
    return r if r is not None else absmax_rows(X, rows, cols, ld)


def fold_amax(out, amx, slot_idx):
    """Record that out's |max| bits are in amx[slot_idx] (folded by the kernel that wrote out)."""
    out._mvml_amax = (amx, slot_idx, out._version, (out.data_ptr(), tuple(out.shape), out.stride()))


def absmax(P, rows, cols, ld, out, slot=0, offset=0, accumulate=False):
    """out[slot] (int32 tensor) = bits of max |P[r, offset + c]| (mvml_absmax_f32)."""
    pp = ctypes.c_void_p(ptr(P).value + 4 * offset)
    op = ctypes.c_void_p(ptr(out).value + 4 * slot)
    call("mvml_absmax_f32", rows, cols, pp, ld, op, int(accumulate), _stream(out.device))


def slot(t, i):
    """Device pointer to element i of an int32 maxima tensor (None passes through)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr() + 4 * i)


# split-fp16 projection: el / er as 2H extra GEMM columns against Wcat's A_l / A_r rows (True)
# or mvml_gat_proj_fwd's logit-partial epilogue over the Z tile (False)
PROJ_ELR_GEMM = os.environ.get("MVML_PROJ_ELR_GEMM", "1") != "0"

# Weights split ONCE per step into the interleaved-by-4 fp16 image (mvml_split_f16x2_il4) that
# the 256x256 split-fp16 tiles load in place of fp32 B: one 16-B load per piece as before and no
# split VALU for B (bitwise the in-kernel split).  MVML_BSPLIT_IL=0: every tile splits B itself.
BSPLIT_IL = os.environ.get("MVML_BSPLIT_IL", "1") != "0"


def split_il4(W, rows, cols, ld, amax_ptr):
    """W (fp32 [rows][ld]) as its interleaved split-fp16 image (same shape), or None when off,
    not the f16x2 algorithm, or not 16-B shaped."""
    if not BSPLIT_IL or GEMM_ALGO != "f16x2" or cols % 4 or ld % 4 or W.data_ptr() % 16:
        return None
    img = torch.empty((rows, ld), dtype=torch.float32, device=W.device)
    call("mvml_split_f16x2_il4", rows, cols, ptr(W), ld, amax_ptr, ptr(img), _stream(W.device))
    return img


def split_il8(P, rows, K, ld, kmajor=0, amax_ptr=None, rows_max=None, out=None):
    """P's il8 split-fp16 image (mvml_split_f16x2_il8) for mvml_gemm_f16x2_planes: fp32
    [rows][K rounded up to 32]; x[r][k] = P[r, k] (kmajor 0) or P[k, r] (kmajor 1: the image of
    P^T); scale from amax_ptr (operand-wide) or rows_max (per row, int32 [rows])."""
    kp = (K + 31) // 32 * 32
    if out is None:
        out = torch.empty((max(rows, 1), kp), dtype=torch.float32, device=P.device)
    call("mvml_split_f16x2_il8", rows, K, ptr(P), ld, int(kmajor), amax_ptr, ptr(rows_max), ptr(out), kp,
         _stream(P.device))
    return out


def gemm_planes(A, M, N, K, lda, bimg, ldb, C, ldc, amax_b, amax_a=None, arows=None, a_image=False,
                bias=None, beta=0.0, act=0, role=None):
    """C[M,N] = act(A B^T + bias + beta C) with B given as its il8 image (split_il8, made with
    amax_b) and A fp32 (or, a_image, its il8 image made with the same maxima): the LDS-DMA
    split-fp16 tile (mvml_gemm_f16x2_planes).  amax_a: pointer to max |A| bits, or arows: per-row
    |A| max bits (int32 [M])."""
    _lib.call_tag[0] = {"flops": 2 * M * N * K, "shape": (M, N, K, 0, 0),
                        "bytes": 4 * (M * N + M * K + N * K), "role": role}
    call("mvml_gemm_f16x2_planes", M, N, K, ptr(A), lda, int(a_image), amax_a, ptr(arows), ptr(bimg), ldb,
         amax_b, ptr(bias), float(beta), int(act), ptr(C), ldc, _stream(C.device))


def gemm(A, B, M, N, K, a_kmajor, b_kmajor, lda, ldb, C, ldc, bias=None, beta=0.0, act=0, algo=None,
         amax=None, arows=None, bil4=None, role=None):
    """C[M,N] = act(A*B + bias + beta*C) on MFMA (see mvml_gemm_f32 / mvml_gemm_f32x3 /
    mvml_gemm_f16x2).  amax = (pointer to |A| max bits, pointer to |B| max bits) from absmax()
    lets split-fp16 products that share an operand share its max pass.  arows (split-fp16,
    K-contiguous A): per-row |A| max bits (int32 [M]) — every A row gets its own scale
    (mvml_gemm_f16x2_rows); amax then only needs B's pointer.  bil4: B's interleaved split
    image (split_il4, made with amax[1])."""
    # bytes: what the product must move at least (A, B and C once) — the small-K products
    # (layer 1's projection) are reported against HBM with it (bench.py roofline_proj_l1)
    _lib.call_tag[0] = {"flops": 2 * M * N * K, "shape": (M, N, K, int(a_kmajor), int(b_kmajor)),
                        "bytes": 4 * (M * N + M * K + N * K), "role": role}
    L = _lib.lib()
    dev = C.device
    wsz = L.mvml_gemm_workspace_size(M, N, K)
    wp, wn = _lib.ws_ptr_size(wsz, dev)
    algo = algo or GEMM_ALGO
    if algo == "f16x2" and arows is not None:
        if a_kmajor or amax is None or amax[1] is None:
            raise ValueError("gemm: per-row A maxima need a K-contiguous A and max |B|")
        # which kernel runs (the small-K memory kernel or the tile): bench.py files the timing
        # under the matching roofline
        fn = getattr(L, "mvml_gemm_rows_smallk", None)  # (absent from older libraries of A/B runs)
        sk = fn(int(b_kmajor), M, N, K, ptr(A), lda, ptr(bil4 if bil4 is not None else B), ldb, float(beta),
                int(act), ptr(C), ldc) if fn is not None else 0
        _lib.call_tag[0]["path"] = "smallk" if sk else "tile"
        call("mvml_gemm_f16x2_rows", M, N, K, ptr(A), lda, ptr(B), ldb, int(b_kmajor), ptr(bil4),
             ptr(arows), amax[1], ptr(bias), float(beta), int(act), ptr(C), ldc, wp, wn, _stream(dev))
        return
    if algo == "f16x2" and amax is not None and bil4 is not None:
        call("mvml_gemm_f16x2_bsplit", int(a_kmajor), int(b_kmajor), M, N, K, ptr(A), lda, ptr(B), ldb,
             ptr(bil4), 0, amax[0], amax[1], ptr(bias), float(beta), int(act), ptr(C), ldc, wp, wn,
             _stream(dev))
        return
    if algo == "f16x2" and amax is not None:
        call("mvml_gemm_f16x2_amax", int(a_kmajor), int(b_kmajor), M, N, K, ptr(A), lda, ptr(B), ldb,
             amax[0], amax[1], ptr(bias), float(beta), int(act), ptr(C), ldc, wp, wn, _stream(dev))
        return
    call(_GEMM_ENTRY[algo][0], int(a_kmajor), int(b_kmajor), M, N, K, ptr(A), lda,
         ptr(B), ldb, ptr(bias), float(beta), int(act), ptr(C), ldc, wp, wn, _stream(dev))


def gemm_batched(A, B, M, N, K, a_kmajor, b_kmajor, lda, ldb, C, ldc, batch, sa, sb, sc, beta=0.0):
    """C_z = A_z * B_z (+ beta C_z) for z < batch, operands at float strides sa / sb / sc
    (mvml_gemm_f32x3_batched: fp32-accurate split-bf16 MFMA, no split-K)."""
    _lib.call_tag[0] = {"flops": 2 * M * N * K * batch, "shape": (M, N, K, int(a_kmajor), int(b_kmajor), batch)}
    call("mvml_gemm_f32x3_batched", int(a_kmajor), int(b_kmajor), M, N, K, batch, ptr(A), lda, sa,
         ptr(B), ldb, sb, None, float(beta), 0, ptr(C), ldc, sc, _stream(C.device))


def colsum(X, M, N, ldx, out, beta=0.0, offset=0, alpha=1.0):
    """out = beta*out + alpha * column sums of X[:, offset:offset+N] (deterministic)."""
    L = _lib.lib()
    dev = out.device
    wp, wn = _lib.ws_ptr_size(L.mvml_colsum_workspace_size(M, N), dev)
    xp = ctypes.c_void_p(ptr(X).value + 4 * offset)
    call("mvml_colsum_f32", M, N, xp, ldx, float(alpha), float(beta), ptr(out), wp, wn, _stream(dev))


# Kernel paths picked per call from the batch's molecule sizes (host counts, no device work):
# "large" batches have half their atoms or more in molecules past the LDS molecule window
# (FLAT_SRC_MIN_ATOMS, gat_agg.hip kWinL) — BASELINE config 5.
#  * Aggregation forward by destination wave (one wave per atom gathers whole projection rows
#    from L2; csrc/gat_agg.hip gat_agg_fwd_dst_kernel), every layer (MVML_DST_FWD_POLICY = all |
#    auto: the head-mean layer on large batches only | off): on small-molecule batches with the
#    edge softmax as its own launch first (dst_fwd = 2: 2.9 / 3.4 ms against the molecule
#    window's 3.5 / 3.7 at config 3), on large ones inside the wave (dst_fwd = 1: 4.5 / 6.2 ms
#    against 5.0 / 6.4 split, config 5) — MVML_DST_FWD_KIND forces one.
#  * Flatten layers' aggregation backward by source atom in one pass (option flat_src = 2,
#    gat_flat_bwd_src1_kernel) on large batches (MVML_FLAT_SRC_AUTO = 0 turns it off).
FLAT_SRC_AUTO = os.environ.get("MVML_FLAT_SRC_AUTO", "1") == "1"
FLAT_SRC_MIN_ATOMS = 128  # the LDS molecule window (gat_agg.hip kWinL)
DST_FWD_POLICY = os.environ.get("MVML_DST_FWD_POLICY", "all")
DST_FWD_KIND = int(os.environ.get("MVML_DST_FWD_KIND", "0"))  # 0: by batch (see above)
#  * The ELU link (EluLink, below): the second layer's data-gradient GEMM applies ELU' in its
#    epilogue, so the first layer's backward gathers g_rst rows only (no `out` rows) — on large
#    batches, where that backward gathers rows per out-edge (flat_src); on small ones the
#    epilogue's extra read costs more than the molecule window saves (MVML_ELU_LINK = auto | on
#    | off).
ELU_LINK_POLICY = os.environ.get("MVML_ELU_LINK", "auto")


def _large_batch(g):
    return g.large_molecule_fraction(FLAT_SRC_MIN_ATOMS) >= 0.5


def _fwd_path(g, mode):
    """Context manager selecting the aggregation forward kernel path for this call."""
    dst = DST_FWD_POLICY == "all" or (DST_FWD_POLICY == "auto" and (mode != MODE_MEAN or _large_batch(g)))
    if not dst:
        return contextlib.nullcontext()
    return _lib.option("dst_fwd", DST_FWD_KIND or (1 if _large_batch(g) else 2))




class EluLink:
    """Fused ELU backward between two GAT layers of one GAT stack (mvml_gat.nn.GAT): the
    flatten + ELU layer's output records a link; the next layer's forward claims it, and its
    data-gradient GEMM then multiplies by ELU'(out) in its epilogue (act 3) and folds max |g|,
    so the first layer receives g_rst itself (no g_out * ELU' pass over N x H F).  The first
    layer's backward checks that the gradient it receives IS the one the claiming layer wrote."""

    __slots__ = ("claimed", "g_rst", "amax")

    def __init__(self, dev):
        self.claimed = False
        self.g_rst = None
        self.amax = zeros(1, dtype=torch.int32, device=dev)


# set by mvml_gat.nn.GAT.forward around its layer loop: links are made and claimed only there,
# where a flatten + ELU layer's output feeds exactly the next layer
ELU_LINK = [False]


def _elu_link_of(X):
    rec = getattr(X, "_mvml_elu", None)
    if rec is None or rec[1] != X._version or rec[2] != (X.data_ptr(), tuple(X.shape), X.stride()):
        return None
    return rec[0]


class GATLayerFunction(torch.autograd.Function):
    """dgllife GATLayer(GATConv) forward/backward (model.py:79-81): projection GEMM (fc and
    res_fc as one MFMA GEMM) + fused el/er, edge-softmax, aggregation, residual, bias and
    flatten/ELU or head-mean kernel."""

    @staticmethod
    def forward(ctx, X, fc_w, res_w, attn_l, attn_r, bias, g, H, F, slope, mode, algo=None):
        for t, n in ((X, "feat"), (fc_w, "fc.weight"), (res_w, "res_fc.weight")):
            _check_cuda_f32(t, n)
        # the batch's atom features may already sit in a zero-padded 16-B-row buffer
        Xpad = zero_padded(X, _round4(X.shape[1])) if X.dim() == 2 else None
        if Xpad is None:
            X = _c(X)
        N, Fin = X.shape
        dev = X.device
        HF = H * F
        mean_res = int(mode == MODE_MEAN)
        C = _lib.lib().mvml_gat_proj_cols(H, F, mean_res)
        st = _stream(dev)
        # Pad the feature dimension to a multiple of 4 (e.g. 74 atom features -> 76) so every
        # GEMM operand row is 16-B aligned and the LDS-DMA path applies; pad columns are zero.
        # (A ones pad column that would make the dW GEMM emit the bias gradient as well was
        # measured 1.02e-5 from float64 on config 3 — the bias sums cancel and the split-fp16
        # representation error shows — so the bias keeps its exact fp32 column sum.)
        Fp = _round4(Fin)
        if Xpad is not None:
            Xp = Xpad
        else:
            Xp = X if Fp == Fin else torch.nn.functional.pad(X, (0, Fp - Fin))
        attn_l, attn_r = _c(attn_l), _c(attn_r)
        HFa = attn_l.numel()
        attn_lr = torch.empty(2 * HFa, dtype=torch.float32, device=X.device)
        copy2d(attn_lr[:HFa], attn_l.reshape(-1))
        copy2d(attn_lr[HFa:], attn_r.reshape(-1))
        ctx.elu_claim = None
        link = _elu_link_of(X) if (ELU_LINK[0] and (algo or GEMM_ALGO) == "f16x2" and ROW_SCALES
                                   and PROJ_ELR_GEMM and X.requires_grad) else None
        # [fc.weight ; res_fc.weight (or its head mean) ; A_l ; A_r]: the projection GEMM uses
        # the first C rows, the backward all C + 2H (the el / er paths, see mvml_gat_agg_bwd)
        Wcat = torch.empty((C + 2 * H, Fp), dtype=torch.float32, device=dev)
        call("mvml_gat_fold_weights", ptr(_c(fc_w)), ptr(_c(res_w)), ptr(attn_lr), H, F, Fin, Fp,
             mean_res, ptr(Wcat), st)
        L = _lib.lib()
        # split-fp16: |max| of X, Wcat (all C + 2H rows) and, in the backward, gY — each operand's
        # pass serves all of its products (projection, dL/dW, dL/dX)
        amx = None
        ax = None  # (tensor, slot) of max |X|
        xr = None  # per-row max |X| bits (ROW_SCALES)
        wil = None  # Wcat's interleaved split image (BSPLIT_IL)
        if (algo or GEMM_ALGO) == "f16x2":
            amx = zeros(4, dtype=torch.int32, device=dev)  # [X, Wcat, gY (bwd), out]
            if ROW_SCALES and PROJ_ELR_GEMM:
                # the projection splits every atom row with its own scale; max |X| (the weight
                # gradient's A-side scale) is the max of the row maxima (N floats, not N x Fp).
                # Layer 1's rows are those of the resident atom features (the pad columns are
                # zeros): computed once and recorded on the feature tensor itself
                xr = known_rows(X)
                if xr is None:
                    # Xp's pad columns are zeros: the whole padded row (float4 loads) has the
                    # same |max| as its Fin features
                    xr = absmax_rows(Xp, N, Fp, Fp)
                    if not X.requires_grad:
                        fold_rows(X, xr)
                absmax(xr, N, 1, 1, amx, 0)
                ax = (amx, 0)
            else:
                ax = known_amax(Xp) if Xp is X else None  # layer 2: folded by layer 1's aggregation
            if ax is None:
                absmax(Xp, N, Fp, Fp, amx, 0)
                ax = (amx, 0)
            absmax(Wcat, C + 2 * H, Fp, Fp, amx, 1)
            # Wcat split once: the projection's tiles and the backward's dL/dX read the image
            wil = split_il4(Wcat, C + 2 * H, Fp, Fp, slot(amx, 1))
        # claim the previous layer's ELU link only where the fused data-gradient product will
        # run (per-row scales and the interleaved weight image: see backward)
        if (link is not None and not link.claimed and Fp == Fin and amx is not None
                and wil is not None):
            link.claimed = True
            ctx.elu_claim = link
        bf16_elr = (algo or GEMM_ALGO) == "bf16" and PROJ_ELR_GEMM
        if (amx is not None or bf16_elr) and PROJ_ELR_GEMM:
            # el / er as 2H more GEMM columns: X [A_l ; A_r]^T with A_l[h] = sum_f attn_l[h, f]
            # fc.weight[h F + f] (Wcat's last 2H rows) — the same values re-associated, no
            # logit-partial epilogue and no finalize pass; then gathered into elr [N, 2H].  The
            # bf16 projection (config 4) takes the same path on the bf16-operand kernel: its C
            # tile leaves through the LDS epilogue instead of the logit-partial one's column
            # stores (9.5 -> ~5 ms per config-3 layer-2 launch)
            ldy = _row_pitch(C + 2 * H)
            Y = torch.empty((N, ldy), dtype=torch.float32, device=dev)
            if xr is not None:
                gemm(Xp, Wcat, N, C + 2 * H, Fp, 0, 0, Fp, Fp, Y, ldy, amax=(None, slot(amx, 1)),
                     arows=xr, bil4=wil, role="gat_proj")
            elif amx is not None:
                gemm(Xp, Wcat, N, C + 2 * H, Fp, 0, 0, Fp, Fp, Y, ldy, amax=(slot(*ax), slot(amx, 1)))
            else:
                gemm(Xp, Wcat, N, C + 2 * H, Fp, 0, 0, Fp, Fp, Y, ldy, algo="bf16")
            # (a native slice copy: torch's strided copy splits into 32-bit-indexable pieces,
            # 8 launches for a 1.75 M-atom batch)
            elr = torch.empty((N, 2 * H), dtype=torch.float32, device=dev)
            call("mvml_copy_cols", N, 2 * H, ptr(Y[:, C:]), ldy, ptr(elr), 2 * H, st)
        else:
            ldy = _row_pitch(C)
            Y = torch.empty((N, ldy), dtype=torch.float32, device=dev)
            elr = torch.empty((N, 2 * H), dtype=torch.float32, device=dev)
            wp, wn = _lib.ws_ptr_size(L.mvml_gat_proj_fwd_workspace_size(N, H, F), dev)
            _lib.call_tag[0] = {"flops": 2 * N * C * Fp}
            call("mvml_gat_proj_fwd", N, ptr(Xp), Fp, Fp, ptr(Wcat), Fp, ptr(attn_lr), H, F, mean_res,
                 _GEMM_ENTRY[algo or GEMM_ALGO][1], ptr(Y), ldy, ptr(elr),
                 None if ax is None else slot(*ax), slot(amx, 1), None, 0, wp, wn, st)
        out_cols = F if mode == MODE_MEAN else HF
        out = torch.empty((N, out_cols), dtype=torch.float32, device=dev)
        E = g.num_edges()
        attn = torch.empty((E, H), dtype=torch.float32, device=dev)
        # per-row max |out| for the consumer's per-row split-fp16 GEMMs (next layer, Set2Set)
        orows = torch.empty(max(N, 1), dtype=torch.int32, device=dev) if (amx is not None and ROW_SCALES) else None
        _lib.call_tag[0] = {"layer": f"H{H}xF{F}", "bytes": agg_fwd_bytes(N, E, H, F, out_cols, C - HF)}
        with _fwd_path(g, mode):
            call("mvml_gat_agg_fwd", N, ptr(g.node_groups), g.num_node_groups, ptr(g.in_rowptr),
                 ptr(g.in_src), ptr(Y), ldy, H, F, ptr(elr), ptr(_c(bias)), float(slope), int(mode),
                 ptr(out), ptr(attn), slot(amx, 3), ptr(orows), st)
        if amx is not None:  # max |out| for the consumer's split-fp16 GEMMs (next layer, Set2Set)
            fold_amax(out, amx, 3)
        if orows is not None:
            fold_rows(out, orows)
        # flatten + ELU inside a GAT stack: the next layer's data-gradient GEMM may apply ELU'
        # in its epilogue (EluLink), so this layer's backward receives g_rst and reads no `out`
        ctx.link = None
        if (mode == MODE_FLATTEN_ELU and ELU_LINK[0] and amx is not None and ROW_SCALES
                and PROJ_ELR_GEMM
                and (ELU_LINK_POLICY == "on" or (ELU_LINK_POLICY == "auto" and _large_batch(g)))):
            ctx.link = EluLink(dev)
            out._mvml_elu = (ctx.link, out._version, (out.data_ptr(), tuple(out.shape), out.stride()))
        if DEBUG_CAPTURE is not None:
            DEBUG_CAPTURE.setdefault("elr_fwd", []).append(elr.detach().clone())
        ctx.save_for_backward(Xp, Wcat, Y, attn, elr, out, attn_l, attn_r, attn_lr)
        ctx.Fin = Fin
        ctx.g, ctx.H, ctx.F, ctx.slope, ctx.mode, ctx.ldy = g, H, F, slope, mode, ldy
        ctx.algo = algo
        ctx.amx = amx
        ctx.ax = ax
        ctx.wil = wil
        return out

    @staticmethod
    def backward(ctx, g_out):
        Xp, Wcat, Y, attn, elr, out, attn_l, attn_r, attn_lr = ctx.saved_tensors
        g, H, F, mode, ldy = ctx.g, ctx.H, ctx.F, ctx.mode, ctx.ldy
        link = ctx.link
        if link is not None and link.claimed:
            # the next layer's data-gradient GEMM applied ELU' already: g_out IS g_rst, and the
            # aggregation backward runs as plain flatten (mode 2: no ELU', no read of `out`)
            gr = link.g_rst
            if gr is None or g_out.data_ptr() != gr.data_ptr() or g_out.shape != gr.shape \
                    or g_out.stride() != gr.stride():
                raise RuntimeError("GAT ELU link: the gradient reaching the first layer is not the one "
                                   "the next layer's fused ELU backward wrote (was its output also "
                                   "consumed elsewhere?)")
            mode = MODE_FLATTEN
        g_out = _c(g_out)
        N, Fp = Xp.shape
        Fin = ctx.Fin
        dev = Xp.device
        HF = H * F
        mean_res = int(mode == MODE_MEAN)
        L = _lib.lib()
        C = L.mvml_gat_proj_cols(H, F, mean_res)
        CE = C + 2 * H  # + [d el | d er]
        ldg = _row_pitch(CE)
        st = _stream(dev)
        gY = torch.empty((N, ldg), dtype=torch.float32, device=dev)
        if ctx.amx is not None:
            zero_(ctx.amx[2:3])  # max |gY| of THIS backward (a second one, retain_graph, refolds it)
        wp, wn = _lib.ws_ptr_size(L.mvml_gat_agg_bwd_workspace_size(g.num_edges(), H), dev)
        # per-row max |gY| for the data-gradient product's per-row scales (not needed by layer 1,
        # whose input gradient is not formed)
        flat_src = FLAT_SRC_AUTO and mode != MODE_MEAN and _large_batch(g)
        gyr = None
        if ctx.amx is not None and ROW_SCALES and (ctx.needs_input_grad[0] or flat_src):
            # (the source-atom kernels then form max |gY| from the row maxima: no per-block atomics)
            gyr = torch.empty(max(N, 1), dtype=torch.int32, device=dev)
        _lib.call_tag[0] = {"layer": f"H{H}xF{F}",
                            "bytes": agg_bwd_bytes(N, g.num_edges(), H, F, g_out.shape[1], mode)}
        with (_lib.option("flat_src", 2) if flat_src else contextlib.nullcontext()):
            call("mvml_gat_agg_bwd", N, ptr(g.node_groups), g.num_node_groups, ptr(g.in_rowptr),
                 ptr(g.in_src), ptr(g.out_rowptr), ptr(g.out_dst), ptr(g.out_inslot), ptr(Y), ldy,
                 ptr(elr), ptr(attn), ptr(out), ptr(g_out), H, F, float(ctx.slope), int(mode), ptr(gY),
                 ldg, slot(ctx.amx, 2), ptr(gyr), wp, wn, st)
        amx = ctx.amx  # slot 2 = max |gY|, folded in by mvml_gat_agg_bwd's stores
        if DEBUG_CAPTURE is not None and amx is not None:
            DEBUG_CAPTURE.setdefault("gy_amax", []).append((gY[:, :CE].clone(), amx[2:3].clone()))
            if gyr is not None:
                DEBUG_CAPTURE.setdefault("gy_rows", []).append(gyr.clone())
        # dL/d[Wcat ; A_l ; A_r] = gY^T X  (split-K over atoms); the bias gradient is the column
        # sums of gY's residual columns (g_rst; mean: g_out / H for every head), formed with it
        # where the product's own reads can (mvml_gemm_f16x2_amax_colsum: layer 1)
        gW = torch.empty((CE, Fp), dtype=torch.float32, device=dev)
        g_bias = torch.empty((HF,), dtype=torch.float32, device=dev)
        bias_done = False
        if amx is not None and (ctx.algo or GEMM_ALGO) == "f16x2" and COLSUM_FUSED and \
                L.mvml_gemm_colsum_fused(CE, Fp, N):
            sum_n = F if mean_res else HF
            _lib.call_tag[0] = {"flops": 2 * CE * Fp * N, "shape": (CE, Fp, N, 1, 1),
                                "bytes": 4 * (CE * Fp + CE * N + Fp * N), "role": "gat_dw"}
            wp, wn = _lib.ws_ptr_size(L.mvml_gemm_colsum_workspace_size(CE, Fp, N, sum_n), dev)
            call("mvml_gemm_f16x2_amax_colsum", CE, Fp, N, ptr(gY), ldg, ptr(Xp), Fp, slot(amx, 2),
                 slot(*ctx.ax), ptr(gW), Fp, HF, sum_n, 1.0 / H if mean_res else 1.0, ptr(g_bias), wp, wn, st)
            bias_done = True
        else:
            gemm(gY, Xp, CE, Fp, N, 1, 1, ldg, Fp, gW, Fp, algo=ctx.algo,
                 amax=None if amx is None else (slot(amx, 2), slot(*ctx.ax)), role="gat_dw")
        g_fc = torch.empty((HF, Fin), dtype=torch.float32, device=dev)
        g_res = torch.empty((HF, Fin), dtype=torch.float32, device=dev)
        call("mvml_gat_unfold_grads", ptr(gW), ptr(attn_lr), H, F, Fin, Fp, mean_res, ptr(g_fc),
             ptr(g_res), st)
        gelr = gY[:, C:CE]
        # dL/dattn_l[h, f] = sum_n d el[n, h] Z[n, h, f] = sum_k G_l[h, k] fc.weight[h F + f, k]
        # with G_l = [d el]^T X — rows C .. C+H of gW, already formed by the dW GEMM (and G_r
        # rows C+H ..): re-associated, a (2 x Fp) x (Fp x F) product per head instead of a pass
        # over the N x H F projection (mvml_gat_attn_grad, kept in the ABI)
        g_alr = torch.empty((2, HF), dtype=torch.float32, device=dev)
        gemm_batched(gW[C:], Wcat, 2, F, Fp, 0, 0, H * Fp, Fp, g_alr, HF, H, Fp, F * Fp, F)
        g_al = g_alr[0].view_as(attn_l)
        g_ar = g_alr[1].view_as(attn_r)
        if DEBUG_CAPTURE is not None:
            DEBUG_CAPTURE.update(elr=elr, gelr=gelr, attn=attn)
        if mean_res:  # every head's bias sees g_out / H: one column sum, replicated over heads
            if not bias_done:
                colsum(gY, N, F, ldg, g_bias, offset=HF, alpha=1.0 / H)
            copy2d(g_bias.view(H, F)[1:], g_bias[:F].view(1, F).expand(H - 1, F))
        elif not bias_done:
            colsum(gY, N, HF, ldg, g_bias, offset=HF)
        gX = None
        if ctx.needs_input_grad[0]:
            gX = torch.empty((N, Fin), dtype=torch.float32, device=dev)
            link = ctx.elu_claim
            if link is not None and amx is not None and ROW_SCALES and ctx.wil is not None:
                # the previous layer's ELU backward in this product's epilogue: gX leaves as its
                # g_rst, with max |g_rst| folded for its GEMMs (EluLink)
                zero_(link.amax)
                _lib.call_tag[0] = {"flops": 2 * N * Fin * CE, "shape": (N, Fin, CE, 0, 1)}
                call("mvml_gemm_f16x2_ex", N, Fin, CE, 1, ptr(gY), ldg, 0, ptr(Wcat), Fp, 1, ptr(ctx.wil),
                     0, ptr(gyr if gyr is not None else absmax_rows(gY, N, CE, ldg)), 0, slot(amx, 1),
                     None, 0, 3, ptr(gX), Fin, 0, ptr(Xp), Fp, ptr(link.amax), None, 0, 0, 0, st)
                link.g_rst = gX
            elif amx is not None and ROW_SCALES:  # every atom's gradient row at its own scale
                gemm(gY, Wcat, N, Fin, CE, 0, 1, ldg, Fp, gX, Fin, amax=(None, slot(amx, 1)),
                     arows=gyr if gyr is not None else absmax_rows(gY, N, CE, ldg), bil4=ctx.wil)
            else:
                gemm(gY, Wcat, N, Fin, CE, 0, 1, ldg, Fp, gX, Fin, algo=ctx.algo,
                     amax=None if amx is None else (slot(amx, 2), slot(amx, 1)))
        return gX, g_fc, g_res, g_al, g_ar, g_bias, None, None, None, None, None, None


# GAT layer weight + bias gradients from one read of gY where the product's plan allows
# (mvml_gemm_f16x2_amax_colsum); MVML_COLSUM_FUSED=0: the product, then a column-sum pass
COLSUM_FUSED = os.environ.get("MVML_COLSUM_FUSED", "1") != "0"


# Set2Set's gates GEMM + LSTM cell as one launch (mvml_lstm_gates_cell_fwd: the cell in the
# GEMM epilogue, interleaved weight rows) where the 256x256 plan applies; False: GEMM + cell
CELL_EPI = True


class Set2SetFunction(torch.autograd.Function):
    """dgl Set2Set.forward (model.py:92): n_iters x {n_layers LSTM cell steps, fused segment
    softmax readout}.  LSTM gates: one MFMA GEMM per cell over [x | h_prev] + pointwise kernel."""

    @staticmethod
    def forward(ctx, X, g, n_iters, n_layers, *lstm_params):
        _check_cuda_f32(X, "feat")
        X = _c(X)
        N, D = X.shape
        B = g.batch_size
        dev = X.device
        st = _stream(dev)
        T, Lr = n_iters, n_layers
        W = [tuple(_c(p) for p in lstm_params[4 * l:4 * l + 4]) for l in range(Lr)]  # w_ih, w_hh, b_ih, b_hh
        f32 = dict(dtype=torch.float32, device=dev)
        # Combined GEMM operands: XH[l][t] = [x_l(t) | h_l(t-1)] (kin_l + D columns) so each
        # cell's gates are ONE GEMM against [W_ih | W_hh]; layer 0's x is q*_{t-1}, so
        # XH[0][t+1][:, :2D] IS q*_t (the readout writes r_t there).  Each cell writes its h
        # twice: its own recurrence slot XH[l][t+1][:, kin:] and its consumer's input slot
        # (XH[l+1][t][:, :D], or q_t = XH[0][t+1][:, :D] for the top layer).
        kin = [2 * D] + [D] * (Lr - 1)
        XH = [torch.empty((T + 1, B, kin[l] + D), **f32) for l in range(Lr)]
        zero_(XH[0][0])
        for l in range(1, Lr):
            zero_(XH[l][0, :, D:])
        L = _lib.lib()
        # [W_ih | W_hh] and (cell epilogue) its interleaved rows: row 4 j + q = row q D + j (unit
        # j's i, f, g, o), both from one mvml_lstm_pack_weights launch per layer
        Wcat = [torch.empty((4 * D, kin[l] + D), **f32) for l in range(Lr)]
        Wperm = [torch.empty((4 * D, kin[l] + D), **f32) if CELL_EPI else None for l in range(Lr)]
        for l in range(Lr):
            call("mvml_lstm_pack_weights", D, kin[l], ptr(W[l][0]), ptr(W[l][1]), ptr(Wcat[l]), ptr(Wperm[l]), st)
        acts = torch.empty((T, Lr, B, 4 * D), **f32)
        cs = torch.empty((T, Lr, B, D), **f32)
        lse = torch.empty((T, B), **f32)
        gates = torch.empty((B, 4 * D), **f32)
        amax_x = amax_w = None
        mrows = None  # per-molecule bound of every cell's A row (ROW_SCALES)
        wsp = [(None, 0)] * Lr
        if GEMM_ALGO == "f16x2":
            # split-fp16 operand maxima of the cells' GEMMs: every A row [x | h_prev] holds
            # LSTM outputs h = o tanh(c) (|h| < 1) and, in layer 0, the readout r = sum_n a_n x_n
            # (a convex combination: |r| <= max |X|), so max(1, max |X|) bounds every cell's A
            # (an upper bound is all the scale needs) — one pass instead of one per cell
            kx = known_amax(X)  # folded by the last GAT layer's aggregation
            if kx is None:
                kx = (zeros(1, dtype=torch.int32, device=dev), 0)
                absmax(X, N, D, D, kx[0], 0, accumulate=True)
            # max(1, max |X|) on the float bits (non-negative: int order), one "segment" [0, 1)
            amax_x = torch.empty(1, dtype=torch.int32, device=dev)
            call("mvml_segment_max_bits", 1, ptr(_unit_segment(dev)), slot(*kx), 0x3F800000, ptr(amax_x), st)
            if ROW_SCALES:
                # per molecule: max(1, max |X| over its atoms) bounds every entry of its cell rows
                # [x | h] (h = o tanh c, the readout a convex combination of its own atoms' rows),
                # so a molecule's cells are split at a scale of its own
                xr = row_maxima(X, N, D, D)
                mrows = torch.empty(max(B, 1), dtype=torch.int32, device=dev)
                call("mvml_segment_max_bits", B, ptr(g.node_offsets), ptr(xr), 0x3F800000, ptr(mrows), st)
            amax_w = torch.empty(Lr, dtype=torch.int32, device=dev)
            for l in range(Lr):
                absmax(Wcat[l], 4 * D, kin[l] + D, kin[l] + D, amax_w, l)  # = Wperm's max
            # the gates' weights split once per forward into the interleaved image (the fused path
            # reads Wperm's, the unfused one Wcat's: the same values per element, so the same
            # products; w_plane = 0)
            wsp = [(split_il4(Wperm[l] if CELL_EPI else Wcat[l], 4 * D, kin[l] + D, kin[l] + D,
                              slot(amax_w, l)), 0) for l in range(Lr)]
        for t in range(T):
            for l in range(Lr):
                w_ih, w_hh, b_ih, b_hh = W[l]
                K = kin[l] + D if t > 0 else kin[l]  # h_l(-1) = 0: the recurrent half is skipped
                own = XH[l][t + 1][:, kin[l]:]
                nxt = XH[l + 1][t] if l < Lr - 1 else XH[0][t + 1]
                c_prev = cs[t - 1, l] if t > 0 else None
                ldn = kin[l + 1] + D if l < Lr - 1 else 3 * D
                if CELL_EPI and not (t == 0 and l == 0) and L.mvml_lstm_gates_cell_plan_ok(B, D, K):
                    pa = pw = None
                    if amax_x is not None:  # split-fp16: the operand maxima of this cell's GEMM
                        pa, pw = slot(amax_x, 0), slot(amax_w, l)
                    _lib.call_tag[0] = {"flops": 2 * B * 4 * D * K, "shape": (B, 4 * D, K, 0, 0, "cell")}
                    call("mvml_lstm_gates_cell_fwd", B, D, K, ptr(XH[l][t]), kin[l] + D, ptr(Wperm[l]),
                         kin[l] + D, ptr(b_ih), ptr(b_hh), ptr(c_prev), ptr(cs[t, l]), ptr(own),
                         kin[l] + D, ptr(acts[t, l]), ptr(nxt), ldn, pa, pw, ptr(mrows),
                         ptr(wsp[l][0]), wsp[l][1], st)
                    continue
                gp = gates
                if t == 0 and l == 0:
                    gp = None  # q*_{-1} = 0 and h_0(-1) = 0: zero pre-activations, the bias alone
                else:
                    gemm(XH[l][t], Wcat[l], B, 4 * D, K, 0, 0, kin[l] + D, kin[l] + D, gates, 4 * D,
                         amax=None if amax_x is None else (slot(amax_x, 0), slot(amax_w, l)),
                         arows=mrows,
                         bil4=wsp[l][0] if not CELL_EPI and wsp[l][1] == 0 else None)
                call("mvml_lstm_cell_fwd", B, D, ptr(gp), ptr(b_ih), ptr(b_hh), ptr(c_prev),
                     ptr(cs[t, l]), ptr(own), kin[l] + D, ptr(acts[t, l]), ptr(nxt), ldn, st)
            call("mvml_set2set_seg_fwd", B, D, ptr(g.node_offsets), ptr(X), ptr(XH[0][t + 1]), 3 * D,
                 ptr(lse[t]), st)
        ctx.save_for_backward(X, acts, cs, lse, *XH, *[p for w in W for p in w])
        ctx.g, ctx.T, ctx.Lr = g, T, Lr
        ctx.amax = (amax_x, amax_w)
        return copy2d(torch.empty((B, 2 * D), **f32), XH[0][T][:, :2 * D])

    @staticmethod
    def backward(ctx, g_out):
        X, acts, cs, lse, *rest = ctx.saved_tensors
        g, T, Lr = ctx.g, ctx.T, ctx.Lr
        XH, flat = rest[:Lr], rest[Lr:]
        W = [tuple(flat[4 * l:4 * l + 4]) for l in range(Lr)]
        qs = XH[0][1:]  # q*_t = XH[0][t+1][:, :2D], row stride 3D
        N, D = X.shape
        B = g.batch_size
        dev = X.device
        st = _stream(dev)
        f32 = dict(dtype=torch.float32, device=dev)
        # Recurrent data gradients as ONE GEMM per cell against [W_ih | W_hh] (4D x (kin+D)):
        # the outputs [dL/dx_l(t) | dL/dh_l(t-1)] land side by side — for layer 0 in the rows of
        # g_qs3[t-1] = [dL/dq*_{t-1} (2D) | dL/dh_0(t-1) (D)], for layers l > 0 in gxh[l] =
        # [dL/dh_{l-1}(t) | dL/dh_l(t-1)].  N = kin + D fills whole 256-column GEMM tiles
        # (768 / 1152) where two products of N = 384 would each waste a quarter of theirs.
        kins = [2 * D] + [D] * (Lr - 1)
        Wcat = [torch.empty((4 * D, kins[l] + D), **f32) for l in range(Lr)]
        for l in range(Lr):
            call("mvml_lstm_pack_weights", D, kins[l], ptr(W[l][0]), ptr(W[l][1]), ptr(Wcat[l]), None, st)
        g_qs3 = torch.empty((T, B, 3 * D), **f32)
        g_qstars = g_qs3[:, :, :2 * D]
        copy2d(g_qstars[T - 1], _c(g_out))
        alphas = torch.empty((T, N), **f32)
        g_es = torch.empty((T, N), **f32)
        gW_ih = [torch.empty_like(w[0]) for w in W]  # written below (one product per layer)
        gW_hh = [torch.empty_like(w[1]) for w in W]
        gb = [torch.empty_like(w[2]) for w in W]
        # every step's gate gradients are kept so that each weight gradient is ONE GEMM over
        # all T*B rows after the recurrence (K = 393k instead of 6 launches of 65k)
        g_gates_all = torch.empty((Lr, T, B, 4 * D), **f32)
        g_h = torch.empty((B, D), **f32)
        gxh = [None] + [torch.empty((B, 2 * D), **f32) for _ in range(1, Lr)]
        g_c = [torch.empty((B, D), **f32) for _ in range(Lr)]  # first read at t = T - 2 (None before)
        g_c_new = torch.empty((B, D), **f32)
        # LSTM bias gradients: every cell backward leaves [R, 4D] partial column sums of its
        # gate gradients (mvml_lstm_cell_bwd's gb_part); one column sum over the T R partial rows
        # per layer replaces a pass over all T B gate-gradient rows
        R = int(_lib.lib().mvml_lstm_cell_bwd_part_rows(B, D))
        gb_part = torch.empty((Lr, T, R, 4 * D), **f32)
        # split-fp16 maxima: the forward's bounds for XH (|x|, |h|) and [W_ih | W_hh], and a
        # running |max| of each layer's gate gradients, folded in by mvml_lstm_cell_bwd (the
        # running value bounds every cell seen so far, which is all a scale needs)
        amax_x, amax_w = ctx.amax
        amax_g = zeros(Lr, dtype=torch.int32, device=dev) if amax_x is not None else None
        wib = [None] * Lr  # [W_ih | W_hh] split once (interleaved image) for the per-cell data-gradient products
        if amax_g is not None:
            wib = [split_il4(Wcat[l], 4 * D, Wcat[l].shape[1], Wcat[l].shape[1], slot(amax_w, l))
                   for l in range(Lr)]
        for t in range(T - 1, -1, -1):
            # readout segment backward: dL/dq_t = g_qstar_t[:, :D] + segment term -> g_h
            call("mvml_set2set_seg_bwd", B, D, ptr(g.node_offsets), ptr(X), ptr(qs[t]), 3 * D,
                 ptr(lse[t]), ptr(g_qs3[t]), 3 * D, ptr(g_h), D, ptr(alphas[t]), ptr(g_es[t]), st)
            for l in range(Lr - 1, -1, -1):
                kin = 2 * D if l == 0 else D
                if l == Lr - 1:
                    gh, ldgh = g_h, D
                else:
                    gh, ldgh = gxh[l + 1][:, :D], 2 * D  # dL/dh_l(t) from layer l+1's input
                gh2, ldgh2 = None, 0
                if t < T - 1:  # + dL/dh_l(t) through the recurrence at step t+1 (summed in the kernel)
                    gh2, ldgh2 = (g_qs3[t][:, 2 * D:], 3 * D) if l == 0 else (gxh[l][:, D:], 2 * D)
                c_prev = cs[t - 1, l] if t > 0 else None
                g_gates = g_gates_all[l, t]
                call("mvml_lstm_cell_bwd", B, D, ptr(acts[t, l]), ptr(cs[t, l]), ptr(c_prev), ptr(gh), ldgh,
                     ptr(gh2), ldgh2,
                     ptr(g_c[l]) if t < T - 1 else None, ptr(g_gates), ptr(g_c_new), slot(amax_g, l),
                     ptr(gb_part[l, t]), st)
                g_c[l], g_c_new = g_c_new, g_c[l]
                # N = kin + D with the recurrent part (t > 0), kin alone at t = 0; layer 0 at
                # t = 0 has neither (its input q*_{-1} = 0 is a constant)
                ncols = kin + D if t > 0 else (kin if l > 0 else 0)
                if ncols:
                    out, ldo = (g_qs3[t - 1], 3 * D) if l == 0 else (gxh[l], 2 * D)
                    # (operand-wide scales here: GraphNorm's backward has already mixed each
                    # 64-molecule group's gradients, so the cells' rows span little)
                    gemm(g_gates, Wcat[l], B, ncols, 4 * D, 0, 1, 4 * D, kin + D, out, ldo,
                         amax=None if amax_g is None else (slot(amax_g, l), slot(amax_w, l)),
                         bil4=wib[l])
        # weight / bias gradients, one product per parameter over all steps:
        #   dW_ih[l] = sum_t g_gates[l,t]^T x_l(t),  dW_hh[l] = sum_{t>=1} g_gates[l,t]^T h_l(t-1)
        # (layer 0's input x_0(t) = q*_{t-1} is zero at t = 0; h_l(-1) = 0)
        # [dW_ih | dW_hh][l] = sum_t g_gates[l,t]^T XH[l][t] as ONE GEMM with N = kin + D: the
        # recurrent half of XH[l][0] is zero (h_l(-1) = 0) and for layer 0 the whole t = 0 block
        # is (q*_{-1} = 0), so it is skipped there.
        for l in range(Lr):
            G = g_gates_all[l]
            kin = 2 * D if l == 0 else D
            ldx = kin + D
            t0 = 1 if l == 0 else 0
            if T > t0:
                gWcat = torch.empty((4 * D, ldx), **f32)
                gemm(G[t0:], XH[l][t0:T], 4 * D, ldx, (T - t0) * B, 1, 1, 4 * D, ldx, gWcat, ldx,
                     amax=None if amax_g is None else (slot(amax_g, l), slot(amax_x, 0)))
                copy2d(gW_ih[l], gWcat[:, :kin])
                copy2d(gW_hh[l], gWcat[:, kin:])
            colsum(gb_part[l], T * R, 4 * D, 4 * D, gb[l])
        gX = torch.empty((N, D), **f32)
        call("mvml_set2set_gx", N, D, T, ptr(g.node_graph), ptr(g.node_offsets), B, ptr(qs), 3 * D, B * 3 * D,
             ptr(g_qs3), 3 * D, B * 3 * D, ptr(alphas), ptr(g_es), ptr(gX), st)
        grads = []
        for l in range(Lr):
            grads += [gW_ih[l], gW_hh[l], gb[l], copy2d(torch.empty_like(gb[l]), gb[l])]
        return (gX, None, None, None, *grads)


class GraphNormFunction(torch.autograd.Function):
    """torch_geometric GraphNorm.forward(x, batch=None) (model.py:93), per group."""

    @staticmethod
    def forward(ctx, x, weight, bias, mean_scale, group_offsets, eps):
        _check_cuda_f32(x, "x")
        x = _c(x)
        G = group_offsets.numel() - 1
        D = x.shape[1]
        y = torch.empty_like(x)
        call("mvml_graphnorm_fwd", G, D, ptr(group_offsets), ptr(x), ptr(_c(weight)), ptr(_c(bias)),
             ptr(_c(mean_scale)), float(eps), ptr(y), _stream(x.device))
        ctx.save_for_backward(x, weight, mean_scale, group_offsets)
        ctx.eps = eps
        return y

    @staticmethod
    def backward(ctx, g_y):
        x, weight, mean_scale, group_offsets = ctx.saved_tensors
        g_y = _c(g_y)
        G = group_offsets.numel() - 1
        D = x.shape[1]
        dev = x.device
        L = _lib.lib()
        gx = torch.empty_like(x)
        gw = torch.empty_like(weight)
        gb = torch.empty_like(weight)
        gms = torch.empty_like(weight)
        wp, wn = _lib.ws_ptr_size(L.mvml_graphnorm_bwd_workspace_size(G, D), dev)
        call("mvml_graphnorm_bwd", G, D, ptr(group_offsets), ptr(x), ptr(_c(weight)), ptr(_c(mean_scale)),
             float(ctx.eps), ptr(g_y), ptr(gx), ptr(gw), ptr(gb), ptr(gms), wp, wn, _stream(dev))
        return gx, gw, gb, gms, None, None


def linear_maxima(x, w):
    """Split-fp16 maxima of a Linear's three products: slots [x, w, grad] (x's from its
    producer when it folded one), one pass per operand instead of one per product, and (ROW_SCALES)
    x's per-row maxima for the forward product; None for the other algorithms."""
    if GEMM_ALGO != "f16x2":
        return None
    amx = zeros(3, dtype=torch.int32, device=x.device)
    xr = None
    if ROW_SCALES:
        xr = row_maxima(x, x.shape[0], x.shape[1], x.shape[1])
        absmax(xr, x.shape[0], 1, 1, amx, 0)
        kx = (amx, 0)
    else:
        kx = known_amax(x)
    if kx is None:
        absmax(x, x.shape[0], x.shape[1], x.shape[1], amx, 0)
        kx = (amx, 0)
    absmax(w, w.shape[0], w.shape[1], w.shape[1], amx, 1)
    return amx, kx, xr, split_il4(w, w.shape[0], w.shape[1], w.shape[1], slot(amx, 1))


def linear_fwd(x, weight, y, M, Nout, K, lm, bias=None, act=0):
    """y = act(x W^T + b): the forward product of a Linear (per-row x scales when lm has them)."""
    if lm is not None and lm[2] is not None:
        gemm(x, weight, M, Nout, K, 0, 0, K, K, y, Nout, bias=bias, act=act, amax=(None, slot(lm[0], 1)),
             arows=lm[2], bil4=lm[3])
    else:
        gemm(x, weight, M, Nout, K, 0, 0, K, K, y, Nout, bias=bias, act=act,
             amax=None if lm is None else (slot(*lm[1]), slot(lm[0], 1)),
             bil4=None if lm is None else lm[3])


def linear_dx(g, weight, gx, M, Nout, K, lm):
    """gx = g W (the data gradient of a Linear; per-row g scales under ROW_SCALES)."""
    if lm is not None and lm[2] is not None:
        gemm(g, weight, M, K, Nout, 0, 1, Nout, K, gx, K, amax=(None, slot(lm[0], 1)),
             arows=absmax_rows(g, M, Nout, Nout), bil4=lm[3])
    else:
        gemm(g, weight, M, K, Nout, 0, 1, Nout, K, gx, K,
             amax=None if lm is None else (slot(lm[0], 2), slot(lm[0], 1)),
             bil4=None if lm is None else lm[3])


def dropout_seed():
    """A seed for mvml_dropout_fwd from torch's default (CPU) generator: reproducible under
    torch.manual_seed like nn.Dropout's draws, and no device round trip."""
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


def dropout_p(module):
    """The probability an nn.Dropout module applies now (0 in eval mode)."""
    return float(module.p) if module.training and module.p > 0 else 0.0


def relu_dropout_(y, p):
    """nn.Dropout(p) in place on a ReLU output y (mvml_dropout_fwd); returns the backward's
    scale 1 / (1 - p) (1.0 for p == 0: nothing launched)."""
    if p <= 0.0:
        return 1.0
    if p >= 1.0:
        raise ValueError("dropout probability must be < 1 on the HIP path")
    call("mvml_dropout_fwd", y.numel(), ptr(y), ptr(y), float(p), dropout_seed(), _stream(y.device))
    return float(np.float32(1.0 / (1.0 - p)))  # the float the kernel multiplied by


class LinearReLUFunction(torch.autograd.Function):
    """nn.Linear + nn.ReLU of GNNModule.fc (model.py:86-87) as one MFMA GEMM with a bias+ReLU
    epilogue, and the nn.Dropout(p) that follows it (model.py:87; p = 0: none) applied in place
    on the ReLU output: the backward then needs no mask (mvml_relu_bwd's scaled form)."""

    @staticmethod
    def forward(ctx, x, weight, bias, p=0.0):
        _check_cuda_f32(x, "x")
        x = _c(x)
        M, K = x.shape
        Nout = weight.shape[0]
        y = torch.empty((M, Nout), dtype=torch.float32, device=x.device)
        weight = _c(weight)
        lm = ctx.lm = linear_maxima(x, weight)
        linear_fwd(x, weight, y, M, Nout, K, lm, bias=_c(bias), act=1)
        if DEBUG_CAPTURE is not None:  # the ReLU sides the product took (parity tests)
            DEBUG_CAPTURE.setdefault("relu_out", []).append(y.detach().clone())
        ctx.scale = relu_dropout_(y, p)
        ctx.save_for_backward(x, weight, y)
        return y

    @staticmethod
    def backward(ctx, g_y):
        x, weight, y = ctx.saved_tensors
        g_y = _c(g_y)
        M, K = x.shape
        Nout = weight.shape[0]
        dev = x.device
        g_pre = torch.empty_like(y)
        call("mvml_relu_bwd", y.numel(), ptr(y), ptr(g_y), ptr(g_pre), float(ctx.scale), _stream(dev))
        lm = ctx.lm
        if lm is not None:
            absmax(g_pre, M, Nout, Nout, lm[0], 2)
        gw = torch.empty_like(weight)
        gemm(g_pre, x, Nout, K, M, 1, 1, Nout, K, gw, K,
             amax=None if lm is None else (slot(lm[0], 2), slot(*lm[1])))
        gb = torch.empty((Nout,), dtype=torch.float32, device=dev)
        colsum(g_pre, M, Nout, Nout, gb)
        gx = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            linear_dx(g_pre, weight, gx, M, Nout, K, lm)
        return gx, gw, gb, None
