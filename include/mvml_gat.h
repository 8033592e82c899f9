/*
 * mvml_gat.h — C ABI of the MI355X-native molecular-graph (GAT) view of MVML-MPI.
 *
 * The reference's hot path is GNNModule (model.py:77-95): dgllife GAT (model.py:81,91)
 * -> dgl Set2Set (model.py:82-84,92) -> PyG GraphNorm, batch=None (model.py:85,93) ->
 * Linear+ReLU+Dropout (model.py:86-87,94), fed by dgl.batch (dataset.py:52-54) over
 * mol_to_bigraph(add_self_loop=True) graphs (dataset.py:33-35).  The reference has no FFI of
 * its own: its operator API is the PyTorch nn.Module API, and the native code it runs is
 * DGL's C kernels (_CAPI_DGLKernelSpMM / SDDMM / EdgeSoftmax, dgl 0.9.1), torch_scatter
 * (GraphNorm) and cuBLAS/MKL (Linear, LSTM).  Each entry point below names the reference
 * operation it replaces; the Python package mvml_gat binds them with ctypes (see
 * INTEGRATION.md) behind the reference's nn.Module signatures.
 *
 * Conventions (all entry points):
 *  - every pointer is a DEVICE pointer owned by the caller (PyTorch caching allocator);
 *    the library never allocates or frees device memory.  Scratch comes from a caller-sized
 *    `workspace` (query the matching *_workspace_size function).
 *  - `stream` is a hipStream_t passed as void* (NULL = legacy default stream); every call
 *    only enqueues work on it: no host synchronisation, no allocation, graph-capturable.
 *  - row-major fp32 tensors; `ld*` are leading dimensions in elements; indices int32 unless
 *    stated (node/edge offsets int64, as dgl's batch_num_nodes/edges).
 *  - return 0 on success, nonzero MVML_ERR_* on failure; mvml_last_error() then describes it.
 *  - deterministic: no floating-point atomics anywhere, results are bitwise reproducible.
 */
#ifndef MVML_GAT_H
#define MVML_GAT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MVML_OK 0
#define MVML_ERR_INVALID 1   /* bad argument / unsupported shape */
#define MVML_ERR_LAUNCH 2    /* HIP launch or runtime error */
#define MVML_ERR_WORKSPACE 3 /* workspace too small */

/* Human-readable description of the last error on the calling thread ("" if none). */
const char* mvml_last_error(void);
/* Library version string, and the gfx target the kernels were built for. */
const char* mvml_version(void);

/* Kernel-path options, for tests and tools (the defaults are the production paths; every path
 * computes the same function and is parity-tested).  Each starts from the environment variable
 * named below, read ONCE when the library loads, and changes at run time only through
 * mvml_set_option, which returns the previous value (-1: unknown option, nothing changed).
 * Process-wide; set them between launches, not while another thread enqueues work. */
#define MVML_OPT_BIG_WINDOW 0   /* MVML_BIG_WINDOW: 1 (default) big-window aggregation kernels for
                                   groups past the molecule window, 0 = per-atom fallbacks */
#define MVML_OPT_BWD_ATOMWISE 1 /* MVML_BWD_ATOMWISE: 1 = aggregation backward by the per-atom
                                   dst / src kernel pair for every group (default 0) */
#define MVML_OPT_GEMM_TILE 2    /* MVML_X3_TILE: 0 (default) planned tile, 128 / 256 = forced */
#define MVML_OPT_GEMM_PERSIST 3 /* MVML_X3W_PERSIST: P > 0 caps a 256x256 launch at P
                                   workgroups looping over tiles (default 256, one per CU;
                                   0: one workgroup per tile) */
#define MVML_OPT_GEMM_NSPLIT 4  /* MVML_GEMM_NSPLIT: 1 (default) N = 256 q + r products as two
                                   launches, 0 = one */
#define MVML_OPT_GEMM_RING 5    /* (rounds 3-5: the LDS-DMA ring kernel; removed in round 6 —
                                   the option is accepted and ignored) */
#define MVML_OPT_LSTM_TILE 6    /* MVML_LSTM_TILE: tile of the wide BiLSTM step products
                                   (mvml_bilstm_wide_step_*): 0 (default) planned from the live
                                   row count, 128 / 256 = forced; 128 also moves
                                   mvml_lstm_gates_cell_fwd to the 128x128 kernel (measured
                                   slower there at 65,536 rows: 0.78 vs 0.70 ms) */
#define MVML_OPT_MEAN_SRC 7     /* MVML_MEAN_SRC: 1 (default) = head-mean (last) GAT layer's
                                   aggregation backward by source atom (one wave per atom reads its
                                   projection row once and gathers the F-wide g_out rows of its
                                   out-edges; no LDS windows), 0 = molecule / big windows +
                                   per-atom pair */
#define MVML_OPT_FLAT_SRC 8     /* MVML_FLAT_SRC: flatten GAT layers' aggregation backward by
                                   source atom (one wave per atom gathers its out-neighbours'
                                   rows; g_rst of each gathered row formed in registers from
                                   g_out / out): 1 or 2 (the same one-pass kernel since round
                                   5); 0 (default) = molecule / big
                                   windows + per-atom pair.  The Python layer sets it per call
                                   for batches of large molecules (mvml_gat.functional) */
#define MVML_OPT_DST_FWD 9      /* MVML_DST_FWD: 1 = aggregation forward by destination wave for
                                   every atom (edge softmax on the lanes, whole projection rows of
                                   the in-edges gathered from L2; no LDS windows), 0 (default) =
                                   molecule / big windows + gather kernel.  The Python layer sets
                                   it per call for batches of large molecules; 2 = the same
                                   with the edge softmax as its own launch first */
#define MVML_OPT_DST_UNR 10     /* MVML_DST_UNR: projection rows in flight per wave of the
                                   destination-wave forward (0 = the default per width; tuning) */
#define MVML_OPT_SMALLK 11      /* MVML_SMALLK: 1 (default) mvml_gemm_f16x2_rows products with
                                   K <= 96 (layer 1's projection) on the wave-per-64-columns
                                   memory kernel (non-temporal stores; 2 = plain stores;
                                   3 .. 6, 10: timing variants, tools/smallk_bench.py);
                                   0 = the 256x256 tile */
int mvml_set_option(int option, int value);
int mvml_get_option(int option);

/* ---------------------------------------------------------------------------------------
 * Batching: dgl.batch (dataset.py:54) + DGL's COO->CSR conversion on first update_all.
 * Inputs are the per-graph LOCAL edge lists of mol_to_bigraph (dataset.py:34-35) concatenated
 * in graph order, plus batch_num_nodes/batch_num_edges (int64[B]).  Outputs are bit-exact with
 * dgl.batch's global src/dst and with a stable counting sort by dst (in-CSR) and by src
 * (out-CSR).  status_flags (int32[2]): [0] = number of nodes with zero in-degree (GATConv
 * raises DGLError on those, dgl 0.9.1 GATConv.forward), [1] = number of out-of-range local ids.
 * ------------------------------------------------------------------------------------- */
size_t mvml_build_csr_workspace_size(int64_t num_graphs, int64_t num_nodes, int64_t num_edges);
int mvml_build_csr(const int32_t* src_local, const int32_t* dst_local,
                   const int64_t* batch_num_nodes, const int64_t* batch_num_edges,
                   int64_t num_graphs, int64_t num_nodes, int64_t num_edges,
                   int64_t* node_offsets /* [B+1] */, int64_t* edge_offsets /* [B+1] */,
                   int32_t* src /* [E] */, int32_t* dst /* [E] */, int32_t* node_graph /* [N] */,
                   int32_t* in_rowptr /* [N+1] */, int32_t* in_src /* [E] */,
                   int32_t* in_eid /* [E] */, int32_t* out_rowptr /* [N+1] */,
                   int32_t* out_dst /* [E] */, int32_t* out_inslot /* [E] */,
                   int32_t* status_flags /* [2] */, void* workspace, size_t workspace_bytes,
                   void* stream);

/* Node groups (no reference counterpart: the launch geometry of the aggregation kernels).
 * Group g = the contiguous range of WHOLE molecules [group_start[g], group_start[g+1]) that
 * begins with the molecule containing atom 64*g; G = mvml_node_group_count(N) groups, some
 * possibly empty.  Every in-edge of a group's atoms starts inside the group, so one workgroup
 * can stage a group's projection rows in LDS and read each of them from HBM once.
 * The PLAN (int32[mvml_node_group_plan_size(N)]) holds, for G groups:
 *   [0, G]          group_start (group_start[G] = N)
 *   [G+1, 2G+1)     kind: bit 0 = forward LDS kernel (<= 128 atoms, <= 512 in-edges, every
 *                   in-degree <= 5), bit 1 = backward LDS kernel (<= 128 atoms, <= 512 edges),
 *                   bit 2 = big LDS window (<= 512 atoms, <= 2432 in-edges, any in-degree:
 *                   the fallback-list groups the big-window kernels take, H <= 4)
 *   2G+1, 2G+2      number of non-empty groups without bit 0 / bit 1
 *   [2G+3, 3G+3)    those groups for the forward fallback kernel (any order)
 *   [3G+3, 4G+3)    those groups for the backward fallback kernels
 * so the aggregation launches never scan the CSR to route groups.  node_offsets: int64[B+1]
 * and in_rowptr: int32[N+1] from mvml_build_csr. */
int64_t mvml_node_group_count(int64_t num_nodes);
int64_t mvml_node_group_plan_size(int64_t num_nodes);
int mvml_build_node_groups(int64_t num_graphs, int64_t num_nodes, const int64_t* node_offsets,
                           const int32_t* in_rowptr, int32_t* plan, void* stream);

/* ---------------------------------------------------------------------------------------
 * Dense fp32 GEMM on CDNA4 MFMA (v_mfma_f32_32x32x2_f32, exact f32 fmaf chains).
 * C[M,N] = act(A[M,K] * B[K,N] + bias[N] + beta * C)
 *   a_kmajor = 0: A(m,k) = A[m*lda + k]      a_kmajor = 1: A(m,k) = A[k*lda + m]
 *   b_kmajor = 0: B(k,n) = B[n*ldb + k]      b_kmajor = 1: B(k,n) = B[k*ldb + n]
 *   act: 0 none, 1 ReLU.  Replaces nn.Linear / torch.matmul (cuBLAS / rocBLAS) used by
 *   GATConv.fc/res_fc, Set2Set's nn.LSTM and GNNModule.fc (model.py:86-87).  K is split over
 *   workgroups when M*N is small (deterministic slab reduction, needs workspace).
 * ------------------------------------------------------------------------------------- */
size_t mvml_gemm_workspace_size(int64_t M, int64_t N, int64_t K);
int mvml_gemm_f32(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                  const float* A, int64_t lda, const float* B, int64_t ldb,
                  const float* bias, float beta, int act, float* C, int64_t ldc,
                  void* workspace, size_t workspace_bytes, void* stream);
/* Same contract, computed on bf16 MFMA (v_mfma_f32_32x32x16_bf16) at fp32 accuracy: each fp32
 * operand is split exactly into three bf16 terms (x = x0 + x1 + x2, 24 significant bits) and
 * the six cross products with relative weight >= 2^-16 are accumulated in fp32; the dropped
 * ones are < 2^-25 relative.  Errors against fp64 are those of an fp32 GEMM (verified in
 * tests/test_gpu_parity.py); results are deterministic but not bitwise equal to mvml_gemm_f32. */
int mvml_gemm_f32x3(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                    const float* A, int64_t lda, const float* B, int64_t ldb,
                    const float* bias, float beta, int act, float* C, int64_t ldc,
                    void* workspace, size_t workspace_bytes, void* stream);
/* mvml_gemm_f32x3 over `batch` independent products (grid z): product z reads A + z stride_a,
 * B + z stride_b and writes C + z stride_c (floats); no split-K, so no workspace.  For the
 * fusion head's per-head 384 x 384 weight products (one launch instead of twelve). */
int mvml_gemm_f32x3_batched(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                            int64_t batch, const float* A, int64_t lda, int64_t stride_a,
                            const float* B, int64_t ldb, int64_t stride_b, const float* bias,
                            float beta, int act, float* C, int64_t ldc, int64_t stride_c,
                            void* stream);
/* bf16 operands (round-to-nearest-even from the fp32 inputs), one v_mfma_f32_32x32x16_bf16 per
 * fragment pair, fp32 accumulate: the "bf16 projection on MFMA" of BASELINE.json config 4
 * (accuracy bar 2e-2 relative, north_star).  Same arguments / workspace as mvml_gemm_f32. */
int mvml_gemm_bf16(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                   const float* A, int64_t lda, const float* B, int64_t ldb,
                   const float* bias, float beta, int act, float* C, int64_t ldc,
                   void* workspace, size_t workspace_bytes, void* stream);
/* Same contract at fp32 accuracy on fp16 MFMA (v_mfma_f32_32x32x16_f16), half the MFMAs of
 * mvml_gemm_f32x3: each operand is scaled by a power of two s (|max| s in [2^14, 2^15), from a
 * deterministic |max| pass over the operand) and split into x s = h + l with h = f16(x s),
 * l = f16(x s - h) (22 significant bits; representation error <= 2^-22 relative, plus 2^-40 of
 * the operand's |max| absolute where l is subnormal); the product keeps h_a h_b + h_a l_b +
 * l_a h_b (the dropped l_a l_b is < 2^-22 relative), fp32 accumulate, and the result is scaled
 * back by 1 / (s_a s_b) exactly.  Errors against fp64 are those of an fp32 GEMM
 * (tests/test_gpu_parity.py).  Products whose plan is not the 256x256 tile (skinny outputs)
 * run the split-bf16 kernels.  Workspace as mvml_gemm_f32 (its first 256 B hold the maxima). */
int mvml_gemm_f16x2(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                    const float* A, int64_t lda, const float* B, int64_t ldb,
                    const float* bias, float beta, int act, float* C, int64_t ldc,
                    void* workspace, size_t workspace_bytes, void* stream);
/* mvml_gemm_f16x2 with the operand maxima supplied: *amax_a / *amax_b = bits of max |A| /
 * max |B| over (at least) the elements the product reads, e.g. from mvml_absmax_f32 — one pass
 * serves every product that reads the operand.  A bound above the true max is allowed (costs
 * accuracy only if it exceeds it by more than ~2^10). */
int mvml_gemm_f16x2_amax(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                         const float* A, int64_t lda, const float* B, int64_t ldb,
                         const uint32_t* amax_a, const uint32_t* amax_b, const float* bias,
                         float beta, int act, float* C, int64_t ldc, void* workspace,
                         size_t workspace_bytes, void* stream);
/* mvml_gemm_f16x2 with PER-ROW A maxima: amax_a_rows[m] = bits of max_k |A[m, k]| (or an upper
 * bound; mvml_absmax_rows_f32, or folded by the kernel that wrote A), A K-contiguous
 * ([M][lda]); *amax_b as mvml_gemm_f16x2_amax.  Every A row is split with its own power-of-two
 * scale and its output row scaled back by it, so (a) a row keeps fp32-GEMM accuracy relative to
 * ITSELF however far it sits below the operand's max (the operand-wide scale loses precision
 * ~2^17 below it, where the low fp16 plane goes subnormal), and (b) a row of C depends only on
 * its own row of A and on B: the same molecule gives bitwise the same output in any batch. */
int mvml_gemm_f16x2_rows(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                         const float* B, int64_t ldb, int b_kmajor, const float* b_il4,
                         const uint32_t* amax_a_rows, const uint32_t* amax_b, const float* bias,
                         float beta, int act, float* C, int64_t ldc, void* workspace,
                         size_t workspace_bytes, void* stream);
/* 1 if mvml_gemm_f16x2_rows with these arguments (b = b_il4 if given, else B) runs on the
 * small-K memory kernel under the current options, else 0 (the 256x256 tile): how a caller
 * or a timer tells which roofline a product belongs to (no device work). */
int mvml_gemm_rows_smallk(int b_kmajor, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                          const float* B, int64_t ldb, float beta, int act, const float* C,
                          int64_t ldc);
/* mvml_gemm_f16x2_rows (no beta, no split-K: K is a feature dimension; the 256x256 tile at any
 * size) with a strided batch and epilogue extras (the ELU link: layer 2's data gradient leaves
 * as layer 1's g_rst through act 3):
 *  - product z < batch reads A + z stride_a, B (or b_il4) + z stride_b, amax_a_rows + z
 *    stride_rows, bias + z stride_bias and writes C + z stride_c;
 *  - act: 0 none, 1 ReLU, 2 ELU after the bias (x > 0 ? x : expm1(x)), 3 the ELU backward
 *    through the layer output aux (ld_aux): v *= aux > 0 ? 1 : aux + 1;
 *  - c_amax (may be NULL): atomicMax of the bits of max |stored value|;
 *  - c_rows (may be NULL): per-row |max| bits of the stored values, row r of column slot
 *    col / c_rows_cols (c_rows_cols = 0: one slot) at c_rows[z stride_c_rows + slot
 *    c_rows_stride + r], by atomicMax (the caller zeroes it; c_rows_cols % 64 == 0).
 * A, B rows and strides 16-B aligned, K % 4 == 0. */
int mvml_gemm_f16x2_ex(int64_t M, int64_t N, int64_t K, int64_t batch, const float* A, int64_t lda,
                       int64_t stride_a, const float* B, int64_t ldb, int b_kmajor,
                       const float* b_il4, int64_t stride_b, const uint32_t* amax_a_rows,
                       int64_t stride_rows, const uint32_t* amax_b, const float* bias,
                       int64_t stride_bias, int act, float* C, int64_t ldc, int64_t stride_c,
                       const float* aux, int64_t ld_aux, uint32_t* c_amax, uint32_t* c_rows,
                       int64_t c_rows_stride, int c_rows_cols, int64_t stride_c_rows, void* stream);
/* Strided-batch split-fp16 GEMM (batch >= 2, no split-K) with operand-wide maxima shared by all
 * products: C + z stride_c = (A + z stride_a)(B + z stride_b), layouts as mvml_gemm_f32. */
int mvml_gemm_f16x2_batched(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                            int64_t batch, const float* A, int64_t lda, int64_t stride_a,
                            const float* B, int64_t ldb, int64_t stride_b, const uint32_t* amax_a,
                            const uint32_t* amax_b, float* C, int64_t ldc, int64_t stride_c,
                            void* stream);
/* B pre-split once as an interleaved-by-4 image for the split-fp16 GEMMs: every 4 consecutive
 * values of a row become [4 scaled high fp16 | 4 low fp16] (16 B, the scale from *amax as the
 * GEMM's own split), written to out with P's own [rows][ld] float indexing, so the image stands
 * in for B in any layout (K-contiguous or K-major): the 256x256 tiles load a piece with one 16-B
 * load and skip B's split (b_il4 of mvml_gemm_f16x2_rows; mvml_gemm_f16x2_bsplit with
 * b_plane = 0; mvml_lstm_gates_cell_fwd with w_plane = 0).  Bitwise the in-kernel split.
 * cols % 4 == 0, ld % 4 == 0, P and out 16-B aligned. */
int mvml_split_f16x2_il4(int64_t rows, int64_t cols, const float* P, int64_t ld,
                         const uint32_t* amax, float* out, void* stream);
/* The "il8" split-fp16 image of an fp32 operand for mvml_gemm_f16x2_planes (round 6): out is
 * [rows][ld_out] floats; per 8-value k group g < ld_out / 8 of row r it holds the 8 scaled high
 * fp16 halves of x[r][8g .. 8g+7], then the 8 low halves (the GEMM's own split: scale from
 * *amax, or from amax_rows[r] — exactly one of the two), k >= K as zeros.  x[r][k] is
 * P[r*ld + k] (kmajor = 0) or P[k*ld + r] (kmajor = 1: the image of the transpose).
 * ld_out >= K rounded up to 32, ld_out % 8 == 0, out 16-B aligned. */
int mvml_split_f16x2_il8(int64_t rows, int64_t K, const float* P, int64_t ld, int kmajor,
                         const uint32_t* amax, const uint32_t* amax_rows, float* out,
                         int64_t ld_out, void* stream);
/* C[M][N] = act(A B^T + bias + beta C) at fp32 accuracy (scaled split-fp16, three fp16 MFMAs
 * per product; the 256x256 tile with both operands staged by LDS-DMA, round 6), B given as its
 * il8 image b_image ([N][ldb], ldb >= K rounded up to 32, made with amax_b).  A is fp32
 * [M][lda] (K % 4 == 0; its scale from *amax_a, or per row from amax_a_rows — exactly one) or,
 * with a_image != 0, its il8 image made with the same maxima (lda >= K rounded up to 32).
 * act 0 / 1 (ReLU); rows 16-B aligned.  The mvml_gemm_f16x2_rows / _amax product of the same
 * operands to fp32 accuracy (a different MFMA order: not bitwise). */
int mvml_gemm_f16x2_planes(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                           int a_image, const uint32_t* amax_a, const uint32_t* amax_a_rows,
                           const float* b_image, int64_t ldb, const uint32_t* amax_b,
                           const float* bias, float beta, int act, float* C, int64_t ldc,
                           void* stream);
/* out[r] = bits of max_c |P[r*ld + c]|, c < cols (accumulate != 0: max with the current out[r]);
 * one writer per row, no atomics. */
int mvml_absmax_rows_f32(int64_t rows, int64_t cols, const float* P, int64_t ld, uint32_t* out,
                         int accumulate, void* stream);
/* mvml_gemm_f16x2_amax with B also given as its interleaved split image (b_planes, from
 * mvml_split_f16x2_il4 with *amax_b, the same [.][ldb] indexing as B; b_plane must be 0 — the
 * two-plane layout was removed in round 6): the 256x256 tiles read the image; plans that do not
 * use that kernel read the fp32 B. */
int mvml_gemm_f16x2_bsplit(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                           const float* A, int64_t lda, const float* B, int64_t ldb,
                           const uint16_t* b_planes, int64_t b_plane, const uint32_t* amax_a,
                           const uint32_t* amax_b, const float* bias, float beta, int act,
                           float* C, int64_t ldc, void* workspace, size_t workspace_bytes,
                           void* stream);
/* out[0] = bits of max |P[r*ld + c]| over r < rows, c < cols (accumulate != 0: max with the
 * current out[0]); deterministic (unsigned atomicMax of non-negative float bits). */
int mvml_absmax_f32(int64_t rows, int64_t cols, const float* P, int64_t ld, uint32_t* out,
                    int accumulate, void* stream);
#define MVML_GEMM_F32 0   /* algo: v_mfma_f32_32x32x2_f32 */
#define MVML_GEMM_F32X3 1 /* algo: split-bf16 x3 */
#define MVML_GEMM_BF16 2  /* algo: bf16 operands, fp32 accumulate */
#define MVML_GEMM_F16X2 3 /* algo: scaled split-fp16 (mvml_gemm_f16x2) */
/* Column sums: out[n] = beta*out[n] + alpha * sum_m X[m*ldx + n], deterministic two-stage
 * tree.  Replaces the bias gradients torch autograd computes for GATConv.bias / LSTM / Linear. */
size_t mvml_colsum_workspace_size(int64_t M, int64_t N);
int mvml_colsum_f32(int64_t M, int64_t N, const float* X, int64_t ldx, float alpha, float beta,
                    float* out, void* workspace, size_t workspace_bytes, void* stream);
/* A weight gradient and the bias gradient of the same output gradient in one call (round 6):
 *   C[M][N]    = A^T B^T, A [K][lda] and B [K][ldb] both k-major (mvml_gemm_f16x2_amax(1, 1, ...))
 *   sum_out[c] = alpha * sum_k A[k][sum_off + c], c < sum_n (mvml_colsum_f32 over those columns)
 * For a GATConv (autograd of gatconv.py's fc / res_fc / bias, model.py:79-81) A = gY, B = X:
 * dL/dWcat and, over gY's residual columns, dL/dbias.  When mvml_gemm_colsum_fused(M, N, K)
 * (the skinny 128x128 plan: layer 1, N = 76 atom features) the column sums come out of the
 * fragments the product reads (fp32 adds, fixed order: deterministic, not the order of
 * mvml_colsum_f32); otherwise the product then mvml_colsum_f32, bitwise the two calls. */
int mvml_gemm_colsum_fused(int64_t M, int64_t N, int64_t K);
size_t mvml_gemm_colsum_workspace_size(int64_t M, int64_t N, int64_t K, int64_t sum_n);
int mvml_gemm_f16x2_amax_colsum(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const float* B,
                                int64_t ldb, const uint32_t* amax_a, const uint32_t* amax_b, float* C,
                                int64_t ldc, int64_t sum_off, int64_t sum_n, float alpha, float* sum_out,
                                void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * GATConv projection (dgl 0.9.1 GATConv.fc and res_fc, gatconv.py forward, homogeneous-graph
 * branch; called from dgllife GATLayer.forward, model.py:79-81) as ONE GEMM:
 *   Y[N, C] = X[N, Fin] * Wcat^T,  Wcat[C, Fin] rows = [fc.weight ; Wr]
 *   Wr = res_fc.weight (H*F rows), or with mean_residual = 1 its head mean
 *        (1/H) sum_h res_fc.weight[h*F+f, :] (F rows): a 'mean' GATLayer only ever uses the
 *        head-mean of the residual, so that layer's GEMM is 37 % smaller.
 *   Y row = [ Z (H*F) | R (H*F or F) ];  C = mvml_gat_proj_cols(H,F,mean).
 *   Wcat has row stride ldw >= Fin; columns Fin..ldw-1 are written as zeros, so a caller can
 *   pad X to a multiple of 4 columns and keep every GEMM operand 16-B aligned.
 * With attn_lr = [attn_l | attn_r] ([2, H*F], may be NULL) mvml_gat_fold_weights also writes
 * 2H rows after the C projection rows, A_l[h,:] = sum_f attn_l[h,f] fc.weight[h*F+f,:] and
 * A_r likewise: the backward multiplies mvml_gat_agg_bwd's [d el | d er] columns by them, which
 * is exactly the el / er path of dL/dX (el = Z . attn_l = X . A_l^T).
 * mvml_gat_unfold_grads maps dL/dWcat back onto fc.weight and res_fc.weight (the mean
 * residual's gradient is replicated / H over the heads); with attn_lr it adds the el / er
 * path of dL/dfc.weight from dL/dWcat's extra rows: attn_l[h,f] * G_l[h,:] + attn_r[h,f] *
 * G_r[h,:], G = [d el | d er]^T X.
 * ------------------------------------------------------------------------------------- */
int mvml_gat_proj_cols(int H, int F, int mean_residual);
int mvml_gat_fold_weights(const float* fc_w, const float* res_fc_w, const float* attn_lr, int H,
                          int F, int Fin, int ldw, int mean_residual, float* Wcat, void* stream);
int mvml_gat_unfold_grads(const float* gWcat, const float* attn_lr, int H, int F, int Fin,
                          int ldg, int mean_residual, float* g_fc_w, float* g_res_fc_w,
                          void* stream);
/* The projection GEMM (X [N, K] with row stride ldx, Wcat [C, K] with row stride ldw, K = the
 * padded feature count) + GATConv's attention logits from the result:
 *   el[n,h] = <Z[n,h,:], attn_l[h,:]>,  er[n,h] = <Z[n,h,:], attn_r[h,:]>
 * (`(feat_src * attn_l).sum(-1)`), computed in the GEMM epilogue as per-32-column partial dots
 * of the fp32 Z tile and summed per head in fixed order — no second pass over Z.
 * attn_lr: [2, H*F] = [attn_l | attn_r]; elr: [N, 2H] = [el | er].  F % 32 == 0.
 * algo MVML_GEMM_F16X2: amax_x / amax_w = bits of max |X| / max |Wcat| (mvml_absmax_f32), or
 * both NULL (computed here); w_planes must be NULL (w_plane ignored: the two-plane weight image
 * was removed in round 6).
 * workspace: mvml_gat_proj_fwd_workspace_size(N, H, F) bytes. */
size_t mvml_gat_proj_fwd_workspace_size(int64_t num_nodes, int H, int F);
int mvml_gat_proj_fwd(int64_t num_nodes, const float* X, int64_t ldx, int64_t K,
                      const float* Wcat, int64_t ldw, const float* attn_lr, int H, int F,
                      int mean_residual, int algo /* MVML_GEMM_* */, float* Y, int64_t ldy,
                      float* elr, const uint32_t* amax_x, const uint32_t* amax_w,
                      const uint16_t* w_planes, int64_t w_plane, void* workspace,
                      size_t workspace_bytes, void* stream);
/* dL/dattn_l[h,f] = sum_n gelr[n, h] * Z[n, h*F+f] and dL/dattn_r with gelr[n, H+h] (autograd
 * of `(feat * attn_l).sum(-1)` in GATConv.forward); gelr rows [d el | d er] have stride ldgl
 * (the backward's gY + C, ldgy); deterministic two-stage reduction. */
size_t mvml_gat_attn_grad_workspace_size(int64_t num_nodes, int H, int F);
int mvml_gat_attn_grad(int64_t num_nodes, int H, int F, const float* Y, int64_t ldy,
                       const float* gelr, int64_t ldgl, float* g_attn_l, float* g_attn_r,
                       void* workspace, size_t workspace_bytes, void* stream);
/* ---------------------------------------------------------------------------------------
 * Fused GAT attention + aggregation, forward (one workgroup per node group; replaces dgl
 * GATConv.forward from apply_edges to the residual/bias, plus dgllife GATLayer's flatten/ELU
 * or head-mean, model.py:77-81):
 *   apply_edges(u_add_v) on elr -> LeakyReLU(slope) -> edge_softmax -> update_all(u_mul_e,
 *   sum) -> + residual R -> + bias -> GATLayer agg (dgllife 0.3.0): mode 0 flatten+ELU,
 *   mode 1 mean over heads, mode 2 flatten (no activation).
 * Y is the projection output (mean_residual layout iff mode 1; ldy >= its C, multiple of 4),
 * elr its logits (mvml_gat_proj_fwd).  out is [N, H*F] (modes 0, 2) or [N, F] (mode 1).
 * attn [E, H] receives the edge_softmax output in in-CSR slot order (needed by the backward).
 * out_amax (may be NULL): *out_amax = max(*out_amax, bits of max |out|), folded into the stores
 * (the split-fp16 operand max of the next layer's / Set2Set's GEMMs; the caller zeroes it).
 * out_row_amax (may be NULL): out_row_amax[n] = bits of max_c |out[n, c]| for every atom, written
 * once per row (no atomics; the per-row scales of the next products, mvml_gemm_f16x2_rows).
 * node_groups is the plan mvml_build_node_groups built from the same in_rowptr (a plan of
 * another graph is undefined behaviour); num_groups = mvml_node_group_count(num_nodes).
 * ------------------------------------------------------------------------------------- */
int mvml_gat_agg_fwd(int64_t num_nodes, const int32_t* node_groups, int64_t num_groups,
                     const int32_t* in_rowptr, const int32_t* in_src, const float* Y, int64_t ldy,
                     int H, int F, const float* elr, const float* bias, float slope, int mode,
                     float* out, float* attn, uint32_t* out_amax, uint32_t* out_row_amax,
                     void* stream);
/* Backward of mvml_gat_agg_fwd (DGL GSpMM / GSDDMM / EdgeSoftmax backward + torch autograd of
 * residual, bias, ELU, mean).  Atomic-free: the u_mul_e-sum transpose is a gather over the
 * out-CSR; one workgroup per node group reads Z, g_out and writes dZ once (molecule groups).
 * Writes gY[N, ldgy] (ldgy >= C + 2H, C = mvml_gat_proj_cols) =
 *   [ dZ_agg (H*F) | dR (H*F or F) | d el (H) | d er (H) ]
 * where dZ_agg is dL/dZ through update_all(u_mul_e, sum) only: the el / er paths of dL/dZ
 * (d el x attn_l + d er x attn_r) reach dL/dX and dL/dfc.weight through the 2H extra columns
 * (GEMM against mvml_gat_fold_weights' A rows; mvml_gat_unfold_grads), and dL/dattn through
 * mvml_gat_attn_grad(gelr = gY + C, ldgl = ldgy).
 * out is the forward output (mode 0 uses ELU'(x) = out + 1 for x <= 0).  gy_amax (may be NULL):
 * *gy_amax = max(*gy_amax, bits of max |gY[:, :C + 2H]|), folded into the stores (the split-fp16
 * operand max of the two GEMMs that read gY; the caller zeroes it).  gy_row_amax (may be NULL):
 * gy_row_amax[n] = bits of max_c |gY[n, c]|, c < C + 2H, for every atom (the per-row scales of the
 * data-gradient product, mvml_gemm_f16x2_rows; no float atomics).  workspace: [E, H]. */
size_t mvml_gat_agg_bwd_workspace_size(int64_t num_edges, int H);
int mvml_gat_agg_bwd(int64_t num_nodes, const int32_t* node_groups, int64_t num_groups,
                     const int32_t* in_rowptr, const int32_t* in_src, const int32_t* out_rowptr,
                     const int32_t* out_dst, const int32_t* out_inslot, const float* Y,
                     int64_t ldy, const float* elr, const float* attn, const float* out,
                     const float* g_out, int H, int F, float slope, int mode, float* gY,
                     int64_t ldgy, uint32_t* gy_amax, uint32_t* gy_row_amax, void* workspace,
                     size_t workspace_bytes, void* stream);
/* A GATConv's whole backward in one call (SURVEY §8(b)'s proj_bwd; the autograd of dgl GATConv /
 * dgllife GATLayer, model.py:81, 91): from the forward's X ([N][Fp], Fp = Fin rounded up to 4,
 * zero-padded), Wcat and attn_lr (mvml_gat_fold_weights' inputs / output), Y (ldy), elr, attn, out
 * and g_out = dL/d out, it writes g_X ([N][Fin]; NULL: not formed), g_fc and g_res ([H F][Fin]:
 * fc.weight's and res_fc.weight's layouts), g_attn ([2][H F]: attn_l's then attn_r's) and g_bias
 * ([H F]).  mean = 0: flatten + ELU layer (aggregation mode 0), 1: head mean (mode 1).
 * The same launches, in the same order, as mvml_gat.functional.GATLayerFunction.backward (so
 * bitwise its results): mvml_gat_agg_bwd, the split-K weight-gradient product
 * (mvml_gemm_f16x2_amax), mvml_gat_unfold_grads, the attention-vector product
 * (mvml_gemm_f32x3_batched), mvml_colsum_f32 and the per-row-scaled data-gradient product
 * (mvml_gemm_f16x2_rows, Wcat as its interleaved image), every operand maximum and scratch
 * buffer inside `workspace` (mvml_gat_layer_bwd_workspace_size bytes).  The aggregation
 * backward's kernel choice follows the process options (mvml_set_option) as for
 * mvml_gat_agg_bwd: the Python layer sets "flat_src" for large-molecule batches. */
size_t mvml_gat_layer_bwd_workspace_size(int64_t num_nodes, int64_t num_edges, int H, int F, int Fin,
                                         int mean);
int mvml_gat_layer_bwd(int64_t num_nodes, const int32_t* node_groups, int64_t num_groups,
                       const int32_t* in_rowptr, const int32_t* in_src, const int32_t* out_rowptr,
                       const int32_t* out_dst, const int32_t* out_inslot, int64_t num_edges, int H,
                       int F, int Fin, int mean, float slope, const float* X, const float* Wcat,
                       const float* attn_lr, const float* Y, int64_t ldy, const float* elr,
                       const float* attn, const float* out, const float* g_out, float* g_X,
                       float* g_fc, float* g_res, float* g_attn, float* g_bias, void* workspace,
                       size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * Set2Set (dgl 0.9.1, model.py:82-84, 92) building blocks.
 * LSTM cell (torch.nn.LSTM gate order i,f,g,o): gates_pre[B, 4D] = x W_ih^T + h W_hh^T (by
 * mvml_gemm_f32), then
 *   c = sigmoid(f)*c_prev + sigmoid(i)*tanh(g);  h = sigmoid(o)*tanh(c)
 * act_out[B,4D] saves the activated gates for the backward.  c_prev may be NULL (zeros), and
 * so may gates_pre (zero pre-activations: the bias alone).
 * h is written with leading dimension ldh, and again to h_out2 (ld ldh2) when h_out2 is not
 * NULL: the cell's output is both its own recurrent input and the next layer's input, each
 * stored inside a combined [x | h_prev] GEMM operand row.
 * ------------------------------------------------------------------------------------- */
/* The gates GEMM with the LSTM cell as its epilogue (Set2Set's cells): pre = A w_perm^T for the
 * D units with w_perm's rows INTERLEAVED (row 4 j + q = row q D + j of [W_ih | W_hh]; K of its
 * columns used, row stride ldw), then exactly mvml_lstm_cell_fwd (b_ih, b_hh gate-major; c_prev
 * may be null) — the gate pre-activations are never stored.  Requires the 256x256 plan without
 * split-K (mvml_lstm_gates_cell_plan_ok(M, D, K) != 0) and 16-B aligned rows. */
int mvml_lstm_gates_cell_plan_ok(int64_t M, int D, int64_t K);
int mvml_lstm_gates_cell_fwd(int64_t M, int D, int64_t K, const float* A, int64_t lda,
                             const float* w_perm, int64_t ldw, const float* b_ih,
                             const float* b_hh, const float* c_prev, float* c_out, float* h_out,
                             int64_t ldh, float* act, float* h_out2, int64_t ldh2,
                             const uint32_t* amax_a, const uint32_t* amax_b /* both NULL:
                               split-bf16; else split-fp16 with these |A|, |w_perm| max bits */,
                             const uint32_t* amax_a_rows /* NULL, or per-row |A| max bits (M
                               entries; replaces amax_a, see mvml_gemm_f16x2_rows) */,
                             const uint16_t* w_planes, int64_t w_plane /* NULL, or w_perm's
                               interleaved image (mvml_split_f16x2_il4 with amax_b; w_plane
                               must be 0) */,
                             void* stream);
/* Per molecule b: out_bits[b] = max(floor_bits, max_{n in [node_offsets[b], node_offsets[b+1])}
 * in_bits[n]) on non-negative float bits — a molecule's bound from its atoms' row maxima (the
 * per-molecule split-fp16 scales of Set2Set's cells; floor 1.0f bounds the LSTM's |h| < 1). */
int mvml_segment_max_bits(int64_t B, const int64_t* node_offsets, const uint32_t* in_bits,
                          uint32_t floor_bits, uint32_t* out_bits, void* stream);
int mvml_lstm_cell_fwd(int64_t B, int D, const float* gates_pre, const float* b_ih,
                       const float* b_hh, const float* c_prev, float* c_out, float* h_out,
                       int64_t ldh, float* act_out, float* h_out2, int64_t ldh2, void* stream);
/* g_h [B,D] (ld ldgh) + g_h2 [B,D] (ld ldgh2; may be NULL: a second consumer's dL/dh, summed
 * in the kernel), g_c [B,D] (carry from t+1, may be NULL) -> g_gates [B,4D] (pre-act),
 * g_c_prev [B,D] (may be NULL).  gg_amax (may be NULL): *gg_amax = max(*gg_amax, bits of
 * max |g_gates|) — the split-fp16 operand max of the GEMMs that read g_gates.  gb_part (may be
 * NULL): [R][4D] partial column sums of g_gates, R = mvml_lstm_cell_bwd_part_rows(B, D) (the
 * bias gradient is their column sum, over every step's partial). */
int64_t mvml_lstm_cell_bwd_part_rows(int64_t B, int D);
int mvml_lstm_cell_bwd(int64_t B, int D, const float* act, const float* c, const float* c_prev,
                       const float* g_h, int64_t ldgh, const float* g_h2, int64_t ldgh2,
                       const float* g_c, float* g_gates, float* g_c_prev, uint32_t* gg_amax,
                       float* gb_part, void* stream);
/* Readout segment pass (one wavefront per molecule): e_n = <x_n, q_g>, alpha = softmax over
 * the molecule's atoms (softmax_nodes), r_g = sum_n alpha_n x_n (sum_nodes).  Writes r into
 * qstar[:, D:2D] (ld ldq, q itself already sits in qstar[:, 0:D]) and lse[g] for backward. */
int mvml_set2set_seg_fwd(int64_t B, int D, const int64_t* node_offsets, const float* X,
                         float* qstar, int64_t ldq, float* lse, void* stream);
/* Backward of one segment pass: from g_qstar[:, D:2D] (= dL/dr) computes dL/dq into
 * g_q (g_q = g_qstar[:, 0:D] + segment term; may alias g_qstar with ld ldgq), and saves
 * alpha[N], g_e[N] for mvml_set2set_gx. */
int mvml_set2set_seg_bwd(int64_t B, int D, const int64_t* node_offsets, const float* X,
                         const float* qstar, int64_t ldq, const float* lse,
                         const float* g_qstar, int64_t ldgq, float* g_q, int64_t ldgout,
                         float* alpha, float* g_e, void* stream);
/* dL/dX[n] = sum_t alpha_t[n] * g_r_t[g(n)] + g_e_t[n] * q_t[g(n)] over T iterations,
 * g(n) = the molecule of atom n.  With node_offsets (int64[num_graphs + 1], mvml_build_csr)
 * and T <= 6, D <= 512: one wavefront per molecule (its 2T vectors loaded once); otherwise one
 * per atom through node_graph[n].  qstars: T consecutive [B, ldq] buffers (stride
 * qstar_stride), g_qstars likewise; alphas / g_es: T consecutive [N] buffers. */
int mvml_set2set_gx(int64_t num_nodes, int D, int T, const int32_t* node_graph,
                    const int64_t* node_offsets, int64_t num_graphs,
                    const float* qstars, int64_t ldq, int64_t qstar_stride,
                    const float* g_qstars, int64_t ldgq, int64_t g_qstar_stride,
                    const float* alphas, const float* g_es, float* gX, void* stream);

/* ---------------------------------------------------------------------------------------
 * GraphNorm (torch_geometric 2.2.0, eps, batch=None at model.py:93): independent statistics
 * per normalisation group (group_offsets int64[G+1], in rows); the reference's group is its
 * 64-molecule mini-batch (config.py:21).
 * ------------------------------------------------------------------------------------- */
int mvml_graphnorm_fwd(int64_t G, int D, const int64_t* group_offsets, const float* x,
                       const float* weight, const float* bias, const float* mean_scale,
                       float eps, float* y, void* stream);
size_t mvml_graphnorm_bwd_workspace_size(int64_t G, int D);
int mvml_graphnorm_bwd(int64_t G, int D, const int64_t* group_offsets, const float* x,
                       const float* weight, const float* mean_scale, float eps,
                       const float* g_y, float* g_x, float* g_weight, float* g_bias,
                       float* g_mean_scale, void* workspace, size_t workspace_bytes,
                       void* stream);

/* Small elementwise helpers.  ReLU backward (threshold_backward on the output), times the
 * Dropout scale when a Dropout followed the ReLU (scale = 1 / (1 - p), 1 without one):
 * g_x = g_y * scale * (y > 0).  y is the DROPPED output: a dropped element reads 0, so its
 * gradient is 0 without a stored mask (nn.Dropout's backward is g * mask * scale). */
int mvml_relu_bwd(int64_t n, const float* y, const float* g_y, float* g_x, float scale, void* stream);
/* nn.Dropout(p) in training mode (model.py:87, 36, 46; torch's fused_dropout): y = x * keep /
 * (1 - p), x == y allowed; element i kept iff a 32-bit counter-based hash of (seed, i) is at
 * least round(p 2^32).  The mask is a function of (seed, i) only: nothing is stored, and after
 * a ReLU the backward is mvml_relu_bwd's scaled form with scale = (float)(1 / (1 - p)), the
 * float this kernel multiplies by.  0 <= p < 1. */
int mvml_dropout_fwd(int64_t n, const float* x, float* y, double p, int64_t seed, void* stream);
/* dst[r][0:cols) = src[r][0:cols) for r < rows (row pitches lds, ldd): a narrow column slice
 * of a wide row-pitched matrix into a dense one (the projection output's 2H logit columns);
 * lds = 0 replicates src's one row into every dst row. */
int mvml_copy_cols(int64_t rows, int cols, const float* src, int64_t lds, float* dst, int64_t ldd,
                   void* stream);
/* Zero `rows` rows of row_bytes bytes at a pitch of pitch_bytes (hipMemsetAsync, or
 * hipMemset2DAsync when pitch_bytes > row_bytes): the zero initial states and accumulators. */
int mvml_fill_zero(void* p, int64_t rows, int64_t row_bytes, int64_t pitch_bytes, void* stream);
/* Set2Set's LSTM weights in the gates products' layouts (nn.LSTM w_ih [4D][kin], w_hh [4D][D]):
 * wcat [4D][kin + D] = [w_ih | w_hh]; wperm (may be NULL) the same rows interleaved for the
 * cell epilogue (row 4 j + q = wcat row q D + j, see mvml_lstm_gates_cell_fwd). */
int mvml_lstm_pack_weights(int D, int kin, const float* w_ih, const float* w_hh, float* wcat,
                           float* wperm, void* stream);
/* dst[c][r] = src[r][c] (row pitches lds, ldd). */
int mvml_transpose(int64_t rows, int64_t cols, const float* src, int64_t lds, float* dst, int64_t ldd,
                   void* stream);
/* y[i] = x[i] * s[0], s a device scalar (x == y allowed). */
int mvml_scale_by(int64_t n, const float* x, const float* s, float* y, void* stream);

/* ---------------------------------------------------------------------------------------
 * Multi-view attention fusion head (MVP, model.py:28-48, 57-71), the consumer
 * of the graph view.  GEMMs (Q/K/V, MLP) use mvml_gemm_f32x3; the rest:
 *   mvml_layernorm_fwd/_bwd: torch.nn.LayerNorm over rows of D <= 512 (model.py:23, 54-56);
 *     fwd saves per-row mean / rstd; bwd writes g_x and g_y_xhat[rows, D] = g_y * xhat, whose
 *     column sums (mvml_colsum_f32) are dL/dgamma (dL/dbeta = column sums of g_y).
 *   mvml_token_attn_fwd/_bwd: the 3-token attention of model.py:62-68 per (molecule, head);
 *     qkv rows 3b+t = [q (H*dk) | k (H*dk) | v (H*dk)] (ld >= 3 H dk), dk = 384; att [B, H, 3,
 *     dk] (the Conv2d input layout), P [B, H, 3, 3] saved softmax; scale = 1/sqrt(dk).
 *   mvml_token_attn_fold_fwd/_bwd: the same attention with Q.K re-associated: s_ij =
 *     <p_i, x_j> scale, p = x M_h (M_h = W_q,h^T W_k,h), pv rows 3b+t = [p (H*dk) | v (H*dk)]
 *     (ld >= 2 H dk), x = the LayerNorm rows (keys of every head, ldx >= dk); the backward
 *     writes g_pv [3B, 2 H dk] and g_k = sum over heads of dL/dx through the keys [3B, dk].
 *   mvml_conv3_fwd/_bwd: Conv2d(12, 12, kernel 3) + ReLU on att (model.py:27, 69):
 *     in [B, 12, 3, W] -> out [B, 12, W-2] (post-ReLU); bwd gives g_in, g_weight [12,12,3,3],
 *     g_bias [12] (deterministic partial sums; workspace mvml_conv3_bwd_workspace_size(B)).
 *   mvml_bce_logits: BCEWithLogitsLoss (mean, main.py:91) element terms and dL/dz.
 * ------------------------------------------------------------------------------------- */
int mvml_layernorm_fwd(int64_t rows, int D, const float* x, int64_t ldx, const float* gamma,
                       const float* beta, float eps, float* y, int64_t ldy, float* mean,
                       float* rstd, void* stream);
int mvml_layernorm_bwd(int64_t rows, int D, const float* x, int64_t ldx, const float* gamma,
                       const float* mean, const float* rstd, const float* g_y, int64_t ldgy,
                       float* g_x, int64_t ldgx, float* g_y_xhat, void* stream);
int mvml_token_attn_fwd(int64_t B, int H, int dk, const float* qkv, int64_t ld, float scale,
                        float* att, float* P, void* stream);
int mvml_token_attn_bwd(int64_t B, int H, int dk, const float* qkv, int64_t ld, float scale,
                        const float* P, const float* g_att, float* g_qkv, int64_t ldg,
                        void* stream);
int mvml_token_attn_fold_fwd(int64_t B, int H, int dk, const float* pv, int64_t ld,
                             const float* x, int64_t ldx, float scale, float* att, float* P,
                             void* stream);
/* g_pv_amax (may be NULL): *g_pv_amax = max(*g_pv_amax, bits of max |g_pv|) (split-fp16 scale
 * of the two GEMMs that read g_pv; the caller zeroes it). */
int mvml_token_attn_fold_bwd(int64_t B, int H, int dk, const float* pv, int64_t ld,
                             const float* x, int64_t ldx, float scale, const float* P,
                             const float* g_att, float* g_pv, int64_t ldg, float* g_k,
                             int64_t ldgk, uint32_t* g_pv_amax, void* stream);
int mvml_conv3_fwd(int64_t B, int C, int O, int W, const float* in, const float* weight,
                   const float* bias, float* out, void* stream);
size_t mvml_conv3_bwd_workspace_size(int64_t B);
int mvml_conv3_bwd(int64_t B, int C, int O, int W, const float* in, const float* weight,
                   const float* out, const float* g_out, float* g_in, float* g_weight,
                   float* g_bias, void* workspace, size_t workspace_bytes, void* stream);
/* mvml_attn_conv_fwd / _bwd: mvml_token_attn_fold_fwd + mvml_conv3_fwd (and the backward pair)
 * fused, H = 12, dk = 384: the (B, 12, 3, 384) attention cube lives only in LDS.  Forward
 * writes P [B, H, 3, 3] (saved softmax) and out [B, 12, dk - 2] (post-ReLU); the backward
 * recomputes the cube from P and pv's v columns and writes g_pv, g_k (as
 * mvml_token_attn_fold_bwd), g_weight, g_bias (as mvml_conv3_bwd; workspace
 * mvml_attn_conv_bwd_workspace_size(B)).  Replaces model.py:66-69's att -> conv round trip.
 * g_pv_rows (may be NULL; zeroed by the caller, 3 B entries): max with the bits of each g_pv
 * row's |max| (the per-row scales of the data-gradient product that reads g_pv).  g_scale:
 * the Dropout after the ReLU (model.py:36) — out is then the dropped output and the ReLU
 * gradient is g_out * g_scale where out > 0 (1: no Dropout).  The forward applies that Dropout
 * in its store when drop_p > 0 (mask of mvml_dropout_fwd for (drop_seed, element index of out);
 * g_scale = (float)(1 / (1 - drop_p))). */
int mvml_attn_conv_fwd(int64_t B, int H, int dk, const float* pv, int64_t ld, const float* x,
                       int64_t ldx, float scale, const float* weight, const float* bias,
                       float* P, float* out, double drop_p, int64_t drop_seed, void* stream);
size_t mvml_attn_conv_bwd_workspace_size(int64_t B);
int mvml_attn_conv_bwd(int64_t B, int H, int dk, const float* pv, int64_t ld, const float* x,
                       int64_t ldx, float scale, const float* P, const float* weight,
                       const float* out, const float* g_out, float g_scale, float* g_pv,
                       int64_t ldg, float* g_k, int64_t ldgk, uint32_t* g_pv_amax, uint32_t* g_pv_rows,
                       float* g_weight, float* g_bias, void* workspace, size_t workspace_bytes,
                       void* stream);
int mvml_bce_logits(int64_t n, const float* z, const float* y, float* loss_terms, float* g_z,
                    void* stream);

/* ---------------------------------------------------------------------------------------
 * SMILES BiLSTM view (RNNModule, model.py:98-135; nn.Embedding + nn.LSTM(bidirectional,
 * batch_first) over pack_padded_sequence(enforce_sorted=False) + the last-step selection of
 * model.py:131-133).  Packed layout: rows t*B + i, batch sorted by descending length
 * (perm[i] = original index of sorted row i, pos = perm^-1), tokens int32 [B, ldtok] in the
 * original order, lens int32 [B] >= 1.  batch_sizes (HOST int32 [T], non-increasing) is the
 * number of sequences alive per step.
 *   gather_rows: out[t*B+i, :] = t < lens[perm[i]] ? table[tokens[perm[i], t], :] : 0
 *                (layer 0's x W_ih^T as rows of the [vocab, 4H] table E W_ih^T; cols % 4 == 0)
 *   token_grad:  out[v, :] = sum of g[t*B+i, :] over live positions holding token v
 *                (fixed order, deterministic; replaces Embedding / W_ih_l0 backward; vocab <= 64;
 *                workspace of mvml_bilstm_token_grad_workspace bytes)
 *   select_last: dir 0: fea[b] = [out[(lens[b]-1)*B + pos[b], 0:H] | out[pos[b], H:2H]];
 *                dir 1: the transpose, fea -> out rows (out must be zeroed by the caller).
 *   seq_fwd:     one layer's recurrence, both directions (torch.nn.LSTM bidirectional over the
 *                packed batch, model.py:121-129): per step t (direction 0) / T-1-t (direction 1)
 *                pre = gates_d[t] + h_prev W_hh_d^T + b_ih_d + b_hh_d, the LSTM cell, h into
 *                out[t*B+i, d*H : (d+1)*H], c into c_d, (i, f, g, o) into act_d.  gates_d =
 *                x W_ih_d^T [T*B, 4H]; out / c_d must be zeroed by the caller (dead rows are
 *                read as the zero state); H % 16 == 0.
 *   seq_bwd:     its backward: g_out [T*B, 2H] (dL/d out); gg_d [T*B, 4H] (zeroed by the
 *                caller) receives dL/d pre; w_hhT_d = W_hh_d^T [H, 4H]; carry [2, B, H] zeroed
 *                scratch (the dL/dc chain).  dW / db / dx follow from gg_d by GEMMs.
 * ------------------------------------------------------------------------------------- */
int mvml_bilstm_gather_rows(int64_t T, int64_t B, int64_t cols, const float* table,
                            const int32_t* tokens, int64_t ldtok, const int32_t* lens,
                            const int32_t* perm, float* out, void* stream);
int64_t mvml_bilstm_token_grad_workspace(int64_t T, int64_t B, int64_t cols, int vocab);
int mvml_bilstm_token_grad(int64_t T, int64_t B, int64_t cols, const float* g,
                           const int32_t* tokens, int64_t ldtok, const int32_t* lens,
                           const int32_t* perm, int vocab, float* out, void* workspace,
                           size_t workspace_bytes, void* stream);
int mvml_bilstm_seq_fwd(int64_t T, int64_t B, int H, const int32_t* batch_sizes,
                        const float* gates0, const float* gates1, const float* w_hh0,
                        const float* w_hh1, const float* b_ih0, const float* b_hh0,
                        const float* b_ih1, const float* b_hh1, float* out, float* c0, float* c1,
                        float* act0, float* act1, void* stream);
int mvml_bilstm_seq_bwd(int64_t T, int64_t B, int H, const int32_t* batch_sizes,
                        const float* w_hhT0, const float* w_hhT1, const float* act0,
                        const float* act1, const float* c0, const float* c1, const float* g_out,
                        float* gg0, float* gg1, float* carry, void* stream);
int mvml_bilstm_select_last(int64_t B, int64_t H, const int32_t* lens, const int32_t* pos,
                            float* out, float* fea, int dir, void* stream);
/* Wide batches (B > 512, BASELINE config 4): one launch per time step for BOTH directions of a
 * bidirectional layer (direction 0 at step t, direction 1 at T - 1 - t; M0 / M1 live rows).
 *   fwd: gates_d = A_d W_d^T + gx_d + b_ih_d + b_hh_d, then the LSTM cell (nn.LSTM,
 *        model.py:114-129): c_d, h_d (row stride ldh), act_d = [i | f | g | o] (gate-major).
 *        W_d = W_hh_d with INTERLEAVED rows (row 4 j + q = gate q of unit j); gx_d the step's
 *        input projection rows (gate-major, ld ldgx); A_d the previous step's h rows (ld lda),
 *        K = 0 at the directions' first step (c_prev NULL).  Split-fp16 GEMM: amax_a = bits of a
 *        bound of |h| (1.0), amax_w_d = bits of max |W_hh_d|.
 *   bwd: dh = gout rows + gn_d W_hh_d (gn_d = the gate gradients of the step this one fed, its
 *        first R_d rows; R_d = 0 at the directions' first backward step), then the cell
 *        backward (mvml_lstm_cell_bwd's arithmetic): gg_d, carry_out_d = dL/dc_prev; gg_amax_d
 *        is the running max |gg_d| (read as gn_d's split-fp16 scale, raised by the step).
 *        wT_d = W_hh_d^T [D][4 D]; workspace mvml_bilstm_wide_step_bwd_workspace_size(max M, D). */
int mvml_bilstm_wide_step_fwd(int64_t M0, int64_t M1, int D, int64_t K, const float* A0,
                              const float* A1, int64_t lda, const float* W0, const float* W1,
                              int64_t ldw, const float* gx0, const float* gx1, int64_t ldgx,
                              const float* bih0, const float* bhh0, const float* bih1,
                              const float* bhh1, const float* cprev0, const float* cprev1,
                              float* c0, float* c1, float* h0, float* h1, int64_t ldh,
                              float* act0, float* act1, const uint32_t* amax_a,
                              const uint32_t* amax_w0, const uint32_t* amax_w1, void* stream);
/* Live rows of a time-major [T, B, cols] buffer (row stride ld_tm) <-> consecutive packed rows
 * (stride ld_pk): packed row offsets[k] + p <-> buffer row (t0 + k + shift) B + p for
 * k < t_count, p < offsets[k + 1] - offsets[k] (int32 offsets[t_count + 1] on the device,
 * nrows = offsets[t_count]).  dir 0 packs, 1 unpacks.  The wide path's products over every
 * position run over the live rows only (pack_padded_sequence's data, model.py:125). */
int mvml_bilstm_pack_rows(int64_t nrows, int64_t t_count, int64_t B, int64_t cols,
                          const int32_t* offsets, int64_t t0, int shift, float* tm,
                          int64_t ld_tm, float* packed, int64_t ld_pk, int dir, void* stream);
/* Token of every packed live row (row offsets[t] + p = step t of sorted sequence p) and the
 * embedding-side gradient out[v] = sum of g's packed rows with token v in packed order
 * (mvml_bilstm_token_grad over the live rows only; workspace
 * mvml_bilstm_token_grad_packed_workspace bytes). */
int mvml_bilstm_packed_tokens(int64_t nrows, int64_t T, const int32_t* offsets,
                              const int32_t* tokens, int64_t ldtok, const int32_t* perm,
                              int32_t* tok, void* stream);
int64_t mvml_bilstm_token_grad_packed_workspace(int64_t nrows, int64_t cols, int vocab);
int mvml_bilstm_token_grad_packed(int64_t nrows, int64_t cols, const float* g, int64_t ldg,
                                  const int32_t* tok, int vocab, float* out, void* workspace,
                                  size_t workspace_bytes, void* stream);
size_t mvml_bilstm_wide_step_bwd_workspace_size(int64_t M, int D);
int mvml_bilstm_wide_step_bwd(int64_t M0, int64_t M1, int64_t R0, int64_t R1, int D,
                              const float* gn0, const float* gn1, const float* wT0,
                              const float* wT1, int64_t ldwT, const float* gout0,
                              const float* gout1, int64_t ldgo, const float* act0,
                              const float* act1, const float* c0, const float* c1,
                              const float* cp0, const float* cp1, const float* carry_in0,
                              const float* carry_in1, float* carry_out0, float* carry_out1,
                              float* gg0, float* gg1, uint32_t* gg_amax0, uint32_t* gg_amax1,
                              const uint32_t* amax_w0, const uint32_t* amax_w1, void* workspace,
                              size_t workspace_bytes, void* stream);
/* The whole recurrence of one wide layer, every step's dual launch above enqueued by a native
 * loop (batch_sizes: host int32[T], positive, non-increasing, <= B — pack_padded_sequence's;
 * D % 8 == 0).  W_hh (resp. its transpose) is split once per call into the workspace.
 *   fwd: W_d interleaved as above; gx_d [T][B][4D] the input projections; c_d [T][B][D];
 *        out [T][B][2D] (direction d in columns d D ..); act_d [T][B][4D]; amax[3] = bits of
 *        (1.0, max |W_hh_0|, max |W_hh_1|); workspace mvml_bilstm_wide_fwd_workspace_size(D).
 *   bwd: wT_d = W_hh_d^T; gout [T][B][2D]; carry [2][2][B][D] ZEROED scratch; gg_d [T][B][4D]
 *        ZEROED when time-major (padding rows stay zero); gg_amax[2] zeroed running maxima; amax as fwd;
 *        workspace mvml_bilstm_wide_bwd_workspace_size(B, D).
 *   gx_packed / gg_packed != 0: gx_d (resp. gg_d) hold the live rows only, step t's
 *        batch_sizes[t] rows after those of steps < t (pack_padded_sequence's data layout,
 *        mvml_bilstm_pack_rows' packed side); gg_d then needs no zeroing. */
size_t mvml_bilstm_wide_fwd_workspace_size(int D);
int mvml_bilstm_wide_fwd(int64_t T, int64_t B, int D, const int32_t* batch_sizes, const float* W0,
                         const float* W1, const float* gx0, const float* gx1, const float* bih0,
                         const float* bhh0, const float* bih1, const float* bhh1, float* c0,
                         float* c1, float* out, float* act0, float* act1, const uint32_t* amax,
                         int gx_packed, void* workspace, size_t workspace_bytes, void* stream);
size_t mvml_bilstm_wide_bwd_workspace_size(int64_t B, int D);
int mvml_bilstm_wide_bwd(int64_t T, int64_t B, int D, const int32_t* batch_sizes, const float* wT0,
                         const float* wT1, const float* gout, const float* act0, const float* act1,
                         const float* c0, const float* c1, float* carry, float* gg0, float* gg1,
                         uint32_t* gg_amax, const uint32_t* amax, int gg_packed, void* workspace,
                         size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * Optimizer step on flat buffers: main.py:88's torch.optim.Adam(params, lr, weight_decay)
 * (amsgrad off, L2 decay into the gradient) over every parameter at once, with "this
 * parameter has a gradient" kept on the device (torch skips parameters whose .grad is None;
 * across ranks, one whose all-reduced flag is 0).  Parameters occupy [param_off[i],
 * param_off[i] + n_i) of the flat buffers; a static chunk table (chunk c covers
 * [chunk_beg[c], chunk_end[c]) of parameter chunk_param[c]) gives one workgroup per chunk.
 * ------------------------------------------------------------------------------------- */
/* flat[param_off[i] ..] = the gradient at src[i] (a device pointer, 0 = none: zeros), and
 * flat[numel + i] = 1.0 / 0.0 (the presence flag) for i < P. */
int mvml_grad_gather(int64_t nchunks, const int32_t* chunk_param, const int64_t* chunk_beg,
                     const int64_t* chunk_end, const int64_t* param_off, const uint64_t* src, int P,
                     float* flat, int64_t numel, void* stream);
/* For every parameter i with flags[i] > 0: step = steps[i] + 1, g = grad * grad_scale (+
 * weight_decay param), exp_avg += (1 - beta1)(g - exp_avg), exp_avg_sq = beta2 exp_avg_sq +
 * (1 - beta2) g^2, param -= lr / (1 - beta1^step) * exp_avg / (sqrt(exp_avg_sq) /
 * sqrt(1 - beta2^step) + eps) (torch's Adam); then steps[i] += 1.  Others are untouched. */
int mvml_adam_flat(int64_t nchunks, const int32_t* chunk_param, const int64_t* chunk_beg,
                   const int64_t* chunk_end, const float* flags, int32_t* steps, int P, float* param,
                   const float* grad, float* exp_avg, float* exp_avg_sq, double lr, double beta1,
                   double beta2, double eps, double weight_decay, float grad_scale, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MVML_GAT_H */
