// SMILES BiLSTM view (RNNModule, /root/reference/model.py:98-135): the
// index kernels around the packed bidirectional LSTM and its fused recurrence.
//
// Packed layout (what pack_padded_sequence(enforce_sorted=False) builds, model.py:128): the
// batch is ordered by descending length (perm[i] = original index of sorted row i) and stored
// time-major, row t*B + i, so the sequences alive at step t are the prefix i < batch_sizes[t].
//
// Layer 0's input projection is a table lookup: Embedding(tok) W_ih^T = (E W_ih^T)[tok], so the
// host computes P = E W_ih^T once ([V, 4H], V = 39 tokens) and mvml_bilstm_gather_rows expands
// it; the backward sums the gate gradients per token (mvml_bilstm_token_grad) and multiplies the
// [V, 4H] result into dE and dW_ih with two small GEMMs.
//
// Recurrence (mvml_bilstm_seq_fwd / _bwd): one launch per time step carries BOTH directions
// (forward direction at t, reverse at T-1-t) and fuses the recurrent product with the cell (the
// tile layout is described above the step kernels).  At KEGG batch sizes (B <= 64, ~20 rows
// alive per step on average) a step is a few microseconds of latency, not FLOPs: a kernel
// boundary (~1.5 us, MI355X_MICROARCH.md price table, row boundary) is cheaper than an
// in-launch grid barrier (barrier-xcd ~4-5 us), so the time loop lives on the host side of the
// C ABI (no Python per step) rather than in a persistent grid; W_hh (2.4 MB per direction)
// stays L2-resident across the step launches.
#include "common.h"

namespace mvml {
namespace {

unsigned grid_1d(int64_t total) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(total, 256), 16384));
}

// out[(t*B+i), :] = t < len(perm[i]) ? table[tok[perm[i], t], :] : 0      (cols % 4 == 0)
__global__ void gather_rows_kernel(int64_t T, int64_t B, int64_t cols4, const float4* table,
                                   const int32_t* tokens, int64_t ldtok, const int32_t* lens,
                                   const int32_t* perm, float4* out) {
  const int64_t total = T * B * cols4;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = e / cols4, j = e - row * cols4;
    const int64_t t = row / B, i = row - t * B;
    const int32_t b = perm[i];
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t < lens[b]) v = table[(int64_t)tokens[b * ldtok + t] * cols4 + j];
    out[e] = v;
  }
}

// out[v, j] = sum over live positions (t ascending, then sorted row i ascending) with token v
// of g[(t*B+i), j].  One workgroup per (token, 256-column slab); fixed order => deterministic.
__global__ void token_grad_kernel(int64_t T, int64_t B, int64_t cols, const float* g,
                                  const int32_t* tokens, int64_t ldtok, const int32_t* lens,
                                  const int32_t* perm, float* out) {
  const int v = blockIdx.x;
  const int64_t j = blockIdx.y * (int64_t)blockDim.x + threadIdx.x;
  float acc = 0.f;
  for (int64_t t = 0; t < T; ++t) {
    for (int64_t i = 0; i < B; ++i) {
      const int32_t b = perm[i];
      if (t >= lens[b]) break;  // sorted by descending length: the rest are padding
      if (tokens[b * ldtok + t] == v && j < cols) acc += g[(t * B + i) * cols + j];
    }
  }
  if (j < cols) out[(int64_t)v * cols + j] = acc;
}

// text_fea[b] = [ out[(len_b - 1)*B + pos_b, 0:H] | out[pos_b, H:2H] ]   (model.py:131-133)
// dir = 0 gathers; dir = 1 scatters g_fea back into g_out (distinct rows, no races).
__global__ void select_last_kernel(int64_t B, int64_t H, const int32_t* lens, const int32_t* pos,
                                   float* out, float* fea, int dir) {
  const int64_t total = B * 2 * H;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / (2 * H), j = e - b * 2 * H;
    const int64_t t = j < H ? lens[b] - 1 : 0;
    float* src = out + (t * B + pos[b]) * 2 * H + j;
    if (dir == 0) fea[e] = *src;
    else *src = fea[e];
  }
}


// ------------------------------------------------------------------ fused recurrence steps
// A workgroup owns a 16-row x 16-column output tile of the step's recurrent product and splits
// its K over the waves: v_mfma_f32_16x16x4_f32 (exact f32), operands straight from global
// memory (L2-resident W_hh, the previous step's rows), every lane's loads issued before the
// first MFMA (one memory round trip), wave partials summed in LDS in a fixed order, then the
// cell runs on the tile.
//   forward:  tile = 16 rows x (4 units x 4 gates); K = H over 4 waves (96 each)
//   backward: tile = 16 rows x 16 units;            K = 4H over 8 waves (192 each)
typedef float f32x4_t __attribute__((ext_vector_type(4)));
constexpr int kStepRows = 16;
constexpr int kFwdUnits = 4, kFwdWaves = 4;
constexpr int kBwdUnits = 16, kBwdWaves = 8;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// acc += A (16 x 16 k) B (16 k x 16) for one float4 of each operand per lane: lane l holds
// A[l % 16][k0 + 4 (l / 16) + s] and B[k0 + 4 (l / 16) + s][l % 16], s = 0..3 (the four MFMA
// k-steps see k = k0 + 4 (l / 16) + s: a permutation of k0 .. k0 + 15, the same on both sides)
__device__ __forceinline__ f32x4_t mfma4(float4 a, float4 b, f32x4_t acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
  return acc;
}

struct FwdDir {          // one direction of a forward step
  const float* gin;      // [T*B][4H] input projection x W_ih^T
  const float* w;        // W_hh [4H][H]
  const float* b_ih;
  const float* b_hh;
  float* c;              // [T*B][H]
  float* act;            // [T*B][4H] (i, f, g, o)
  int t, prev, bs;       // prev: the step whose h / c feed this one (-1: none)
};

// pre = x W_ih^T + h_prev W_hh^T + b_ih + b_hh; i, f, o = sigmoid, g = tanh;
// c = f c_prev + i g; h = o tanh(c)      (nn.LSTM, model.py:121; lstm_cell_fwd_kernel's order)
template <int H>
__global__ void __launch_bounds__(64 * kFwdWaves)
bilstm_step_fwd_kernel(int B, FwdDir d0, FwdDir d1, float* __restrict__ out) {
  constexpr int KW = H / kFwdWaves;  // K per wave
  constexpr int NF = KW / 16;        // float4 loads per lane and operand
  constexpr int G = 4 * H;
  static_assert(KW % 16 == 0, "H % 64 == 0");
  __shared__ float s_part[kFwdWaves][16][17];
  const int dir = blockIdx.y;
  const FwdDir D = dir ? d1 : d0;
  constexpr int nsl = H / kFwdUnits;
  const int sl = blockIdx.x % nsl, rb = blockIdx.x / nsl;
  const int r0 = rb * kStepRows;
  if (r0 >= D.bs) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j0 = sl * kFwdUnits;
  // the cell's operands first (threads < 64: one (row, unit) each), in flight with the MFMA
  // operands below
  const int row = (tid >> 2) & 15, u = tid & 3, r = r0 + row, j = j0 + u;
  const bool cell = tid < 64 && r < D.bs;
  const int64_t rt = (int64_t)D.t * B + (cell ? r : r0);
  float pre[4], bi[4], bh[4], cp = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) pre[q] = bi[q] = bh[q] = 0.f;
  if (cell) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      pre[q] = D.gin[rt * G + q * H + j];
      bi[q] = D.b_ih[q * H + j];
      bh[q] = D.b_hh[q * H + j];
    }
    if (D.prev >= 0) cp = D.c[((int64_t)D.prev * B + r) * H + j];
  }
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  if (D.prev >= 0) {
    // A: h_prev rows (dead rows read the zero state, rows past B clamp to a live row)
    const int ra = min(r0 + (lane & 15), B - 1);
    const float* ap = out + ((int64_t)D.prev * B + ra) * 2 * H + dir * H + w * KW + 4 * (lane >> 4);
    // B: W_hh row of gate column n = lane % 16 (gate n / 4, unit j0 + n % 4)
    const int n = lane & 15;
    const float* bp = D.w + (int64_t)((n >> 2) * H + j0 + (n & 3)) * H + w * KW + 4 * (lane >> 4);
    float4 a[NF], b[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      a[i] = ld4(ap + 16 * i);
      b[i] = ld4(bp + 16 * i);
    }
    __builtin_amdgcn_sched_barrier(0);  // every load in flight before the first MFMA
#pragma unroll
    for (int i = 0; i < NF; ++i) acc = mfma4(a[i], b[i], acc);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) s_part[w][4 * (lane >> 4) + r][lane & 15] = acc[r];
  __syncthreads();
  // 64 (row, unit) pairs: the four gates of unit u sit in columns 4q + u
  if (!cell) return;
  float a[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float sum = s_part[0][row][4 * q + u];
#pragma unroll
    for (int ww = 1; ww < kFwdWaves; ++ww) sum += s_part[ww][row][4 * q + u];
    a[q] = pre[q] + sum + bi[q] + bh[q];
  }
  const float i = sigm(a[0]), f = sigm(a[1]), gt = tanhf(a[2]), o = sigm(a[3]);
  const float c = f * cp + i * gt;
  const float h = o * tanhf(c);
  float* av = D.act + rt * G + j;
  av[0] = i;
  av[H] = f;
  av[2 * H] = gt;
  av[3 * H] = o;
  D.c[rt * H + j] = c;
  out[rt * 2 * H + dir * H + j] = h;
}

struct BwdDir {          // one direction of a backward step
  const float* wT;       // W_hh^T [H][4H]
  const float* act;      // [T*B][4H]
  const float* c;        // [T*B][H]
  float* gg;             // [T*B][4H] gate gradients (out)
  float* carry;          // [B][H] dL/dc carried between steps (zeroed by the caller)
  int t, nxt, tp, bs, bs_nxt;  // nxt: the step this one fed (-1: none); tp: c_prev's step
};

// g_h = g_out[t] + gg[nxt] W_hh (rows alive at nxt); lstm_cell_bwd_kernel's cell backward with
// the carried dL/dc (in place: each (row, unit) is read and rewritten by its own thread)
template <int H>
__global__ void __launch_bounds__(64 * kBwdWaves)
bilstm_step_bwd_kernel(int B, BwdDir d0, BwdDir d1, const float* __restrict__ g_out) {
  constexpr int G = 4 * H;
  constexpr int KW = G / kBwdWaves;
  constexpr int NF = KW / 16;
  constexpr int NB = NF / 2;  // two batches of loads (registers)
  static_assert(KW % 32 == 0, "H % 64 == 0");
  __shared__ float s_part[kBwdWaves][16][17];
  const int dir = blockIdx.y;
  const BwdDir D = dir ? d1 : d0;
  constexpr int nsl = H / kBwdUnits;
  const int sl = blockIdx.x % nsl, rb = blockIdx.x / nsl;
  const int r0 = rb * kStepRows;
  if (r0 >= D.bs) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j0 = sl * kBwdUnits;
  // the cell's operands first (threads < 256: one (row, unit) each)
  const int row = (tid >> 4) & 15, u = tid & 15, r = r0 + row, j = j0 + u;
  const bool cell = tid < 256 && r < D.bs;
  const int64_t rt = (int64_t)D.t * B + (cell ? r : r0);
  float go = 0.f, gcar = 0.f, cc = 0.f, cp = 0.f, av[4] = {0.f, 0.f, 0.f, 0.f};
  if (cell) {
    go = g_out[rt * 2 * H + dir * H + j];
    gcar = D.carry[(int64_t)r * H + j];
    cc = D.c[rt * H + j];
    if (D.tp >= 0) cp = D.c[((int64_t)D.tp * B + r) * H + j];
#pragma unroll
    for (int q = 0; q < 4; ++q) av[q] = D.act[rt * G + q * H + j];
  }
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  if (D.nxt >= 0 && r0 < D.bs_nxt) {
    // A: gg[nxt] rows (rows past bs_nxt hold zeros: the caller zeroes gg), B: W_hh^T rows
    const int ra = min(r0 + (lane & 15), B - 1);
    const float* ap = D.gg + ((int64_t)D.nxt * B + ra) * G + w * KW + 4 * (lane >> 4);
    const float* bp = D.wT + (int64_t)(j0 + (lane & 15)) * G + w * KW + 4 * (lane >> 4);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float4 a[NB], b[NB];
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        a[i] = ld4(ap + 16 * (h * NB + i));
        b[i] = ld4(bp + 16 * (h * NB + i));
      }
      __builtin_amdgcn_sched_barrier(0);  // the batch's loads in flight before its MFMAs
#pragma unroll
      for (int i = 0; i < NB; ++i) acc = mfma4(a[i], b[i], acc);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) s_part[w][4 * (lane >> 4) + r][lane & 15] = acc[r];
  __syncthreads();
  if (!cell) return;
  float rec = s_part[0][row][u];
#pragma unroll
  for (int ww = 1; ww < kBwdWaves; ++ww) rec += s_part[ww][row][u];
  const float gh = go + rec;
  const float i = av[0], f = av[1], gt = av[2], o = av[3];
  const float tc = tanhf(cc);
  const float gc = gcar + gh * o * (1.f - tc * tc);
  float* gq = D.gg + rt * G + j;
  gq[0] = gc * gt * i * (1.f - i);
  gq[H] = gc * cp * f * (1.f - f);
  gq[2 * H] = gc * i * (1.f - gt * gt);
  gq[3 * H] = gh * tc * o * (1.f - o);
  D.carry[(int64_t)r * H + j] = gc * f;
}

// Deterministic token gradient: chunk k of kTokChunk positions (t-major) x 256-column slab sums
// its live positions per token in LDS, then partial_tok_kernel adds the chunks in order.
constexpr int kTokChunk = 256;
constexpr int kTokMaxVocab = 64;
__global__ void __launch_bounds__(256)
token_grad_chunk_kernel(int64_t T, int64_t B, int64_t cols, const float* __restrict__ g,
                        const int32_t* __restrict__ tokens, int64_t ldtok,
                        const int32_t* __restrict__ lens, const int32_t* __restrict__ perm,
                        int vocab, float* __restrict__ part) {
  __shared__ float s_acc[kTokMaxVocab][256];
  const int tid = threadIdx.x;
  const int64_t j = blockIdx.y * 256 + tid;
  for (int v = 0; v < vocab; ++v) s_acc[v][tid] = 0.f;
  const int64_t p0 = (int64_t)blockIdx.x * kTokChunk, p1 = min<int64_t>(T * B, p0 + kTokChunk);
  for (int64_t p = p0; p < p1; ++p) {  // same token order in every lane: no LDS races
    const int64_t t = p / B, i = p - t * B;
    const int32_t b = perm[i];
    if (t >= lens[b]) continue;
    const int v = tokens[b * ldtok + t];
    if (j < cols) s_acc[v][tid] += g[p * cols + j];
  }
  if (j < cols)
    for (int v = 0; v < vocab; ++v) part[((int64_t)blockIdx.x * vocab + v) * cols + j] = s_acc[v][tid];
}

__global__ void token_grad_sum_kernel(int64_t nchunk, int64_t n, const float* __restrict__ part,
                                      float* __restrict__ out) {
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e >= n) return;
  float acc = 0.f;
  for (int64_t k = 0; k < nchunk; ++k) acc += part[k * n + e];
  out[e] = acc;
}

}  // namespace
}  // namespace mvml

using namespace mvml;

extern "C" int mvml_bilstm_gather_rows(int64_t T, int64_t B, int64_t cols, const float* table,
                                       const int32_t* tokens, int64_t ldtok,
                                       const int32_t* lens, const int32_t* perm, float* out,
                                       void* stream) {
  clear_error();
  MVML_REQUIRE(T >= 0 && B >= 0 && cols > 0 && cols % 4 == 0 && ldtok >= T,
               "bilstm_gather_rows: bad shape (cols %% 4 == 0, ldtok >= T)");
  if (T * B == 0) return MVML_OK;
  gather_rows_kernel<<<grid_1d(T * B * cols / 4), 256, 0, as_stream(stream)>>>(
      T, B, cols / 4, reinterpret_cast<const float4*>(table), tokens, ldtok, lens, perm,
      reinterpret_cast<float4*>(out));
  return check_launch("bilstm_gather_rows");
}

extern "C" int64_t mvml_bilstm_token_grad_workspace(int64_t T, int64_t B, int64_t cols, int vocab) {
  return ceil_div(T * B, kTokChunk) * vocab * cols * (int64_t)sizeof(float);
}

extern "C" int mvml_bilstm_token_grad(int64_t T, int64_t B, int64_t cols, const float* g,
                                      const int32_t* tokens, int64_t ldtok, const int32_t* lens,
                                      const int32_t* perm, int vocab, float* out, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  clear_error();
  MVML_REQUIRE(T >= 0 && B >= 0 && cols > 0 && vocab > 0 && vocab <= kTokMaxVocab && ldtok >= T,
               "bilstm_token_grad: bad shape (vocab <= 64)");
  hipStream_t st = as_stream(stream);
  const int64_t nchunk = ceil_div(T * B, kTokChunk);
  if (nchunk == 0) {
    (void)hipMemsetAsync(out, 0, (size_t)vocab * cols * sizeof(float), st);
    return check_launch("bilstm_token_grad(empty)");
  }
  MVML_REQUIRE(workspace && (int64_t)workspace_bytes >= mvml_bilstm_token_grad_workspace(T, B, cols, vocab),
               "bilstm_token_grad: workspace too small");
  float* part = static_cast<float*>(workspace);
  dim3 grid((unsigned)nchunk, (unsigned)ceil_div(cols, 256));
  token_grad_chunk_kernel<<<grid, 256, 0, st>>>(T, B, cols, g, tokens, ldtok, lens, perm, vocab, part);
  int rc = check_launch("bilstm_token_grad(chunks)");
  if (rc) return rc;
  const int64_t n = (int64_t)vocab * cols;
  token_grad_sum_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(nchunk, n, part, out);
  return check_launch("bilstm_token_grad(sum)");
}

extern "C" int mvml_bilstm_seq_fwd(int64_t T, int64_t B, int H, const int32_t* batch_sizes,
                                   const float* gates0, const float* gates1, const float* w_hh0,
                                   const float* w_hh1, const float* b_ih0, const float* b_hh0,
                                   const float* b_ih1, const float* b_hh1, float* out, float* c0,
                                   float* c1, float* act0, float* act1, void* stream) {
  clear_error();
  MVML_REQUIRE(T >= 0 && B > 0 && B <= (1 << 20) && H == 384 && batch_sizes,
               "bilstm_seq_fwd: bad shape (H = 384, MVP's blstm_dim; host batch_sizes)");
  for (int64_t t = 0; t < T; ++t)
    MVML_REQUIRE(batch_sizes[t] >= 0 && batch_sizes[t] <= B && (t == 0 || batch_sizes[t] <= batch_sizes[t - 1]),
                 "bilstm_seq_fwd: batch_sizes must be non-increasing in [0, B]");
  hipStream_t st = as_stream(stream);
  constexpr int kH = 384;
  const int nsl = kH / kFwdUnits;
  for (int64_t s = 0; s < T; ++s) {
    const int ta = (int)s, tb = (int)(T - 1 - s);
    const FwdDir da{gates0, w_hh0, b_ih0, b_hh0, c0, act0, ta, ta - 1, batch_sizes[ta]};
    const FwdDir db{gates1, w_hh1, b_ih1, b_hh1, c1, act1, tb, tb + 1 < T ? tb + 1 : -1, batch_sizes[tb]};
    const int rbs = (int)ceil_div(std::max(da.bs, db.bs), kStepRows);
    if (rbs == 0) continue;
    bilstm_step_fwd_kernel<kH><<<dim3((unsigned)(nsl * rbs), 2), 64 * kFwdWaves, 0, st>>>((int)B, da, db, out);
  }
  return check_launch("bilstm_step_fwd_kernel");
}

extern "C" int mvml_bilstm_seq_bwd(int64_t T, int64_t B, int H, const int32_t* batch_sizes,
                                   const float* w_hhT0, const float* w_hhT1, const float* act0,
                                   const float* act1, const float* c0, const float* c1,
                                   const float* g_out, float* gg0, float* gg1, float* carry,
                                   void* stream) {
  clear_error();
  MVML_REQUIRE(T >= 0 && B > 0 && B <= (1 << 20) && H == 384 && batch_sizes,
               "bilstm_seq_bwd: bad shape (H = 384, MVP's blstm_dim; host batch_sizes)");
  for (int64_t t = 0; t < T; ++t)
    MVML_REQUIRE(batch_sizes[t] >= 0 && batch_sizes[t] <= B && (t == 0 || batch_sizes[t] <= batch_sizes[t - 1]),
                 "bilstm_seq_bwd: batch_sizes must be non-increasing in [0, B]");
  hipStream_t st = as_stream(stream);
  constexpr int kH = 384;
  const int nsl = kH / kBwdUnits;
  float* carry1 = carry + B * (int64_t)H;
  for (int64_t s = 0; s < T; ++s) {
    const int ta = (int)(T - 1 - s), tb = (int)s;  // forward direction walks back, reverse forth
    const int na = ta + 1 < T ? ta + 1 : -1, nb = tb - 1;
    const BwdDir da{w_hhT0, act0, c0, gg0, carry, ta, na, ta - 1, batch_sizes[ta],
                    na >= 0 ? batch_sizes[na] : 0};
    const BwdDir db{w_hhT1, act1, c1, gg1, carry1, tb, nb, tb + 1 < T ? tb + 1 : -1, batch_sizes[tb],
                    nb >= 0 ? batch_sizes[nb] : 0};
    const int rbs = (int)ceil_div(std::max(da.bs, db.bs), kStepRows);
    if (rbs == 0) continue;
    bilstm_step_bwd_kernel<kH><<<dim3((unsigned)(nsl * rbs), 2), 64 * kBwdWaves, 0, st>>>((int)B, da, db, g_out);
  }
  return check_launch("bilstm_step_bwd_kernel");
}

extern "C" int mvml_bilstm_select_last(int64_t B, int64_t H, const int32_t* lens,
                                       const int32_t* pos, float* out, float* fea, int dir,
                                       void* stream) {
  clear_error();
  MVML_REQUIRE(B >= 0 && H > 0 && (dir == 0 || dir == 1), "bilstm_select_last: bad args");
  if (B == 0) return MVML_OK;
  select_last_kernel<<<grid_1d(B * 2 * H), 256, 0, as_stream(stream)>>>(B, H, lens, pos, out,
                                                                         fea, dir);
  return check_launch("bilstm_select_last");
}

// ---- packed rows (wide batches) ------------------------------------------------------------
// The time-major [T, B, cols] buffers hold at step t only the live prefix of bs_t rows (the
// batch sorted by descending length); the products over every position (input projections,
// weight and input gradients) run over the N = sum_t bs_t live rows only: pack copies rows
// (t + shift, p) for t in [t0, t1), p < bs_t, into consecutive packed rows (offsets[t - t0] =
// sum_{t' < t} bs_t' over [t0, t)); unpack (dir 1) is the reverse copy.  A wave per row, float4.
namespace mvml {
namespace {
__global__ void __launch_bounds__(256) pack_rows_kernel(int64_t nrows, int64_t t_count, int64_t B,
                                                        int64_t cols4, const int32_t* __restrict__ offs,
                                                        int64_t t0, int shift, float4* __restrict__ tm,
                                                        int64_t ld_tm4, float4* __restrict__ pk,
                                                        int64_t ld_pk4, int dir) {
  // blockIdx.y = step k of the range, one wave per live row p of that step (no search over
  // the step offsets: a per-row binary search was a chain of dependent loads per wave)
  const int64_t lo = blockIdx.y;
  const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t rb = offs[lo];
  if (p >= offs[lo + 1] - rb) return;
  const int64_t r = rb + p;
  float4* a = tm + ((t0 + lo + shift) * B + p) * ld_tm4;
  float4* b = pk + r * ld_pk4;
  for (int64_t c = lane; c < cols4; c += 64) {
    if (dir == 0) b[c] = a[c];
    else a[c] = b[c];
  }
}
}  // namespace
}  // namespace mvml

extern "C" int mvml_bilstm_pack_rows(int64_t nrows, int64_t t_count, int64_t B, int64_t cols,
                                     const int32_t* offsets, int64_t t0, int shift, float* tm,
                                     int64_t ld_tm, float* packed, int64_t ld_pk, int dir,
                                     void* stream) {
  using namespace mvml;
  clear_error();
  MVML_REQUIRE(nrows >= 0 && t_count > 0 && B > 0 && cols > 0 && cols % 4 == 0 && ld_tm % 4 == 0 &&
                   ld_pk % 4 == 0 && ld_tm >= cols && ld_pk >= cols && (dir == 0 || dir == 1) &&
                   ((uintptr_t)tm & 15) == 0 && ((uintptr_t)packed & 15) == 0,
               "bilstm_pack_rows: bad shape / alignment");
  if (nrows == 0) return MVML_OK;
  MVML_REQUIRE(t_count <= 65535, "bilstm_pack_rows: t_count must be <= 65535");
  // a step holds at most B live rows (the packed sequence's batch sizes never exceed B)
  pack_rows_kernel<<<dim3((unsigned)ceil_div(std::min(nrows, B), 4), (unsigned)t_count), 256, 0,
                     as_stream(stream)>>>(
      nrows, t_count, B, cols / 4, offsets, t0, shift, reinterpret_cast<float4*>(tm), ld_tm / 4,
      reinterpret_cast<float4*>(packed), ld_pk / 4, dir);
  return check_launch("pack_rows_kernel");
}

// ---- embedding / layer-0 input-projection gradient over the packed live rows ----------------
// out[v, j] = sum of g[r, j] over the packed rows r whose token is v, r ascending (the packed
// order: t ascending, then sorted row ascending, as token_grad_kernel): chunks of kTokPChunk rows
// x 256-column slabs accumulate per token in LDS with 8 rows' loads in flight, then
// token_grad_sum_kernel adds the chunks in order (deterministic, no atomics).
namespace mvml {
namespace {
constexpr int kTokPChunk = 1024;
__global__ void __launch_bounds__(256)
token_grad_packed_kernel(int64_t nrows, int64_t cols, const float* __restrict__ g, int64_t ldg,
                         const int32_t* __restrict__ tok, int vocab, float* __restrict__ part) {
  __shared__ float s_acc[kTokMaxVocab][256];
  const int tid = threadIdx.x;
  const int64_t j = blockIdx.y * 256 + tid;
  const int64_t jc = min(j, cols - 1);  // lanes past the last column read a valid one, store nothing
  for (int v = 0; v < vocab; ++v) s_acc[v][tid] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * kTokPChunk, r1 = min<int64_t>(nrows, r0 + kTokPChunk);
  int64_t r = r0;
  for (; r + 8 <= r1; r += 8) {
    float x[8];
    int v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      x[u] = g[(r + u) * ldg + jc];
      v[u] = tok[r + u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s_acc[v[u]][tid] += x[u];  // one lane per column: no races
  }
  for (; r < r1; ++r) s_acc[tok[r]][tid] += g[r * ldg + jc];
  if (j < cols)
    for (int v = 0; v < vocab; ++v) part[((int64_t)blockIdx.x * vocab + v) * cols + j] = s_acc[v][tid];
}

// token of every packed live row: row offsets[t] + p is step t of sorted sequence p
__global__ void packed_tokens_kernel(int64_t nrows, int64_t T, const int32_t* __restrict__ offs,
                                     const int32_t* __restrict__ tokens, int64_t ldtok,
                                     const int32_t* __restrict__ perm, int32_t* __restrict__ tok) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  int64_t lo = 0, hi = T;
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (offs[mid] <= r) lo = mid; else hi = mid;
  }
  tok[r] = tokens[(int64_t)perm[r - offs[lo]] * ldtok + lo];
}
}  // namespace
}  // namespace mvml

extern "C" int mvml_bilstm_packed_tokens(int64_t nrows, int64_t T, const int32_t* offsets,
                                         const int32_t* tokens, int64_t ldtok, const int32_t* perm,
                                         int32_t* tok, void* stream) {
  clear_error();
  MVML_REQUIRE(nrows >= 0 && T > 0 && ldtok >= T, "bilstm_packed_tokens: bad shape");
  if (nrows == 0) return MVML_OK;
  packed_tokens_kernel<<<(unsigned)ceil_div(nrows, 256), 256, 0, as_stream(stream)>>>(
      nrows, T, offsets, tokens, ldtok, perm, tok);
  return check_launch("packed_tokens_kernel");
}

extern "C" int64_t mvml_bilstm_token_grad_packed_workspace(int64_t nrows, int64_t cols, int vocab) {
  return ceil_div(nrows > 0 ? nrows : 1, kTokPChunk) * vocab * cols * (int64_t)sizeof(float);
}

extern "C" int mvml_bilstm_token_grad_packed(int64_t nrows, int64_t cols, const float* g,
                                             int64_t ldg, const int32_t* tok, int vocab, float* out,
                                             void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  MVML_REQUIRE(nrows >= 0 && cols > 0 && ldg >= cols && vocab > 0 && vocab <= kTokMaxVocab,
               "bilstm_token_grad_packed: bad shape (vocab <= 64)");
  MVML_REQUIRE(workspace && (int64_t)workspace_bytes >= mvml_bilstm_token_grad_packed_workspace(nrows, cols, vocab),
               "bilstm_token_grad_packed: workspace too small");
  hipStream_t st = as_stream(stream);
  const int64_t nchunk = ceil_div(nrows > 0 ? nrows : 1, kTokPChunk);
  float* part = static_cast<float*>(workspace);
  if (nrows > 0) {
    token_grad_packed_kernel<<<dim3((unsigned)nchunk, (unsigned)ceil_div(cols, 256)), 256, 0, st>>>(
        nrows, cols, g, ldg, tok, vocab, part);
    int rc = check_launch("token_grad_packed_kernel");
    if (rc) return rc;
  } else {
    hipMemsetAsync(part, 0, (size_t)vocab * cols * sizeof(float), st);
  }
  const int64_t n = (int64_t)vocab * cols;
  token_grad_sum_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(nchunk, n, part, out);
  return check_launch("token_grad_sum_kernel");
}
