// SMILES BiLSTM view (RNNModule, /root/reference/model.py:98-135): the
// index kernels around the packed bidirectional LSTM.  The recurrence itself reuses the MFMA
// GEMM (h_prev W_hh^T per time step, beta = 1 onto the input projection) and the LSTM cell
// kernels of set2set.hip.
//
// Packed layout (what pack_padded_sequence(enforce_sorted=False) builds, model.py:128): the
// batch is ordered by descending length (perm[i] = original index of sorted row i) and stored
// time-major, row t*B + i, so the sequences alive at step t are the prefix i < batch_sizes[t].
//
// Layer 0's input projection is a table lookup: Embedding(tok) W_ih^T = (E W_ih^T)[tok], so the
// host computes P = E W_ih^T once ([V, 4H], V = 39 tokens) and mvml_bilstm_gather_rows expands
// it; the backward sums the gate gradients per token (mvml_bilstm_token_grad) and multiplies the
// [V, 4H] result into dE and dW_ih with two small GEMMs.
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

extern "C" int mvml_bilstm_token_grad(int64_t T, int64_t B, int64_t cols, const float* g,
                                      const int32_t* tokens, int64_t ldtok, const int32_t* lens,
                                      const int32_t* perm, int vocab, float* out, void* stream) {
  clear_error();
  MVML_REQUIRE(T >= 0 && B >= 0 && cols > 0 && vocab > 0 && ldtok >= T,
               "bilstm_token_grad: bad shape");
  dim3 grid(vocab, (unsigned)ceil_div(cols, 256));
  token_grad_kernel<<<grid, 256, 0, as_stream(stream)>>>(T, B, cols, g, tokens, ldtok, lens, perm,
                                                         out);
  return check_launch("bilstm_token_grad");
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
