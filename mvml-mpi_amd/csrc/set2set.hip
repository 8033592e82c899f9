// Set2Set readout (dgl 0.9.1 Set2Set, model.py:82-84 and 92): LSTM cell pointwise kernels and
// the fused per-molecule segment pass (broadcast_nodes -> dot -> softmax_nodes -> sum_nodes).
//
// The LSTM gate GEMMs run on mvml_gemm_f32; these kernels apply the torch.nn.LSTM cell
// (gate order i, f, g, o):  c = sig(f)*c_prev + sig(i)*tanh(g);  h = sig(o)*tanh(c).
// The segment pass gives each molecule one wavefront that streams its atoms' 384-float rows
// once (online max/sum softmax), so the six Set2Set iterations read the node features six
// times in total, never materialising broadcast q or per-node products.
#include <numeric>

#include "common.h"

namespace mvml {
namespace {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float dot4(float4 a, float4 b) {
  return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}

__global__ void lstm_cell_fwd_kernel(int64_t B, int D, const float* __restrict__ gp,
                                     const float* __restrict__ b_ih, const float* __restrict__ b_hh,
                                     const float* __restrict__ c_prev, float* __restrict__ c_out,
                                     float* __restrict__ h_out, int64_t ldh, float* __restrict__ act,
                                     float* __restrict__ h_out2, int64_t ldh2) {
  const int64_t total = B * D;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / D;
    const int d = (int)(e - b * D);
    // gp NULL: the pre-activations are zero (Set2Set's first cell: q*_{-1} = 0, h(-1) = 0);
    // 0 + b_ih + b_hh rounds as the zero-filled buffer did
    const float* g = gp ? gp + b * 4 * D : nullptr;
    const float gi = (g ? g[d] : 0.f) + b_ih[d] + b_hh[d];
    const float gf = (g ? g[D + d] : 0.f) + b_ih[D + d] + b_hh[D + d];
    const float gg = (g ? g[2 * D + d] : 0.f) + b_ih[2 * D + d] + b_hh[2 * D + d];
    const float go = (g ? g[3 * D + d] : 0.f) + b_ih[3 * D + d] + b_hh[3 * D + d];
    const float i = sigm(gi), f = sigm(gf), gt = tanhf(gg), o = sigm(go);
    const float cp = c_prev ? c_prev[e] : 0.f;
    // explicit rounding (no contraction choice left to the compiler): the split-fp16 GEMM's
    // cell epilogue (gemm_f32.hip, CellEpi) uses the same two operations, bit for bit
    const float c = __fmaf_rn(f, cp, __fmul_rn(i, gt));
    c_out[e] = c;
    const float h = __fmul_rn(o, tanhf(c));
    h_out[b * ldh + d] = h;
    if (h_out2) h_out2[b * ldh2 + d] = h;
    float* a = act + b * 4 * D;
    a[d] = i;
    a[D + d] = f;
    a[2 * D + d] = gt;
    a[3 * D + d] = o;
  }
}

// gb_part (optional): the gate gradients' column sums of this thread's rows, i.e. the partial
// bias gradient.  The host sizes the grid so that gridDim * 256 = R D (mvml_lstm_cell_bwd_
// part_rows): thread gid then always sees unit d = gid % D, rows gid / D + j R, and writes its
// four gate sums to row gid / D of the [R][4 D] partial (summed over rows and time steps by one
// column-sum pass afterwards — instead of a pass over all T x B gate-gradient rows).
__global__ void lstm_cell_bwd_kernel(int64_t B, int D, const float* __restrict__ act,
                                     const float* __restrict__ c, const float* __restrict__ c_prev,
                                     const float* __restrict__ g_h, int64_t ldgh,
                                     const float* __restrict__ g_h2, int64_t ldgh2,
                                     const float* __restrict__ g_c, float* __restrict__ g_gates,
                                     float* __restrict__ g_c_prev, uint32_t* __restrict__ gg_amax,
                                     float* __restrict__ gb_part) {
  const int64_t total = B * D;
  float mx = 0.f;  // |max| of this thread's gate gradients (split-fp16 operand scale)
  float sb[4] = {0.f, 0.f, 0.f, 0.f};  // gb_part: this thread's gate column sums
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / D;
    const int d = (int)(e - b * D);
    const float* a = act + b * 4 * D;
    const float i = a[d], f = a[D + d], gt = a[2 * D + d], o = a[3 * D + d];
    // dL/dh from its two consumers (the next layer's input, the next step's recurrence): the
    // sum autograd would form with a separate add, formed here
    const float gh = g_h2 ? g_h[b * ldgh + d] + g_h2[b * ldgh2 + d] : g_h[b * ldgh + d];
    const float tc = tanhf(c[e]);
    const float gc = (g_c ? g_c[e] : 0.f) + gh * o * (1.f - tc * tc);
    const float cp = c_prev ? c_prev[e] : 0.f;
    float* gg = g_gates + b * 4 * D;
    const float g0 = gc * gt * i * (1.f - i), g1 = gc * cp * f * (1.f - f);
    const float g2 = gc * i * (1.f - gt * gt), g3 = gh * tc * o * (1.f - o);
    gg[d] = g0;
    gg[D + d] = g1;
    gg[2 * D + d] = g2;
    gg[3 * D + d] = g3;
    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(g0), fabsf(g1)), fmaxf(fabsf(g2), fabsf(g3))));
    if (g_c_prev) g_c_prev[e] = gc * f;
    sb[0] += g0;
    sb[1] += g1;
    sb[2] += g2;
    sb[3] += g3;
  }
  if (gb_part) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r0 = gid / D, d = gid - r0 * D;
    float* pr = gb_part + r0 * 4 * D + d;
#pragma unroll
    for (int q = 0; q < 4; ++q) pr[q * D] = sb[q];
  }
  if (gg_amax) {  // block max -> one unsigned atomicMax of the non-negative float bits
    mx = wave_max(mx);
    __shared__ float red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0)
      atomicMax(gg_amax, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
  }
}

// One wave per molecule; lane holds float4 column groups col = 4*(lane + 64*c).
template <int NV>
__global__ void __launch_bounds__(256)
seg_fwd_kernel(int64_t B, int D, const int64_t* __restrict__ node_off, const float* __restrict__ X,
               float* __restrict__ qstar, int64_t ldq, float* __restrict__ lse) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= B) return;
  const int64_t n0 = node_off[g], n1 = node_off[g + 1];
  float4 q[NV], r[NV];
  bool ok[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int col = 4 * (lane + 64 * c);
    ok[c] = col < D;
    q[c] = ok[c] ? ld4(qstar + g * ldq + col) : make_float4(0, 0, 0, 0);
    r[c] = make_float4(0, 0, 0, 0);
  }
  float m = -INFINITY, s = 0.f;
  for (int64_t n = n0; n < n1; ++n) {
    float4 x[NV];
    float part = 0.f;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      x[c] = ok[c] ? ld4(X + n * D + 4 * (lane + 64 * c)) : make_float4(0, 0, 0, 0);
      part += dot4(x[c], q[c]);
    }
    const float e = wave_sum(part);
    const float mn = fmaxf(m, e);
    const float sc = expf(m - mn);
    const float p = expf(e - mn);
    s = s * sc + p;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      r[c].x = r[c].x * sc + p * x[c].x;
      r[c].y = r[c].y * sc + p * x[c].y;
      r[c].z = r[c].z * sc + p * x[c].z;
      r[c].w = r[c].w * sc + p * x[c].w;
    }
    m = mn;
  }
  const float inv = (n1 > n0) ? 1.f / s : 0.f;
#pragma unroll
  for (int c = 0; c < NV; ++c)
    if (ok[c])
      st4(qstar + g * ldq + D + 4 * (lane + 64 * c),
          make_float4(r[c].x * inv, r[c].y * inv, r[c].z * inv, r[c].w * inv));
  if (lane == 0) lse[g] = (n1 > n0) ? m + logf(s) : -INFINITY;
}

template <int NV>
__global__ void __launch_bounds__(256)
seg_bwd_kernel(int64_t B, int D, const int64_t* __restrict__ node_off, const float* __restrict__ X,
               const float* __restrict__ qstar, int64_t ldq, const float* __restrict__ lse,
               const float* g_qstar, int64_t ldgq, float* g_q,
               int64_t ldgout, float* __restrict__ alpha, float* __restrict__ g_e) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= B) return;
  const int64_t n0 = node_off[g], n1 = node_off[g + 1];
  float4 q[NV], gr[NV], gq[NV];
  bool ok[NV];
  float cpart = 0.f;
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int col = 4 * (lane + 64 * c);
    ok[c] = col < D;
    q[c] = ok[c] ? ld4(qstar + g * ldq + col) : make_float4(0, 0, 0, 0);
    gr[c] = ok[c] ? ld4(g_qstar + g * ldgq + D + col) : make_float4(0, 0, 0, 0);
    const float4 rr = ok[c] ? ld4(qstar + g * ldq + D + col) : make_float4(0, 0, 0, 0);
    cpart += dot4(rr, gr[c]);
    gq[c] = make_float4(0, 0, 0, 0);
  }
  const float cdot = wave_sum(cpart);  // sum_n alpha_n <x_n, g_r> = <r, g_r>
  const float L = lse[g];
  for (int64_t n = n0; n < n1; ++n) {
    float4 x[NV];
    float pe = 0.f, pa = 0.f;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      x[c] = ok[c] ? ld4(X + n * D + 4 * (lane + 64 * c)) : make_float4(0, 0, 0, 0);
      pe += dot4(x[c], q[c]);
      pa += dot4(x[c], gr[c]);
    }
    const float e = wave_sum(pe);
    const float ga = wave_sum(pa);
    const float al = expf(e - L);
    const float ge = al * (ga - cdot);
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      gq[c].x += ge * x[c].x;
      gq[c].y += ge * x[c].y;
      gq[c].z += ge * x[c].z;
      gq[c].w += ge * x[c].w;
    }
    if (lane == 0) {
      alpha[n] = al;
      g_e[n] = ge;
    }
  }
#pragma unroll
  for (int c = 0; c < NV; ++c)
    if (ok[c]) {
      const int col = 4 * (lane + 64 * c);
      const float4 gd = ld4(g_qstar + g * ldgq + col);
      st4(g_q + g * ldgout + col,
          make_float4(gd.x + gq[c].x, gd.y + gq[c].y, gd.z + gq[c].z, gd.w + gq[c].w));
    }
}

// One wave per node: gX[n] = sum_t alpha_t[n] * g_r_t[g] + g_e_t[n] * q_t[g].
template <int NV>
__global__ void __launch_bounds__(256)
seg_gx_kernel(int64_t N, int D, int T, const int32_t* __restrict__ node_graph,
              const float* __restrict__ qstars, int64_t ldq, int64_t qs_stride,
              const float* __restrict__ g_qstars, int64_t ldgq, int64_t gqs_stride,
              const float* __restrict__ alphas, const float* __restrict__ g_es,
              float* __restrict__ gX) {
  const int lane = threadIdx.x & 63;
  const int64_t n = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  const int64_t g = node_graph[n];
  float4 acc[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) acc[c] = make_float4(0, 0, 0, 0);
  for (int t = 0; t < T; ++t) {
    const float al = alphas[(int64_t)t * N + n];
    const float ge = g_es[(int64_t)t * N + n];
    const float* q = qstars + t * qs_stride + g * ldq;
    const float* gr = g_qstars + t * gqs_stride + g * ldgq + D;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int col = 4 * (lane + 64 * c);
      if (col < D) {
        const float4 a = ld4(gr + col), b = ld4(q + col);
        acc[c].x += al * a.x + ge * b.x;
        acc[c].y += al * a.y + ge * b.y;
        acc[c].z += al * a.z + ge * b.z;
        acc[c].w += al * a.w + ge * b.w;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int col = 4 * (lane + 64 * c);
    if (col < D) st4(gX + n * D + col, acc[c]);
  }
}

// The same sum with one wave per MOLECULE: its 2 T vectors q_t, g_r_t are loaded once into
// registers (shared by all its atoms), the per-atom coefficients alpha_t[n], g_e_t[n] are loaded
// 64 atoms at a time with the lanes on the atoms (coalesced), and each atom's row is formed from
// its coefficients broadcast by v_readlane — no per-atom chain of dependent global loads (the
// node-per-wave kernel above walked T of them per atom: latency-bound at ~1.1 TB/s of gX).
// T <= kGxT; the same per-element expression and t order as seg_gx_kernel.
constexpr int kGxT = 6;
template <int NV>
__global__ void __launch_bounds__(256)
seg_gx_mol_kernel(int64_t B, int D, int T, const int64_t* __restrict__ node_off,
                  const float* __restrict__ qstars, int64_t ldq, int64_t qs_stride,
                  const float* __restrict__ g_qstars, int64_t ldgq, int64_t gqs_stride,
                  const float* __restrict__ alphas, const float* __restrict__ g_es, int64_t N,
                  float* __restrict__ gX) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= B) return;
  const int64_t n0 = node_off[g], n1 = node_off[g + 1];
  float4 qv[kGxT][NV], gv[kGxT][NV];
#pragma unroll
  for (int t = 0; t < kGxT; ++t)
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int col = 4 * (lane + 64 * c);
      const bool ok = t < T && col < D;
      qv[t][c] = ok ? ld4(qstars + t * qs_stride + g * ldq + col) : make_float4(0, 0, 0, 0);
      gv[t][c] = ok ? ld4(g_qstars + t * gqs_stride + g * ldgq + D + col) : make_float4(0, 0, 0, 0);
    }
  for (int64_t base = n0; base < n1; base += 64) {
    const int64_t n = base + lane;
    const bool live = n < n1;
    float al[kGxT], ge[kGxT];
#pragma unroll
    for (int t = 0; t < kGxT; ++t) {
      al[t] = (live && t < T) ? alphas[(int64_t)t * N + n] : 0.f;
      ge[t] = (live && t < T) ? g_es[(int64_t)t * N + n] : 0.f;
    }
    const int cnt = (int)min<int64_t>(64, n1 - base);
    for (int i = 0; i < cnt; ++i) {
      float4 acc[NV];
#pragma unroll
      for (int c = 0; c < NV; ++c) acc[c] = make_float4(0, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < kGxT; ++t) {
        if (t >= T) break;  // uniform
        const float a_ = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(al[t]), i));
        const float e_ = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ge[t]), i));
#pragma unroll
        for (int c = 0; c < NV; ++c) {
          const float4 a = gv[t][c], b = qv[t][c];
          acc[c].x += a_ * a.x + e_ * b.x;
          acc[c].y += a_ * a.y + e_ * b.y;
          acc[c].z += a_ * a.z + e_ * b.z;
          acc[c].w += a_ * a.w + e_ * b.w;
        }
      }
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        const int col = 4 * (lane + 64 * c);
        if (col < D) st4(gX + (base + i) * D + col, acc[c]);
      }
    }
  }
}

// out[b] = max(floor, max over the molecule's atoms of in[n]) on non-negative float bits (an
// integer max): one thread per molecule, the atoms' row maxima read in order.
__global__ void __launch_bounds__(256) segment_max_bits_kernel(int64_t B, const int64_t* __restrict__ offs,
                                                               const uint32_t* __restrict__ in,
                                                               uint32_t floor_bits, uint32_t* __restrict__ out) {
  for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < B; b += (int64_t)gridDim.x * 256) {
    uint32_t m = floor_bits;
    for (int64_t n = offs[b]; n < offs[b + 1]; ++n) m = max(m, in[n]);
    out[b] = m;
  }
}

unsigned grid_for(int64_t total) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(total, 256), 16384));
}

int check_d(int D, const char* who) {
  MVML_REQUIRE(D > 0 && D % 4 == 0 && D <= 1024, "%s: feature size must be a multiple of 4 <= 1024 (got %d)", who, D);
  return MVML_OK;
}

}  // namespace
}  // namespace mvml

using namespace mvml;

#define MVML_NV_SWITCH(KERNEL, GRID, ...)                                                   \
  switch ((int)ceil_div(D, 256)) {                                                          \
    case 1: KERNEL<1><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                            \
    case 2: KERNEL<2><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                            \
    case 3: KERNEL<3><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                            \
    default: KERNEL<4><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                           \
  }

extern "C" int mvml_segment_max_bits(int64_t B, const int64_t* node_offsets, const uint32_t* in_bits,
                                     uint32_t floor_bits, uint32_t* out_bits, void* stream) {
  clear_error();
  MVML_REQUIRE(B >= 0 && (B == 0 || (node_offsets && in_bits && out_bits)), "segment_max_bits: bad args");
  if (B == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  segment_max_bits_kernel<<<grid_for(B), 256, 0, st>>>(B, node_offsets, in_bits, floor_bits, out_bits);
  return check_launch("segment_max_bits_kernel");
}

extern "C" int mvml_lstm_cell_fwd(int64_t B, int D, const float* gates_pre, const float* b_ih,
                                  const float* b_hh, const float* c_prev, float* c_out,
                                  float* h_out, int64_t ldh, float* act_out, float* h_out2,
                                  int64_t ldh2, void* stream) {
  clear_error();
  MVML_REQUIRE(B >= 0 && D > 0 && ldh >= D && (!h_out2 || ldh2 >= D), "lstm_cell_fwd: bad shape");
  if (B == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  lstm_cell_fwd_kernel<<<grid_for(B * D), 256, 0, st>>>(B, D, gates_pre, b_ih, b_hh, c_prev, c_out,
                                                        h_out, ldh, act_out, h_out2, ldh2);
  return check_launch("lstm_cell_fwd_kernel");
}

// Rows of the bias-gradient partial of mvml_lstm_cell_bwd: R with R D % 256 == 0 and about 16
// rows of B per thread (the amax fold's grain).
static int64_t cell_bwd_part_rows(int64_t B, int D) {
  const int64_t step = 256 / std::gcd<int64_t>(D, 256);  // smallest R with R D % 256 == 0
  return std::max<int64_t>(step, ceil_div(ceil_div(B, 16), step) * step);
}
extern "C" int64_t mvml_lstm_cell_bwd_part_rows(int64_t B, int D) {
  return (B > 0 && D > 0) ? cell_bwd_part_rows(B, D) : 0;
}

extern "C" int mvml_lstm_cell_bwd(int64_t B, int D, const float* act, const float* c,
                                  const float* c_prev, const float* g_h, int64_t ldgh,
                                  const float* g_h2, int64_t ldgh2,
                                  const float* g_c, float* g_gates, float* g_c_prev,
                                  uint32_t* gg_amax, float* gb_part, void* stream) {
  clear_error();
  MVML_REQUIRE(B >= 0 && D > 0 && ldgh >= D && (!g_h2 || ldgh2 >= D), "lstm_cell_bwd: bad shape");
  if (B == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  if (gb_part) {  // grid * 256 = R D: every thread keeps one unit (see the kernel)
    const int64_t R = cell_bwd_part_rows(B, D);
    lstm_cell_bwd_kernel<<<(unsigned)(R * D / 256), 256, 0, st>>>(B, D, act, c, c_prev, g_h, ldgh,
                                                                  g_h2, ldgh2, g_c, g_gates, g_c_prev,
                                                                  gg_amax, gb_part);
    return check_launch("lstm_cell_bwd_kernel");
  }
  // with gg_amax, one atomicMax per workgroup on a single word: a short kernel whose thousands
  // of workgroups end together saturates it (~88 per us), so each thread takes >= 16 elements
  // (MVP's 8k-row cells: 768 workgroups instead of 12k; Set2Set's 64k-row cells: 6k)
  const unsigned grid = gg_amax ? (unsigned)std::min<int64_t>(
                                      grid_for(B * D), std::max<int64_t>(256, ceil_div(B * D, 4096)))
                                : grid_for(B * D);
  lstm_cell_bwd_kernel<<<grid, 256, 0, st>>>(B, D, act, c, c_prev, g_h, ldgh, g_h2, ldgh2, g_c,
                                             g_gates, g_c_prev, gg_amax, nullptr);
  return check_launch("lstm_cell_bwd_kernel");
}

extern "C" int mvml_set2set_seg_fwd(int64_t B, int D, const int64_t* node_offsets, const float* X,
                                    float* qstar, int64_t ldq, float* lse, void* stream) {
  clear_error();
  int rc = check_d(D, "set2set_seg_fwd");
  if (rc) return rc;
  MVML_REQUIRE(ldq >= 2 * D && ldq % 4 == 0, "set2set_seg_fwd: bad ldq");
  if (B == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)ceil_div(B, 4);
  MVML_NV_SWITCH(seg_fwd_kernel, grid, B, D, node_offsets, X, qstar, ldq, lse)
  return check_launch("seg_fwd_kernel");
}

extern "C" int mvml_set2set_seg_bwd(int64_t B, int D, const int64_t* node_offsets, const float* X,
                                    const float* qstar, int64_t ldq, const float* lse,
                                    const float* g_qstar, int64_t ldgq, float* g_q,
                                    int64_t ldgout, float* alpha, float* g_e, void* stream) {
  clear_error();
  int rc = check_d(D, "set2set_seg_bwd");
  if (rc) return rc;
  MVML_REQUIRE(ldq >= 2 * D && ldgq >= 2 * D && ldgout >= D, "set2set_seg_bwd: bad ld");
  if (B == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)ceil_div(B, 4);
  MVML_NV_SWITCH(seg_bwd_kernel, grid, B, D, node_offsets, X, qstar, ldq, lse, g_qstar, ldgq, g_q,
                 ldgout, alpha, g_e)
  return check_launch("seg_bwd_kernel");
}

extern "C" int mvml_set2set_gx(int64_t num_nodes, int D, int T, const int32_t* node_graph,
                               const int64_t* node_offsets, int64_t num_graphs,
                               const float* qstars, int64_t ldq, int64_t qstar_stride,
                               const float* g_qstars, int64_t ldgq, int64_t g_qstar_stride,
                               const float* alphas, const float* g_es, float* gX, void* stream) {
  clear_error();
  int rc = check_d(D, "set2set_gx");
  if (rc) return rc;
  MVML_REQUIRE(T >= 0 && ldq >= 2 * D && ldgq >= 2 * D, "set2set_gx: bad shape");
  if (num_nodes == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  if (node_offsets && num_graphs > 0 && T <= kGxT && D <= 512) {  // one wave per molecule
    const unsigned grid = (unsigned)ceil_div(num_graphs, 4);
    if (D <= 256)
      seg_gx_mol_kernel<1><<<grid, 256, 0, st>>>(num_graphs, D, T, node_offsets, qstars, ldq,
                                                 qstar_stride, g_qstars, ldgq, g_qstar_stride,
                                                 alphas, g_es, num_nodes, gX);
    else
      seg_gx_mol_kernel<2><<<grid, 256, 0, st>>>(num_graphs, D, T, node_offsets, qstars, ldq,
                                                 qstar_stride, g_qstars, ldgq, g_qstar_stride,
                                                 alphas, g_es, num_nodes, gX);
    return check_launch("seg_gx_mol_kernel");
  }
  MVML_REQUIRE(node_graph != nullptr, "set2set_gx: node_graph or node_offsets required");
  const unsigned grid = (unsigned)ceil_div(num_nodes, 4);
  MVML_NV_SWITCH(seg_gx_kernel, grid, num_nodes, D, T, node_graph, qstars, ldq, qstar_stride,
                 g_qstars, ldgq, g_qstar_stride, alphas, g_es, gX)
  return check_launch("seg_gx_kernel");
}
