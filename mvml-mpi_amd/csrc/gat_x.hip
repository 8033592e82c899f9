// GATConv re-associated for a narrow input (dgllife's first GATLayer, model.py:81: 74 atom
// features -> 4 heads x 192, flatten + ELU).  Aggregating the projected rows
//   rst_v,h = sum_e a_e,h (X[src_e] W_h^T) + X[v] Wres_h^T + b_h
// is the same sum re-associated as
//   rst_v,h = (sum_e a_e,h X[src_e]) W_h^T + X[v] Wres_h^T + b_h = [AX_h[v] | X[v]] [W_h | Wres_h]^T + b_h
// so the aggregation runs over the Fp = 76-wide feature rows (304 B) instead of the 1544-column
// projection (6.2 KB per atom written by a GEMM and read back), and one batched GEMM per head
// (K = 2 Fp) produces the layer output with bias + ELU in its epilogue (mvml_gemm_f16x2_ex).
// The attention logits need only el[n,h] = <X[n], A_l[h]>, A_l[h] = W_h^T attn_l[h] (the rows
// mvml_gat_fold_weights already appends to Wcat), so no projected row is ever formed.
//
// Backward (g_rst = dL/d rst, i.e. the ELU backward already applied — by the layer-2 data-gradient
// GEMM's epilogue or mvml_gat_elu_bwd):
//   dAX_h = g_rst_h W_h                                  (batched GEMM, mvml_gemm_f16x2_batched)
//   g_a_e,h = <dAX_h[dst_e], X[src_e]>  (= <g_rst_h[dst], Z_h[src]>)        mvml_gat_x_bwd
//   g_s = a (g_a - sum_v a g_a), g_pre = g_s leaky'(s_e), d er[v] = sum_in g_pre, d el[u] = sum_out g_pre
//   dL/d[W_h | Wres_h] = g_rst_h^T [AX_h | X], dL/d[A_l ; A_r] = [d el | d er]^T X   (GEMMs)
// with the same per-edge arithmetic order as gat_agg.hip's softmax_pair (edge order, expf,
// a = exp(s - max) / sum).
//
// Layout: X [N][Fp] (zero pad columns); AXc [N][H][2 Fp] = per head [AX_h | X] — the batched
// GEMM's A operand for head h is the column block h at row pitch 2 H Fp (X is stored once per
// head: one contiguous K = 2 Fp row per head, no two-segment K loop); per-row |max| bits of
// each head's block in arows [H][N] (the GEMM's per-row split-fp16 scales).
//
// Mapping: 16 lanes per atom, each lane owns float4 columns c and c + 16 of the feature row
// (Fp <= 128), four atoms per wave; every shuffle stays inside the atom's 16 lanes.
#include "common.h"

namespace mvml {
namespace {

constexpr int kXLanes = 16;
constexpr int kXThreads = 256;

__device__ __forceinline__ float leaky_x(float x, float slope) { return x > 0.f ? x : x * slope; }
__device__ __forceinline__ float4 ld4x(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4x(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float dot4x(float4 a, float4 b) {
  return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}
__device__ __forceinline__ float4 fma4x(float a, float4 x, float4 c) {
  return make_float4(fmaf(a, x.x, c.x), fmaf(a, x.y, c.y), fmaf(a, x.z, c.z), fmaf(a, x.w, c.w));
}
__device__ __forceinline__ float amax4x(float m, float4 v) {
  return fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
}
__device__ __forceinline__ float sum16(float v) {
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float max16(float v) {
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// el / er of every atom: elr[n] = [X[n] A_l^T | X[n] A_r^T] (Alr = [A_l ; A_r], 2H x Fp).
template <int H>
__global__ void __launch_bounds__(kXThreads) gat_x_elr_kernel(int64_t N, int Fp,
                                                              const float* __restrict__ X,
                                                              const float* __restrict__ Alr,
                                                              float* __restrict__ elr) {
  __shared__ __attribute__((aligned(16))) float s_a[2 * H * 128];
  for (int i = threadIdx.x; i < 2 * H * Fp; i += kXThreads) s_a[i] = Alr[i];
  __syncthreads();
  const int64_t n = (int64_t)blockIdx.x * (kXThreads / kXLanes) + threadIdx.x / kXLanes;
  const int l = threadIdx.x % kXLanes, nc = Fp / 4;
  if (n >= N) return;  // (whole 16-lane groups: the shuffles below stay inside live groups)
  float p[2 * H];
#pragma unroll
  for (int k = 0; k < 2 * H; ++k) p[k] = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int c = l + kXLanes * t;
    if (c < nc) {
      const float4 x = ld4x(X + n * Fp + 4 * c);
#pragma unroll
      for (int k = 0; k < 2 * H; ++k) p[k] += dot4x(x, ld4x(s_a + k * Fp + 4 * c));
    }
  }
#pragma unroll
  for (int k = 0; k < 2 * H; ++k) p[k] = sum16(p[k]);
  if (l == 0) {
#pragma unroll
    for (int k = 0; k < 2 * H; ++k) elr[n * 2 * H + k] = p[k];
  }
}

// Forward: edge softmax per (destination, head) in softmax_pair's order, then
// AX[v,h] = sum_e a_e,h X[src_e] and the GEMM operand block [AX_h | X] per head, with its per-row
// |max| bits; attn[e, h] (in-CSR slot order) for the backward.
// The atom's 16 lanes take its in-edges 16 at a time, one edge per lane (source id and logits
// loaded in parallel, not walked); the exp sums and the aggregation still run in edge order (each
// lane reads edge j's value by a shuffle), so the values are softmax_pair's bit for bit.
template <int H>
__global__ void __launch_bounds__(kXThreads) gat_x_fwd_kernel(
    int64_t N, int Fp, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ in_src,
    const float* __restrict__ X, const float* __restrict__ elr, float slope, float* __restrict__ attn,
    float* __restrict__ axc, uint32_t* __restrict__ arows) {
  const int64_t v = xcd_block(blockIdx.x, gridDim.x) * (kXThreads / kXLanes) + threadIdx.x / kXLanes;
  const int l = threadIdx.x % kXLanes, nc = Fp / 4;
  const int gb = (threadIdx.x & 63) & ~(kXLanes - 1);  // the atom's first lane in the wave
  if (v >= N) return;  // (whole 16-lane groups: every shuffle below stays inside a live group)
  float er[H];
  {
    const float* p = elr + v * 2 * H + H;
#pragma unroll
    for (int h = 0; h < H; ++h) er[h] = p[h];
  }
  const int eb = rowptr[v], ee = rowptr[v + 1];
  // logits of one 16-edge chunk, one edge per lane (-inf past the end)
  auto logits = [&](int base, int& src, float (&s)[H]) {
    const bool ok = base + l < ee;
    src = ok ? in_src[base + l] : 0;
    const float* el = elr + (int64_t)src * 2 * H;
#pragma unroll
    for (int h = 0; h < H; ++h) s[h] = ok ? leaky_x(el[h] + er[h], slope) : -INFINITY;
  };
  const bool one = ee - eb <= kXLanes;  // (group-uniform) the first chunk's logits are kept
  int src0;
  float s0[H], m[H], sum[H];
  logits(eb, src0, s0);
#pragma unroll
  for (int h = 0; h < H; ++h) { m[h] = s0[h]; sum[h] = 0.f; }
  for (int base = eb + kXLanes; base < ee; base += kXLanes) {
    int sr;
    float s[H];
    logits(base, sr, s);
#pragma unroll
    for (int h = 0; h < H; ++h) m[h] = fmaxf(m[h], s[h]);
  }
#pragma unroll
  for (int h = 0; h < H; ++h) m[h] = max16(m[h]);
  for (int base = eb; base < ee; base += kXLanes) {
    int sr;
    float s[H], x[H];
    if (one) {
#pragma unroll
      for (int h = 0; h < H; ++h) s[h] = s0[h];
    } else {
      logits(base, sr, s);
    }
#pragma unroll
    for (int h = 0; h < H; ++h) x[h] = expf(s[h] - m[h]);  // exp(-inf) = 0 past the end
    const int cnt = min(kXLanes, ee - base);
    for (int j = 0; j < cnt; ++j)
#pragma unroll
      for (int h = 0; h < H; ++h) sum[h] += __shfl(x[h], gb + j, 64);
  }
  const bool v1 = l + kXLanes < nc;
  float4 acc[H][2];
#pragma unroll
  for (int h = 0; h < H; ++h) acc[h][0] = acc[h][1] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int base = eb; base < ee; base += kXLanes) {
    int src;
    float s[H], a[H];
    if (one) {
      src = src0;
#pragma unroll
      for (int h = 0; h < H; ++h) s[h] = s0[h];
    } else {
      logits(base, src, s);
    }
#pragma unroll
    for (int h = 0; h < H; ++h) a[h] = expf(s[h] - m[h]) / sum[h];
    if (base + l < ee) {
#pragma unroll
      for (int h = 0; h < H; ++h) attn[(int64_t)(base + l) * H + h] = a[h];
    }
    const int cnt = min(kXLanes, ee - base);
    for (int j = 0; j < cnt; j += 2) {  // two source rows in flight
      const int j1 = min(j + 1, cnt - 1);
      const float* xr0 = X + (int64_t)__shfl(src, gb + j, 64) * Fp;
      const float* xr1 = X + (int64_t)__shfl(src, gb + j1, 64) * Fp;
      float aj0[H], aj1[H];
#pragma unroll
      for (int h = 0; h < H; ++h) { aj0[h] = __shfl(a[h], gb + j, 64); aj1[h] = __shfl(a[h], gb + j1, 64); }
      const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 x00 = l < nc ? ld4x(xr0 + 4 * l) : z4, x01 = v1 ? ld4x(xr0 + 4 * (l + kXLanes)) : z4;
      const float4 x10 = l < nc ? ld4x(xr1 + 4 * l) : z4, x11 = v1 ? ld4x(xr1 + 4 * (l + kXLanes)) : z4;
#pragma unroll
      for (int h = 0; h < H; ++h) { acc[h][0] = fma4x(aj0[h], x00, acc[h][0]); acc[h][1] = fma4x(aj0[h], x01, acc[h][1]); }
      if (j + 1 < cnt) {
#pragma unroll
        for (int h = 0; h < H; ++h) { acc[h][0] = fma4x(aj1[h], x10, acc[h][0]); acc[h][1] = fma4x(aj1[h], x11, acc[h][1]); }
      }
    }
  }
  const float* xv = X + v * Fp;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 xd0 = l < nc ? ld4x(xv + 4 * l) : z4;
  const float4 xd1 = v1 ? ld4x(xv + 4 * (l + kXLanes)) : z4;
  const float mx = amax4x(amax4x(0.f, xd0), xd1);
  float* row = axc + v * (2 * H * (int64_t)Fp);
#pragma unroll
  for (int h = 0; h < H; ++h) {
    float* blk = row + h * 2 * Fp;
    if (l < nc) { st4x(blk + 4 * l, acc[h][0]); st4x(blk + Fp + 4 * l, xd0); }
    if (v1) { st4x(blk + 4 * (l + kXLanes), acc[h][1]); st4x(blk + Fp + 4 * (l + kXLanes), xd1); }
    const float r = max16(amax4x(amax4x(mx, acc[h][0]), acc[h][1]));
    if (l == 0) arows[h * N + v] = __float_as_uint(r);
  }
}

// Backward, per destination: g_a per in-edge from dAX (a 16-lane dot per edge and head), then the
// softmax / LeakyReLU backward with one edge per lane: gpre[e] = g_pre, d er[v] -> gelr[v][H ..].
// Sums over the edges (sum a g_a, d er) run in edge order through shuffles, as the serial walk.
template <int H>
__global__ void __launch_bounds__(kXThreads) gat_x_bwd_kernel(
    int64_t N, int Fp, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ in_src,
    const float* __restrict__ X, const float* __restrict__ elr, const float* __restrict__ attn,
    float slope, const float* __restrict__ dax, float* __restrict__ gpre, float* __restrict__ gelr) {
  const int64_t v = xcd_block(blockIdx.x, gridDim.x) * (kXThreads / kXLanes) + threadIdx.x / kXLanes;
  const int l = threadIdx.x % kXLanes, nc = Fp / 4;
  const int gb = (threadIdx.x & 63) & ~(kXLanes - 1);
  if (v >= N) return;
  const bool v0 = l < nc, v1 = l + kXLanes < nc;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 d[H][2];
  const float* dr = dax + v * (H * (int64_t)Fp);
#pragma unroll
  for (int h = 0; h < H; ++h) {
    d[h][0] = v0 ? ld4x(dr + h * Fp + 4 * l) : z4;
    d[h][1] = v1 ? ld4x(dr + h * Fp + 4 * (l + kXLanes)) : z4;
  }
  const int eb = rowptr[v], ee = rowptr[v + 1];
  const bool one = ee - eb <= kXLanes;
  float S[H], er[H];
#pragma unroll
  for (int h = 0; h < H; ++h) { S[h] = 0.f; er[h] = elr[v * 2 * H + H + h]; }
  float ga0[H], a0[H];  // the first chunk's g_a and attention, one edge per lane
  int src0 = 0;
  for (int base = eb; base < ee; base += kXLanes) {
    const bool ok = base + l < ee;
    const int src = ok ? in_src[base + l] : 0;
    float ga[H], a[H];
#pragma unroll
    for (int h = 0; h < H; ++h) { ga[h] = 0.f; a[h] = ok ? attn[(int64_t)(base + l) * H + h] : 0.f; }
    const int cnt = min(kXLanes, ee - base);
    for (int j = 0; j < cnt; j += 2) {  // two source rows in flight
      const int j1 = min(j + 1, cnt - 1);
      const float* xr0 = X + (int64_t)__shfl(src, gb + j, 64) * Fp;
      const float* xr1 = X + (int64_t)__shfl(src, gb + j1, 64) * Fp;
      const float4 x00 = v0 ? ld4x(xr0 + 4 * l) : z4, x01 = v1 ? ld4x(xr0 + 4 * (l + kXLanes)) : z4;
      const float4 x10 = v0 ? ld4x(xr1 + 4 * l) : z4, x11 = v1 ? ld4x(xr1 + 4 * (l + kXLanes)) : z4;
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const float t0 = sum16(dot4x(d[h][0], x00) + dot4x(d[h][1], x01));
        const float t1 = sum16(dot4x(d[h][0], x10) + dot4x(d[h][1], x11));
        ga[h] = l == j ? t0 : l == j1 ? t1 : ga[h];
      }
    }
    for (int j = 0; j < cnt; ++j)
#pragma unroll
      for (int h = 0; h < H; ++h) S[h] += __shfl(a[h] * ga[h], gb + j, 64);
    if (base == eb) {
      src0 = src;
#pragma unroll
      for (int h = 0; h < H; ++h) { ga0[h] = ga[h]; a0[h] = a[h]; }
    }
    if (!one && ok) {
#pragma unroll
      for (int h = 0; h < H; ++h) gpre[(int64_t)(base + l) * H + h] = ga[h];
    }
  }
  float ger[H];
#pragma unroll
  for (int h = 0; h < H; ++h) ger[h] = 0.f;
  for (int base = eb; base < ee; base += kXLanes) {
    const bool ok = base + l < ee;
    int src;
    float ga[H], a[H];
    if (one) {
      src = src0;
#pragma unroll
      for (int h = 0; h < H; ++h) { ga[h] = ga0[h]; a[h] = a0[h]; }
    } else {
      src = ok ? in_src[base + l] : 0;
#pragma unroll
      for (int h = 0; h < H; ++h) {
        ga[h] = ok ? gpre[(int64_t)(base + l) * H + h] : 0.f;
        a[h] = ok ? attn[(int64_t)(base + l) * H + h] : 0.f;
      }
    }
    const float* el = elr + (int64_t)src * 2 * H;
    float gp[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float gs = a[h] * (ga[h] - S[h]);
      gp[h] = ok ? ((el[h] + er[h]) > 0.f ? gs : gs * slope) : 0.f;
    }
    if (ok) {
#pragma unroll
      for (int h = 0; h < H; ++h) gpre[(int64_t)(base + l) * H + h] = gp[h];
    }
    const int cnt = min(kXLanes, ee - base);
    for (int j = 0; j < cnt; ++j)
#pragma unroll
      for (int h = 0; h < H; ++h) ger[h] += __shfl(gp[h], gb + j, 64);
  }
  if (l == 0) {
#pragma unroll
    for (int h = 0; h < H; ++h) gelr[v * 2 * H + H + h] = ger[h];
  }
}

// d el[u] = sum over u's out-edges of g_pre (out-CSR order), and the |max| of u's [d el | d er]
// folded into *amax (block max, one unsigned atomicMax).
template <int H>
__global__ void __launch_bounds__(256) gat_x_gel_kernel(int64_t N, const int32_t* __restrict__ out_rowptr,
                                                        const int32_t* __restrict__ out_inslot,
                                                        const float* __restrict__ gpre,
                                                        float* __restrict__ gelr, uint32_t* amax) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float m = 0.f;
  if (u < N) {
    float g[H];
#pragma unroll
    for (int h = 0; h < H; ++h) g[h] = 0.f;
    for (int j = out_rowptr[u]; j < out_rowptr[u + 1]; ++j) {
      const float* p = gpre + (int64_t)out_inslot[j] * H;
#pragma unroll
      for (int h = 0; h < H; ++h) g[h] += p[h];
    }
#pragma unroll
    for (int h = 0; h < H; ++h) {
      gelr[u * 2 * H + h] = g[h];
      m = fmaxf(m, fmaxf(fabsf(g[h]), fabsf(gelr[u * 2 * H + H + h])));
    }
  }
  if (amax) {
    __shared__ float red[4];
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(amax, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
  }
}

// g_rst = g_out * ELU'(out) with ELU' = out > 0 ? 1 : out + 1 (torch elu_backward on the result),
// |max| folded into *amax.  The unfused fallback of the layer-2 GEMM epilogue (act 3).
__global__ void __launch_bounds__(256) gat_elu_bwd_kernel(int64_t total4, const float* __restrict__ g_out,
                                                          const float* __restrict__ out,
                                                          float* __restrict__ g_rst, uint32_t* amax) {
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 g = ld4x(g_out + 4 * i);
    const float4 o = ld4x(out + 4 * i);
    g.x *= o.x > 0.f ? 1.f : o.x + 1.f;
    g.y *= o.y > 0.f ? 1.f : o.y + 1.f;
    g.z *= o.z > 0.f ? 1.f : o.z + 1.f;
    g.w *= o.w > 0.f ? 1.f : o.w + 1.f;
    st4x(g_rst + 4 * i, g);
    m = amax4x(m, g);
  }
  __shared__ float red[4];
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0 && amax) atomicMax(amax, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

// [W_h | Wres_h] rows of the batched forward GEMM from Wcat = [fc.weight ; res_fc.weight ; ...]
// (both HF x Fp): Wb[r] = [Wcat[r] | Wcat[HF + r]], r < HF.
__global__ void __launch_bounds__(256) gat_x_pack_kernel(int64_t HF, int Fp, const float* __restrict__ Wcat,
                                                         float* __restrict__ Wb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HF * 2 * Fp) return;
  const int64_t r = i / (2 * Fp);
  const int c = (int)(i % (2 * Fp));
  Wb[i] = c < Fp ? Wcat[r * Fp + c] : Wcat[(HF + r) * Fp + (c - Fp)];
}

}  // namespace
}  // namespace mvml

using namespace mvml;

#define MVML_X_HEADS(H_, CALL) \
  switch (H_) {                \
    case 1: CALL(1); break;    \
    case 2: CALL(2); break;    \
    case 4: CALL(4); break;    \
    case 8: CALL(8); break;    \
    default: break;            \
  }

extern "C" int mvml_gat_x_supported(int H, int Fp) {
  return (H == 1 || H == 2 || H == 4 || H == 8) && Fp > 0 && Fp % 4 == 0 && Fp <= 4 * 2 * kXLanes;
}

extern "C" int mvml_gat_x_fwd(int64_t N, const int32_t* in_rowptr, const int32_t* in_src,
                              const float* X, int Fp, const float* Alr, int H, float slope,
                              float* elr, float* attn, float* axc, uint32_t* arows, void* stream) {
  clear_error();
  MVML_REQUIRE(N >= 0 && mvml_gat_x_supported(H, Fp), "gat_x_fwd: H in {1,2,4,8}, Fp %% 4 == 0, Fp <= 128");
  MVML_REQUIRE(N == 0 || (in_rowptr && in_src && X && Alr && elr && attn && axc && arows),
               "gat_x_fwd: null pointer");
  MVML_REQUIRE(((uintptr_t)X % 16) == 0 && ((uintptr_t)axc % 16) == 0 && ((uintptr_t)elr % 16) == 0,
               "gat_x_fwd: X / axc / elr must be 16-B aligned");
  if (N == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  const unsigned blocks = (unsigned)ceil_div(N, kXThreads / kXLanes);
#define MVML_X_ELR(HH) gat_x_elr_kernel<HH><<<blocks, kXThreads, 0, st>>>(N, Fp, X, Alr, elr)
  MVML_X_HEADS(H, MVML_X_ELR)
#undef MVML_X_ELR
  int rc = check_launch("gat_x_elr_kernel");
  if (rc) return rc;
#define MVML_X_FWD(HH) \
  gat_x_fwd_kernel<HH><<<blocks, kXThreads, 0, st>>>(N, Fp, in_rowptr, in_src, X, elr, slope, attn, axc, arows)
  MVML_X_HEADS(H, MVML_X_FWD)
#undef MVML_X_FWD
  return check_launch("gat_x_fwd_kernel");
}

extern "C" int mvml_gat_x_bwd(int64_t N, const int32_t* in_rowptr, const int32_t* in_src,
                              const int32_t* out_rowptr, const int32_t* out_inslot, const float* X,
                              int Fp, const float* elr, const float* attn, int H, float slope,
                              const float* dax, float* gpre, float* gelr, uint32_t* gelr_amax,
                              void* stream) {
  clear_error();
  MVML_REQUIRE(N >= 0 && mvml_gat_x_supported(H, Fp), "gat_x_bwd: H in {1,2,4,8}, Fp %% 4 == 0, Fp <= 128");
  MVML_REQUIRE(N == 0 || (in_rowptr && in_src && out_rowptr && out_inslot && X && elr && attn && dax &&
                          gpre && gelr), "gat_x_bwd: null pointer");
  MVML_REQUIRE(((uintptr_t)X % 16) == 0 && ((uintptr_t)dax % 16) == 0, "gat_x_bwd: X / dax must be 16-B aligned");
  if (N == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  const unsigned blocks = (unsigned)ceil_div(N, kXThreads / kXLanes);
#define MVML_X_BWD(HH) \
  gat_x_bwd_kernel<HH><<<blocks, kXThreads, 0, st>>>(N, Fp, in_rowptr, in_src, X, elr, attn, slope, dax, gpre, gelr)
  MVML_X_HEADS(H, MVML_X_BWD)
#undef MVML_X_BWD
  int rc = check_launch("gat_x_bwd_kernel");
  if (rc) return rc;
  const unsigned b2 = (unsigned)ceil_div(N, 256);
#define MVML_X_GEL(HH) gat_x_gel_kernel<HH><<<b2, 256, 0, st>>>(N, out_rowptr, out_inslot, gpre, gelr, gelr_amax)
  MVML_X_HEADS(H, MVML_X_GEL)
#undef MVML_X_GEL
  return check_launch("gat_x_gel_kernel");
}

extern "C" int mvml_gat_elu_bwd(int64_t n, const float* g_out, const float* out, float* g_rst,
                                uint32_t* amax, void* stream) {
  clear_error();
  MVML_REQUIRE(n >= 0 && n % 4 == 0, "gat_elu_bwd: n must be a multiple of 4");
  MVML_REQUIRE(n == 0 || (g_out && out && g_rst && ((uintptr_t)g_out % 16) == 0 &&
                          ((uintptr_t)out % 16) == 0 && ((uintptr_t)g_rst % 16) == 0),
               "gat_elu_bwd: null or unaligned pointer");
  if (n == 0) return MVML_OK;
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(n / 4, 256), 8192);
  gat_elu_bwd_kernel<<<blocks, 256, 0, as_stream(stream)>>>(n / 4, g_out, out, g_rst, amax);
  return check_launch("gat_elu_bwd_kernel");
}

extern "C" int mvml_gat_x_pack_weights(const float* Wcat, int H, int F, int Fp, float* Wb, void* stream) {
  clear_error();
  MVML_REQUIRE(H > 0 && F > 0 && Fp > 0 && Wcat && Wb, "gat_x_pack_weights: bad arguments");
  const int64_t HF = (int64_t)H * F, total = HF * 2 * Fp;
  gat_x_pack_kernel<<<(unsigned)ceil_div(total, 256), 256, 0, as_stream(stream)>>>(HF, Fp, Wcat, Wb);
  return check_launch("gat_x_pack_kernel");
}
