// Multi-view attention fusion head of MVP (model.py:28-48, 57-71), the consumer of the graph
// view: shared LayerNorm(384) on the three view embeddings, Q/K/V projection
// (three bias-free Linear(384 -> 12 x 384), one GEMM), attention over the 3 view tokens per head,
// Conv2d(12, 12, 3) + ReLU over the (head, token, feature) cube, MLP 4584 -> 1024 -> 11, and
// BCEWithLogitsLoss (main.py:91).  The GEMMs go through mvml_gemm_f32x3; this file holds the
// non-GEMM kernels and their backward:
//   * LayerNorm rows: one wave per row, two-pass statistics in registers.
//   * token attention: one wave per (molecule, head); the 3x3 scores are nine wave dot
//     products, the softmax is lane-local, the 384-wide rows stream once (HBM bound).
//   * 3x3 convolution: one workgroup per molecule stages the (12, 3, 384) cube in LDS; a thread
//     per output column computes all 12 output channels (weights as uniform LDS broadcasts).
//     Weight gradients: per-workgroup partials over a run of molecules, summed in fixed order
//     by a second kernel (deterministic, no atomics).
#include "common.h"
#include "dropout.h"

namespace mvml {
namespace {

constexpr int kFuseMaxVpl = 8;  // LayerNorm rows up to 512 wide

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// LayerNorm (torch.nn.LayerNorm, biased variance, eps inside the sqrt), one wave per row.
__global__ void __launch_bounds__(256)
layernorm_fwd_kernel(int64_t rows, int D, const float* __restrict__ x, int64_t ldx,
                     const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                     float* __restrict__ y, int64_t ldy, float* __restrict__ mean_out,
                     float* __restrict__ rstd_out) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  float v[kFuseMaxVpl];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kFuseMaxVpl; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < D ? x[r * ldx + c] : 0.f;
    s += v[i];
  }
  const float mean = wsum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < kFuseMaxVpl; ++i) {
    const int c = lane + 64 * i;
    const float d = c < D ? v[i] - mean : 0.f;
    q += d * d;
  }
  const float rstd = 1.f / sqrtf(wsum(q) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < kFuseMaxVpl; ++i) {
    const int c = lane + 64 * i;
    if (c < D) y[r * ldy + c] = (v[i] - mean) * rstd * gamma[c] + beta[c];
  }
  if (lane == 0) {
    mean_out[r] = mean;
    rstd_out[r] = rstd;
  }
}

// g_x = rstd * (g_xh - mean(g_xh) - xh * mean(g_xh * xh)), g_xh = g_y * gamma;
// gxh_out = g_y * xh (its column sums are dL/dgamma; column sums of g_y are dL/dbeta).
__global__ void __launch_bounds__(256)
layernorm_bwd_kernel(int64_t rows, int D, const float* __restrict__ x, int64_t ldx,
                     const float* __restrict__ gamma, const float* __restrict__ mean_in,
                     const float* __restrict__ rstd_in, const float* __restrict__ gy,
                     int64_t ldgy, float* __restrict__ gx, int64_t ldgx,
                     float* __restrict__ gyxh) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float mean = mean_in[r], rstd = rstd_in[r];
  float xh[kFuseMaxVpl], g[kFuseMaxVpl];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < kFuseMaxVpl; ++i) {
    const int c = lane + 64 * i;
    xh[i] = c < D ? (x[r * ldx + c] - mean) * rstd : 0.f;
    const float gyv = c < D ? gy[r * ldgy + c] : 0.f;
    g[i] = c < D ? gyv * gamma[c] : 0.f;
    if (c < D) gyxh[r * D + c] = gyv * xh[i];
    s1 += g[i];
    s2 += g[i] * xh[i];
  }
  const float m1 = wsum(s1) / (float)D, m2 = wsum(s2) / (float)D;
#pragma unroll
  for (int i = 0; i < kFuseMaxVpl; ++i) {
    const int c = lane + 64 * i;
    if (c < D) gx[r * ldgx + c] = rstd * (g[i] - m1 - xh[i] * m2);
  }
}

// Attention over the NT = 3 view tokens of one molecule, per head (model.py:62-68):
//   q/k/v of token t = QKV row 3b+t, columns [h*dk | HD + h*dk | 2HD + h*dk] (dk wide)
//   s_ij = <q_i, k_j> * scale;  p = softmax_j(s);  att[b][h][i] = sum_j p_ij v_j
constexpr int NT = 3;
constexpr int kDkVpl = 6;  // dk = 384 = 6 x 64

__global__ void __launch_bounds__(256)
token_attn_fwd_kernel(int64_t B, int H, int dk, const float* __restrict__ qkv, int64_t ld,
                      float scale, float* __restrict__ att, float* __restrict__ P) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= B * H) return;
  const int64_t b = w / H;
  const int h = (int)(w % H);
  const int64_t HD = (int64_t)H * dk;
  float q[NT][kDkVpl], k[NT][kDkVpl], v[NT][kDkVpl];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const float* row = qkv + (b * NT + t) * ld + (int64_t)h * dk;
#pragma unroll
    for (int i = 0; i < kDkVpl; ++i) {
      const int c = lane + 64 * i;
      q[t][i] = row[c];
      k[t][i] = row[HD + c];
      v[t][i] = row[2 * HD + c];
    }
  }
  float p[NT][NT];
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < kDkVpl; ++i) s = fmaf(q[a][i], k[c][i], s);
      p[a][c] = wsum(s) * scale;
    }
#pragma unroll
  for (int a = 0; a < NT; ++a) {
    const float m = fmaxf(p[a][0], fmaxf(p[a][1], p[a][2]));
    float z = 0.f;
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      p[a][c] = expf(p[a][c] - m);
      z += p[a][c];
    }
#pragma unroll
    for (int c = 0; c < NT; ++c) p[a][c] /= z;
  }
  float* out = att + w * NT * dk;
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int i = 0; i < kDkVpl; ++i) {
      float o = 0.f;
#pragma unroll
      for (int c = 0; c < NT; ++c) o = fmaf(p[a][c], v[c][i], o);
      out[a * dk + lane + 64 * i] = o;
    }
  if (lane < NT * NT) {
    float pv = p[0][0];
#pragma unroll
    for (int e = 1; e < NT * NT; ++e) pv = lane == e ? p[e / NT][e % NT] : pv;
    P[w * NT * NT + lane] = pv;
  }
}

// Backward of token_attn_fwd: g_v_j = sum_i p_ij g_i;  g_p_ij = <g_i, v_j>;
// g_s_ij = p_ij (g_p_ij - sum_j' p_ij' g_p_ij');  g_q_i = scale sum_j g_s_ij k_j;
// g_k_j = scale sum_i g_s_ij q_i.  gqkv has the layout of qkv.
__global__ void __launch_bounds__(256)
token_attn_bwd_kernel(int64_t B, int H, int dk, const float* __restrict__ qkv, int64_t ld,
                      float scale, const float* __restrict__ P, const float* __restrict__ g_att,
                      float* __restrict__ gqkv, int64_t ldg) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= B * H) return;
  const int64_t b = w / H;
  const int h = (int)(w % H);
  const int64_t HD = (int64_t)H * dk;
  float p[NT][NT];
#pragma unroll
  for (int e = 0; e < NT * NT; ++e) p[e / NT][e % NT] = P[w * NT * NT + e];
  float g[NT][kDkVpl], v[NT][kDkVpl];
  const float* ga = g_att + w * NT * dk;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const float* row = qkv + (b * NT + t) * ld + (int64_t)h * dk;
#pragma unroll
    for (int i = 0; i < kDkVpl; ++i) {
      const int c = lane + 64 * i;
      g[t][i] = ga[t * dk + c];
      v[t][i] = row[2 * HD + c];
    }
  }
  float gs[NT][NT];
#pragma unroll
  for (int a = 0; a < NT; ++a) {
    float gp[NT];
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < kDkVpl; ++i) s = fmaf(g[a][i], v[c][i], s);
      gp[c] = wsum(s);
    }
    const float dot = p[a][0] * gp[0] + p[a][1] * gp[1] + p[a][2] * gp[2];
#pragma unroll
    for (int c = 0; c < NT; ++c) gs[a][c] = p[a][c] * (gp[c] - dot) * scale;
  }
  // g_v (reuses v registers), then g_q, g_k from q, k
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    float* grow = gqkv + (b * NT + c) * ldg + (int64_t)h * dk;
#pragma unroll
    for (int i = 0; i < kDkVpl; ++i) {
      float o = 0.f;
#pragma unroll
      for (int a = 0; a < NT; ++a) o = fmaf(p[a][c], g[a][i], o);
      grow[2 * HD + lane + 64 * i] = o;
    }
  }
  float q[NT][kDkVpl], k[NT][kDkVpl];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const float* row = qkv + (b * NT + t) * ld + (int64_t)h * dk;
#pragma unroll
    for (int i = 0; i < kDkVpl; ++i) {
      q[t][i] = row[lane + 64 * i];
      k[t][i] = row[HD + lane + 64 * i];
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    float* grow = gqkv + (b * NT + t) * ldg + (int64_t)h * dk;
#pragma unroll
    for (int i = 0; i < kDkVpl; ++i) {
      float oq = 0.f, ok = 0.f;
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        oq = fmaf(gs[t][c], k[c][i], oq);
        ok = fmaf(gs[c][t], q[c][i], ok);
      }
      grow[lane + 64 * i] = oq;
      grow[HD + lane + 64 * i] = ok;
    }
  }
}

// Softmax backward of one head's 3 x 3 scores: g_p_ac = <g_a, v_c> (wave sums), then
// g_s_ac = p_ac (g_p_ac - sum_c' p_ac' g_p_ac') scale, with every product and sum explicit (no
// contraction left to the compiler), so the fused and unfused kernels agree bit for bit.
__device__ __forceinline__ void fold_grad_scores(const float (&g)[NT][kDkVpl],
                                                 const float (&v)[NT][kDkVpl],
                                                 const float (&p)[NT][NT], float scale,
                                                 float (&gs)[NT][NT]) {
#pragma unroll
  for (int a = 0; a < NT; ++a) {
    float gp[NT];
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      float sc = 0.f;
#pragma unroll
      for (int i = 0; i < kDkVpl; ++i) sc = fmaf(g[a][i], v[c][i], sc);
      gp[c] = wsum(sc);
    }
    const float dot = fmaf(p[a][2], gp[2], fmaf(p[a][1], gp[1], __fmul_rn(p[a][0], gp[0])));
#pragma unroll
    for (int c = 0; c < NT; ++c) gs[a][c] = __fmul_rn(__fmul_rn(p[a][c], __fsub_rn(gp[c], dot)), scale);
  }
}

// Folded Q.K (the QK^T of model.py:65-68 re-associated): s_ij = <q_i, k_j> = x_i W_q^T W_k x_j^T
// = <p_i, x_j> with p = x M_h, M_h = W_q,h^T W_k,h (D x D per head), so the product GEMM forms
// [P | V] = X [M_1 .. M_H | W_v^T] (2 H D columns instead of 3 H D) and the attention reads the
// LayerNorm rows x_j themselves as the keys of every head.  One wave per MOLECULE walks the
// heads in order: the three key rows are loaded once, and the backward sums the key gradient
// over the heads in registers (fixed order) into g_k = sum_h g_k,h, so the data-gradient GEMM
// also runs over 2 H D columns.
//   pv rows 3b+t = [p (H dk) | v (H dk)] (ld >= 2 H dk); x rows 3b+t (dk); att, P as above.
__global__ void __launch_bounds__(256)
token_attn_fold_fwd_kernel(int64_t B, int H, int dk, const float* __restrict__ pv, int64_t ld,
                           const float* __restrict__ x, int64_t ldx, float scale,
                           float* __restrict__ att, float* __restrict__ P) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const int64_t HD = (int64_t)H * dk;
  float k[NT][kDkVpl];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < kDkVpl; ++i) k[t][i] = x[(b * NT + t) * ldx + lane + 64 * i];
  for (int h = 0; h < H; ++h) {
    float q[NT][kDkVpl], v[NT][kDkVpl];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float* row = pv + (b * NT + t) * ld + (int64_t)h * dk;
#pragma unroll
      for (int i = 0; i < kDkVpl; ++i) {
        q[t][i] = row[lane + 64 * i];
        v[t][i] = row[HD + lane + 64 * i];
      }
    }
    float p[NT][NT];
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        float sc = 0.f;
#pragma unroll
        for (int i = 0; i < kDkVpl; ++i) sc = fmaf(q[a][i], k[c][i], sc);
        p[a][c] = wsum(sc) * scale;
      }
#pragma unroll
    for (int a = 0; a < NT; ++a) {
      const float m = fmaxf(p[a][0], fmaxf(p[a][1], p[a][2]));
      float z = 0.f;
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        p[a][c] = expf(p[a][c] - m);
        z += p[a][c];
      }
#pragma unroll
      for (int c = 0; c < NT; ++c) p[a][c] /= z;
    }
    const int64_t w = b * H + h;
    float* out = att + w * NT * dk;
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int i = 0; i < kDkVpl; ++i) {
        float o = 0.f;
#pragma unroll
        for (int c = 0; c < NT; ++c) o = fmaf(p[a][c], v[c][i], o);
        out[a * dk + lane + 64 * i] = o;
      }
    if (lane < NT * NT) {
      float pvv = p[0][0];
#pragma unroll
      for (int e = 1; e < NT * NT; ++e) pvv = lane == e ? p[e / NT][e % NT] : pvv;
      P[w * NT * NT + lane] = pvv;
    }
  }
}

// Backward of token_attn_fold_fwd: g_v_j = sum_i p_ij g_i; g_s = p (g_p - <p, g_p>) scale;
// g_p_i = sum_j g_s_ij x_j; g_k_j = sum_h sum_i g_s_ij p_i (heads in order).
__global__ void __launch_bounds__(256)
token_attn_fold_bwd_kernel(int64_t B, int H, int dk, const float* __restrict__ pv, int64_t ld,
                           const float* __restrict__ x, int64_t ldx, float scale,
                           const float* __restrict__ P, const float* __restrict__ g_att,
                           float* __restrict__ gpv, int64_t ldg, float* __restrict__ gk,
                           int64_t ldgk, uint32_t* __restrict__ gpv_amax) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  float gmx = 0.f;  // |max| of this lane's gpv stores (split-fp16 scale of the two GEMMs)
  const int64_t HD = (int64_t)H * dk;
  float k[NT][kDkVpl], gks[NT][kDkVpl];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < kDkVpl; ++i) {
      k[t][i] = x[(b * NT + t) * ldx + lane + 64 * i];
      gks[t][i] = 0.f;
    }
  for (int h = 0; h < H; ++h) {
    const int64_t w = b * H + h;
    float p[NT][NT];
#pragma unroll
    for (int e = 0; e < NT * NT; ++e) p[e / NT][e % NT] = P[w * NT * NT + e];
    float g[NT][kDkVpl], v[NT][kDkVpl];
    const float* ga = g_att + w * NT * dk;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float* row = pv + (b * NT + t) * ld + (int64_t)h * dk;
#pragma unroll
      for (int i = 0; i < kDkVpl; ++i) {
        g[t][i] = ga[t * dk + lane + 64 * i];
        v[t][i] = row[HD + lane + 64 * i];
      }
    }
    float gs[NT][NT];
    fold_grad_scores(g, v, p, scale, gs);
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      float* grow = gpv + (b * NT + c) * ldg + (int64_t)h * dk;
#pragma unroll
      for (int i = 0; i < kDkVpl; ++i) {
        float o = 0.f;
#pragma unroll
        for (int a = 0; a < NT; ++a) o = fmaf(p[a][c], g[a][i], o);
        grow[HD + lane + 64 * i] = o;
        gmx = fmaxf(gmx, fabsf(o));
      }
    }
    float q[NT][kDkVpl];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float* row = pv + (b * NT + t) * ld + (int64_t)h * dk;
#pragma unroll
      for (int i = 0; i < kDkVpl; ++i) q[t][i] = row[lane + 64 * i];
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float* grow = gpv + (b * NT + t) * ldg + (int64_t)h * dk;
#pragma unroll
      for (int i = 0; i < kDkVpl; ++i) {
        float oq = 0.f, ok = 0.f;
#pragma unroll
        for (int c = 0; c < NT; ++c) {
          oq = fmaf(gs[t][c], k[c][i], oq);
          ok = fmaf(gs[c][t], q[c][i], ok);
        }
        grow[lane + 64 * i] = oq;
        gmx = fmaxf(gmx, fabsf(oq));
        gks[t][i] += ok;
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < kDkVpl; ++i) gk[(b * NT + t) * ldgk + lane + 64 * i] = gks[t][i];
  if (gpv_amax) {  // one unsigned atomicMax of the float bits per wave (waves may exit early)
    gmx = wave_max(gmx);
    if (lane == 0) atomicMax(gpv_amax, __float_as_uint(gmx));
  }
}

// Conv2d(C, O, 3) over the (C, 3, W) cube of one molecule (model.py:27, 69): the kernel height
// equals the token count, so the output is (O, 1, W - 2); + bias, ReLU (model.py:27-28).
constexpr int kConvC = 12, kConvO = 12, kConvH = 3;
constexpr int kConvThreads = 384;
constexpr int kConvWg = kConvO * kConvC * kConvH * 3;  // 1296 weights
constexpr int kConvLd = 385;  // LDS row stride (W <= 384): rows land on different banks

// rows x W floats from global (row-contiguous) into LDS rows of stride kConvLd.  The aligned path
// issues all of a thread's loads (<= kStageIt float4: 36 rows x 384 / 384 threads = 9) before its
// first LDS store — one memory round trip per molecule instead of one per float4.
constexpr int kStageIt = 9;
__device__ __forceinline__ void conv_stage(float* dst, const float* __restrict__ src, int rows, int W,
                                           int tid) {
  const int w4 = W >> 2;
  if ((W & 3) == 0 && ((uintptr_t)src & 15) == 0 && rows * w4 <= kStageIt * kConvThreads) {
    float4 v[kStageIt];
#pragma unroll
    for (int it = 0; it < kStageIt; ++it) {
      const int i = tid + it * kConvThreads;
      if (i < rows * w4) {
        const int r = i / w4, c = (i - r * w4) * 4;
        v[it] = *reinterpret_cast<const float4*>(src + (int64_t)r * W + c);
      }
    }
#pragma unroll
    for (int it = 0; it < kStageIt; ++it) {
      const int i = tid + it * kConvThreads;
      if (i < rows * w4) {
        const int r = i / w4, c = (i - r * w4) * 4;
        float* d = dst + r * kConvLd + c;
        d[0] = v[it].x; d[1] = v[it].y; d[2] = v[it].z; d[3] = v[it].w;
      }
    }
  } else {
    for (int i = tid; i < rows * W; i += kConvThreads) dst[(i / W) * kConvLd + i % W] = src[i];
  }
}

__global__ void __launch_bounds__(kConvThreads)
conv3_fwd_kernel(int64_t B, int W, const float* __restrict__ in, const float* __restrict__ wgt,
                 const float* __restrict__ bias, float* __restrict__ out) {
  __shared__ float s_in[kConvC * kConvH * kConvLd];
  __shared__ __attribute__((aligned(16))) float s_wt[kConvC * kConvH * 3][kConvO];  // [(c,dy,dx)][o]
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const int Wo = W - 2;
  for (int i = tid; i < kConvWg; i += kConvThreads) s_wt[i % (kConvC * 9)][i / (kConvC * 9)] = wgt[i];
  conv_stage(s_in, in + b * (int64_t)(kConvC * kConvH * W), kConvC * kConvH, W, tid);
  __syncthreads();
  const int x = tid;
  if (x >= Wo) return;
  float acc[kConvO];
#pragma unroll
  for (int o = 0; o < kConvO; ++o) acc[o] = bias[o];
#pragma unroll 2
  for (int cd = 0; cd < kConvC * kConvH; ++cd) {
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const float a = s_in[cd * kConvLd + x + dx];
      const float4* wr = reinterpret_cast<const float4*>(s_wt[cd * 3 + dx]);  // uniform: broadcast
#pragma unroll
      for (int j = 0; j < kConvO / 4; ++j) {
        const float4 w4 = wr[j];
        acc[4 * j] = fmaf(w4.x, a, acc[4 * j]);
        acc[4 * j + 1] = fmaf(w4.y, a, acc[4 * j + 1]);
        acc[4 * j + 2] = fmaf(w4.z, a, acc[4 * j + 2]);
        acc[4 * j + 3] = fmaf(w4.w, a, acc[4 * j + 3]);
      }
    }
  }
  float* dst = out + b * (int64_t)(kConvO * Wo);
#pragma unroll
  for (int o = 0; o < kConvO; ++o) dst[o * Wo + x] = fmaxf(acc[o], 0.f);
}

// Input gradient of conv3 (through the ReLU: g_pre = g_out * (out > 0)):
//   g_in[c][dy][x'] = sum_o sum_dx w[o][c][dy][dx] g_pre[o][x' - dx]   (0 <= x' - dx < W - 2)
// and per-workgroup weight / bias gradient partials over molecules [b0, b1):
//   part[blk][(o, c, dy, dx)] = sum_b sum_x g_pre[o][x] in[c][dy][x + dx], part[blk][1296 + o].

// Weight-gradient role: thread (o, c, half) with o, c < 12 and half < 2 sums over the half of
// the columns x in [x0, x1) all nine (dy, dx) products g_pre[o][x] * in[c][dy][x + dx] with a
// three-column sliding window per dy (4 LDS reads per 9 FMAs); the two halves land in separate
// partial slots.  Thread o < 12 (half 0, c 0) also sums the bias of channel o.
constexpr int kConvPart = 2 * kConvWg + kConvO;  // per-workgroup partial row

__global__ void __launch_bounds__(kConvThreads, 3)  // two workgroups per CU
conv3_bwd_kernel(int64_t B, int W, int64_t per_block, const float* __restrict__ in,
                 const float* __restrict__ wgt, const float* __restrict__ out,
                 const float* __restrict__ g_out, float* __restrict__ g_in,
                 float* __restrict__ part) {
  __shared__ float s_in[kConvC * kConvH * kConvLd];
  __shared__ float s_g[kConvO * kConvLd];
  __shared__ __attribute__((aligned(16))) float s_wt[kConvO * 3][kConvC * kConvH];  // [(o,dx)][(c,dy)]
  const int tid = threadIdx.x;
  for (int i = tid; i < kConvWg; i += kConvThreads) {
    const int o = i / (kConvC * 9), c = (i / 9) % kConvC, dy = (i / 3) % 3, dx = i % 3;
    s_wt[o * 3 + dx][c * kConvH + dy] = wgt[i];
  }
  const int Wo = W - 2;
  const int wo = tid / (2 * kConvC), wc = (tid / 2) % kConvC, wh = tid & 1;  // weight role
  const bool wrole = tid < kConvO * kConvC * 2;
  const int xmid = (Wo + 1) / 2;
  const int x0 = wh ? xmid : 0, x1 = wh ? Wo : xmid;
  float pw[kConvH][3];
#pragma unroll
  for (int dy = 0; dy < kConvH; ++dy)
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) pw[dy][dx] = 0.f;
  float pb = 0.f;
  const int64_t b0 = (int64_t)blockIdx.x * per_block, b1 = min(B, b0 + per_block);
  for (int64_t b = b0; b < b1; ++b) {
    __syncthreads();  // previous molecule's LDS reads done
    conv_stage(s_in, in + b * (int64_t)(kConvC * kConvH * W), kConvC * kConvH, W, tid);
    const float* go = g_out + b * (int64_t)(kConvO * Wo);
    const float* oo = out + b * (int64_t)(kConvO * Wo);
    for (int i = tid; i < kConvO * kConvLd; i += kConvThreads) {
      const int o = i / kConvLd, x = i % kConvLd;
      s_g[i] = (x < Wo && oo[o * Wo + x] > 0.f) ? go[o * Wo + x] : 0.f;  // zero-padded
    }
    __syncthreads();
    // input gradient: thread per column x' < W, all 36 (c, dy) outputs in registers; each
    // g_pre[o][x' - dx] is read once, the weights are wave-uniform (scalar) loads
#ifndef MVML_CONV_NOIN
    if (tid < W) {
      const int xp = tid;
      float acc[kConvC][kConvH];
#pragma unroll
      for (int c = 0; c < kConvC; ++c)
#pragma unroll
        for (int dy = 0; dy < kConvH; ++dy) acc[c][dy] = 0.f;
#pragma unroll 1
      for (int od = 0; od < kConvO * 3; ++od) {
        const int o = od / 3, dx = od % 3;
        const int x = xp - dx;
        const float gv = x >= 0 ? s_g[o * kConvLd + x] : 0.f;  // x >= Wo reads the padding
        const float4* wr = reinterpret_cast<const float4*>(s_wt[od]);  // uniform: broadcast
#pragma unroll
        for (int j = 0; j < kConvC * kConvH / 4; ++j) {
          const float4 w4 = wr[j];
          float* a = &acc[0][0] + 4 * j;
          a[0] = fmaf(w4.x, gv, a[0]);
          a[1] = fmaf(w4.y, gv, a[1]);
          a[2] = fmaf(w4.z, gv, a[2]);
          a[3] = fmaf(w4.w, gv, a[3]);
        }
      }
      float* dst = g_in + b * (int64_t)(kConvC * kConvH * W);
#pragma unroll
      for (int c = 0; c < kConvC; ++c)
#pragma unroll
        for (int dy = 0; dy < kConvH; ++dy) dst[(c * kConvH + dy) * W + xp] = acc[c][dy];
    }
#endif
#ifndef MVML_CONV_NOW
    if (wrole) {
      const float* gi = s_g + wo * kConvLd;
      const float* a0p = s_in + (wc * kConvH + 0) * kConvLd;
      const float* a1p = s_in + (wc * kConvH + 1) * kConvLd;
      const float* a2p = s_in + (wc * kConvH + 2) * kConvLd;
      float w0[kConvH] = {a0p[x0], a1p[x0], a2p[x0]};
      float w1[kConvH] = {a0p[x0 + 1], a1p[x0 + 1], a2p[x0 + 1]};
#pragma unroll 4
      for (int x = x0; x < x1; ++x) {
        const float gv = gi[x];
        const float w2[kConvH] = {a0p[x + 2], a1p[x + 2], a2p[x + 2]};
#pragma unroll
        for (int dy = 0; dy < kConvH; ++dy) {
          pw[dy][0] = fmaf(gv, w0[dy], pw[dy][0]);
          pw[dy][1] = fmaf(gv, w1[dy], pw[dy][1]);
          pw[dy][2] = fmaf(gv, w2[dy], pw[dy][2]);
          w0[dy] = w1[dy];
          w1[dy] = w2[dy];
        }
      }
      if (wh == 0 && wc == 0) {
        float s = 0.f;
        for (int x = 0; x < Wo; ++x) s += gi[x];
        pb += s;
      }
    }
#endif
  }
  if (wrole) {
    float* dst = part + (int64_t)blockIdx.x * kConvPart + wh * kConvWg;
#pragma unroll
    for (int dy = 0; dy < kConvH; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) dst[((wo * kConvC + wc) * 3 + dy) * 3 + dx] = pw[dy][dx];
    if (wh == 0 && wc == 0) part[(int64_t)blockIdx.x * kConvPart + 2 * kConvWg + wo] = pb;
  }
}

// ---- conv3, register-blocked (round 2) ---------------------------------------------------
// Forward: thread per output column x holds its 108 inputs in[c][dy][x + dx] in registers and
// walks the 12 output channels with the weights as wave-uniform (scalar) loads — 1296 FMAs per
// thread with no LDS traffic in the loop (the LDS-broadcast weight reads of conv3_fwd_kernel
// made it LDS-bound).  Same summation order per output as conv3_fwd_kernel ((c, dy) outer, dx
// inner).
__global__ void __launch_bounds__(kConvThreads, 2)
conv3_fwd2_kernel(int64_t B, int W, const float* __restrict__ in, const float* __restrict__ wgt,
                  const float* __restrict__ bias, float* __restrict__ out) {
  __shared__ float s_in[kConvC * kConvH * kConvLd + 4];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const int Wo = W - 2;
  conv_stage(s_in, in + b * (int64_t)(kConvC * kConvH * W), kConvC * kConvH, W, tid);
  __syncthreads();
  const int x = tid;
  if (x >= Wo) return;
  float a[kConvC * kConvH * 3];
#pragma unroll
  for (int cd = 0; cd < kConvC * kConvH; ++cd)
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) a[cd * 3 + dx] = s_in[cd * kConvLd + x + dx];
  float* dst = out + b * (int64_t)(kConvO * Wo) + x;
#pragma unroll
  for (int o = 0; o < kConvO; ++o) {
    const float* w = wgt + o * (kConvC * kConvH * 3);
    float acc = bias[o];
#pragma unroll
    for (int j = 0; j < kConvC * kConvH * 3; ++j) acc = fmaf(w[j], a[j], acc);
    dst[o * Wo] = fmaxf(acc, 0.f);
  }
}

// Backward, one workgroup (6 waves) per range of molecules:
//  * input gradient: thread per column x' holds g_pre[o][x' - dx] (36 values) in registers and
//    accumulates the 36 (c, dy) outputs with scalar-loaded weights (1296 FMAs, no LDS in the
//    loop);
//  * weight / bias gradient on the f32 matrix cores: per molecule gW[o][n] += sum_x g_pre[o][x]
//    im2col[x][n] with n = (c, dy, dx) < 108 and n = 108 a column of ones (the bias), as
//    v_mfma_f32_16x16x4_f32 over 7 column tiles of 16; wave w owns the x-steps [64 w, 64 w + 64)
//    of every molecule, the fragments are per-lane LDS reads of the staged rows.  The six waves'
//    16 x 112 partial tiles are summed in fixed order at the end (deterministic, no atomics).
typedef float f32x4_t __attribute__((ext_vector_type(4)));
constexpr int kConvWaves = kConvThreads / 64;  // 6
#ifndef MVML_CONV_MFMA_DX
// 1: the input gradient on v_mfma_f32_16x16x4_f32 (36 x 36 weight matrix in 27 registers per
// lane) — measured 6.34 vs 5.75 ms for the VALU loop at 65,536 molecules (register pressure)
#define MVML_CONV_MFMA_DX 0
#endif
constexpr int kConvNT = 7;                     // 16-column tiles of n (108 weights + bias)
#ifndef MVML_CONV_BWD_WAVES
#define MVML_CONV_BWD_WAVES 2  // waves per SIMD the register budget is cut for (3: two workgroups per CU)
#endif
__global__ void __launch_bounds__(kConvThreads, MVML_CONV_BWD_WAVES)
conv3_bwd2_kernel(int64_t B, int W, int64_t per_block, const float* __restrict__ in,
                  const float* __restrict__ wgt, const float* __restrict__ out,
                  const float* __restrict__ g_out, float* __restrict__ g_in,
                  float* __restrict__ part) {
  __shared__ float s_in[kConvC * kConvH * kConvLd + 8];
  __shared__ float s_g[kConvO * kConvLd];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int Wo = W - 2;
  if (tid < 8) s_in[kConvC * kConvH * kConvLd + tid] = 0.f;  // reads past the last row: finite
  // the pad columns [W, kConvLd) of every row are read by the weight-gradient MFMA steps past
  // Wo (against a zero g_out): they must be finite (0 x NaN of stale LDS would be NaN)
  for (int i = tid; i < kConvC * kConvH * (kConvLd - W); i += kConvThreads)
    s_in[(i / (kConvLd - W)) * kConvLd + W + i % (kConvLd - W)] = 0.f;
  f32x4_t acc[kConvNT];
#pragma unroll
  for (int j = 0; j < kConvNT; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // this lane's fixed fragment coordinates: A row o = lane & 15; B column n = 16 j + (lane & 15)
  const int lo = lane & 15, lk = lane >> 4;
  int boff[kConvNT];  // LDS offset of im2col(x = 0, n) (row (c, dy), column dx), or -1 / -2
#pragma unroll
  for (int j = 0; j < kConvNT; ++j) {
    const int n = 16 * j + lo;
    boff[j] = n < 108 ? (n / 3) * kConvLd + n % 3 : (n == 108 ? -1 : -2);
  }
#if MVML_CONV_MFMA_DX
  // input-gradient A fragments: W[o][(c, dy)][dx] as a 36 x 36 matrix, rows (c, dy) = 16 rt + lo,
  // columns k = (o, dx) = 4 ks + lk; loaded once, held in 27 registers
  float wfr[3][9];
#pragma unroll
  for (int rt = 0; rt < 3; ++rt)
#pragma unroll
    for (int ks = 0; ks < 9; ++ks) {
      const int cd = 16 * rt + lo, k = 4 * ks + lk;
      wfr[rt][ks] = cd < kConvC * kConvH ? wgt[(k / 3) * 108 + cd * 3 + k % 3] : 0.f;
    }
#endif
  const int64_t b0 = (int64_t)blockIdx.x * per_block, b1 = min(B, b0 + per_block);
  for (int64_t b = b0; b < b1; ++b) {
    __syncthreads();  // previous molecule's LDS reads done
    conv_stage(s_in, in + b * (int64_t)(kConvC * kConvH * W), kConvC * kConvH, W, tid);
    const float* go = g_out + b * (int64_t)(kConvO * Wo);
    const float* oo = out + b * (int64_t)(kConvO * Wo);
    {  // g_pre = g_out where out > 0, zero-padded rows; all loads before the stores
      constexpr int kIt = (kConvO * kConvLd + kConvThreads - 1) / kConvThreads;
      float gv[kIt], ov[kIt];
#pragma unroll
      for (int it = 0; it < kIt; ++it) {
        const int i = tid + it * kConvThreads, o = i / kConvLd, x = i % kConvLd;
        const bool ok = i < kConvO * kConvLd && x < Wo;
        gv[it] = ok ? go[o * Wo + x] : 0.f;
        ov[it] = ok ? oo[o * Wo + x] : 0.f;
      }
#pragma unroll
      for (int it = 0; it < kIt; ++it) {
        const int i = tid + it * kConvThreads;
        if (i < kConvO * kConvLd) s_g[i] = ov[it] > 0.f ? gv[it] : 0.f;
      }
    }
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);  // phases stay apart (registers)
#if MVML_CONV_MFMA_DX
    {  // input gradient on the matrix cores: g_in[(c, dy)][x'] = sum_(o, dx) W g_pre[o][x' - dx];
       // wave w owns the columns [64 w, 64 w + 64) (4 tiles), all three row tiles
      f32x4_t gacc[3][4];
#pragma unroll
      for (int rt = 0; rt < 3; ++rt)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) gacc[rt][ct] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 9; ++ks) {
        const int k = 4 * ks + lk, o = k / 3, dx = k % 3;
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          const int xi = 64 * wid + 16 * ct + lo - dx;
          const float bv = xi >= 0 ? s_g[o * kConvLd + max(xi, 0)] : 0.f;
#pragma unroll
          for (int rt = 0; rt < 3; ++rt)
            gacc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(wfr[rt][ks], bv, gacc[rt][ct], 0, 0, 0);
        }
      }
      float* gb = g_in + b * (int64_t)(kConvC * kConvH * W);
#pragma unroll
      for (int rt = 0; rt < 3; ++rt)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          const int xp = 64 * wid + 16 * ct + lo;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int cd = 16 * rt + 4 * lk + r;
            if (cd < kConvC * kConvH && xp < W) gb[cd * W + xp] = gacc[rt][ct][r];
          }
        }
    }
#else
    if (tid < W) {  // input gradient
      const int xp = tid;
      float g[kConvO][3];
#pragma unroll
      for (int o = 0; o < kConvO; ++o)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) g[o][dx] = xp - dx >= 0 ? s_g[o * kConvLd + xp - dx] : 0.f;
      float acc_in[kConvC * kConvH];
#pragma unroll
      for (int i = 0; i < kConvC * kConvH; ++i) acc_in[i] = 0.f;
#pragma unroll
      for (int o = 0; o < kConvO; ++o) {  // (o, dx) order as conv3_bwd_kernel
        const float* w = wgt + o * (kConvC * kConvH * 3);
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
          for (int cd = 0; cd < kConvC * kConvH; ++cd)
            acc_in[cd] = fmaf(w[cd * 3 + dx], g[o][dx], acc_in[cd]);
      }
      float* dst = g_in + b * (int64_t)(kConvC * kConvH * W) + xp;
#pragma unroll
      for (int cd = 0; cd < kConvC * kConvH; ++cd) dst[cd * W] = acc_in[cd];
    }
#endif
    __builtin_amdgcn_sched_barrier(0);
    // weight / bias gradient: x-steps of 4 columns, wave w takes steps [16 w, 16 w + 16)
    for (int ks = 16 * wid; ks < 16 * wid + 16; ++ks) {
      const int x = 4 * ks + lk;
      const float av = lo < kConvO ? s_g[lo * kConvLd + x] : 0.f;  // 0 past Wo (padding)
#pragma unroll
      for (int j = 0; j < kConvNT; ++j) {
        const float bv = boff[j] >= 0 ? s_in[boff[j] + x] : (boff[j] == -1 ? 1.f : 0.f);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[j], 0, 0, 0);
      }
    }
  }
  // fixed-order reduction of the six waves' 16 x 112 tiles: C[i][n], i = 4 (lane >> 4) + r
  __syncthreads();
  float* red = s_in;  // 6 x 16 x 112 floats = 42 KB <= s_in
#pragma unroll
  for (int j = 0; j < kConvNT; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(wid * 16 + 4 * lk + r) * 112 + 16 * j + lo] = acc[j][r];
  __syncthreads();
  for (int i = tid; i < kConvO * 109; i += kConvThreads) {
    const int o = i / 109, n = i % 109;
    float s = 0.f;
    for (int w = 0; w < kConvWaves; ++w) s += red[(w * 16 + o) * 112 + n];
    if (n < 108) part[(int64_t)blockIdx.x * kConvPart + o * 108 + n] = s;
    else part[(int64_t)blockIdx.x * kConvPart + 2 * kConvWg + o] = s;
  }
}

// Forward on the matrix cores: out[o][x] = ReLU(b[o] + sum_k W[o][k] im2col[k][x]), k = (c, dy,
// dx) < 108 in 27 steps of v_mfma_f32_16x16x4_f32, M = 12 output channels (one 16-row tile), wave w
// the columns [64 w, 64 w + 64); the weight fragments (27 per lane) are loaded once per
// workgroup, the im2col operand is a per-lane LDS read of the staged rows.  Replaces the
// per-thread VALU loop, whose 1296 weights arrived as 81 serialised scalar loads per molecule.
__global__ void __launch_bounds__(kConvThreads, 3)  // two workgroups per CU (3 waves per SIMD)
conv3_fwd3_kernel(int64_t B, int W, int64_t per_block, const float* __restrict__ in,
                  const float* __restrict__ wgt, const float* __restrict__ bias,
                  float* __restrict__ out) {
  __shared__ float s_in[kConvC * kConvH * kConvLd + 8];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lo = lane & 15, lk = lane >> 4;
  const int Wo = W - 2;
  float wfr[27];
#pragma unroll
  for (int ks = 0; ks < 27; ++ks) wfr[ks] = lo < kConvO ? wgt[lo * 108 + 4 * ks + lk] : 0.f;
  float bo[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bo[r] = 4 * lk + r < kConvO ? bias[4 * lk + r] : 0.f;
  if (tid < 8) s_in[kConvC * kConvH * kConvLd + tid] = 0.f;
  const int64_t b0 = (int64_t)blockIdx.x * per_block, b1 = min(B, b0 + per_block);
  for (int64_t b = b0; b < b1; ++b) {
    __syncthreads();  // previous molecule's LDS reads done
    conv_stage(s_in, in + b * (int64_t)(kConvC * kConvH * W), kConvC * kConvH, W, tid);
    __syncthreads();
    f32x4_t acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[ct] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 27; ++ks) {
      const int k = 4 * ks + lk;  // im2col row: (c, dy) = k / 3, shift dx = k % 3
      const int koff = (k / 3) * kConvLd + k % 3;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const float bv = s_in[koff + 64 * wid + 16 * ct + lo];  // columns >= Wo: discarded
        acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(wfr[ks], bv, acc[ct], 0, 0, 0);
      }
    }
    float* ob = out + b * (int64_t)(kConvO * Wo);
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int x = 64 * wid + 16 * ct + lo;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = 4 * lk + r;
        if (o < kConvO && x < Wo) ob[o * Wo + x] = fmaxf(acc[ct][r] + bo[r], 0.f);
      }
    }
  }
}

// ---- token attention + Conv2d fused (round 3) ---------------------------------------------
// The (12, 3, 384) attention cube of a molecule is formed in LDS and consumed there by the
// convolution: it never makes the HBM round trip between the attention and the Conv2d (forward:
// 55 KB written + read per molecule; backward: the cube read, its gradient written and read
// again).  One workgroup of 12 waves per run of molecules, wave h = head h; the attention
// arithmetic is token_attn_fold_fwd / _bwd's (same operation order, so the cube and every g_pv
// element are bit-identical to the unfused pair), the convolution conv3_fwd3 / conv3_bwd2's
// with the column tiles spread over 12 waves.  The backward recomputes the cube as P V (bitwise
// the forward's values) instead of reading a saved copy, and sums the keys' gradient over heads
// as twelve wave partials added in head order (the unfused kernel's order).
constexpr int kFuseWaves = 12;  // = kConvC heads
constexpr int kFuseThreads = 64 * kFuseWaves;
constexpr int kFuseW = 64 * kDkVpl;              // 384 columns
constexpr int kFuseCube = kConvC * kConvH * kConvLd + 8;  // cube rows (h, t) + a zero tail
constexpr int kFuseG = kConvO * kConvLd;          // g_pre rows o
static_assert(kFuseW <= kConvLd - 1, "one pad column per cube row");

// softmax(scale * <q_a, k_c>) over c for the 3 x 3 scores of one head (token_attn_fold_fwd's order)
__device__ __forceinline__ void fold_scores(const float (&q)[NT][kDkVpl], const float (&k)[NT][kDkVpl],
                                            float scale, float (&p)[NT][NT]) {
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      float sc = 0.f;
#pragma unroll
      for (int i = 0; i < kDkVpl; ++i) sc = fmaf(q[a][i], k[c][i], sc);
      p[a][c] = wsum(sc) * scale;
    }
#pragma unroll
  for (int a = 0; a < NT; ++a) {
    const float m = fmaxf(p[a][0], fmaxf(p[a][1], p[a][2]));
    float z = 0.f;
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      p[a][c] = expf(p[a][c] - m);
      z += p[a][c];
    }
#pragma unroll
    for (int c = 0; c < NT; ++c) p[a][c] /= z;
  }
}

// att rows (h, a) = sum_c p_ac v_c into the LDS cube (row stride kConvLd)
__device__ __forceinline__ void fold_att_lds(const float (&p)[NT][NT], const float (&v)[NT][kDkVpl],
                                             float* s_rows, int lane) {
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int i = 0; i < kDkVpl; ++i) {
      float o = 0.f;
#pragma unroll
      for (int c = 0; c < NT; ++c) o = fmaf(p[a][c], v[c][i], o);
      s_rows[a * kConvLd + lane + 64 * i] = o;
    }
}

__device__ __forceinline__ void load_rows3(const float* __restrict__ base, int64_t ld, int lane,
                                           float (&r)[NT][kDkVpl]) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < kDkVpl; ++i) r[t][i] = base[t * ld + lane + 64 * i];
}

__global__ void __launch_bounds__(kFuseThreads, 3)  // one workgroup per CU
attn_conv_fwd_kernel(int64_t B, int64_t per_block, const float* __restrict__ pv, int64_t ld,
                     const float* __restrict__ x, int64_t ldx, float scale,
                     const float* __restrict__ wgt, const float* __restrict__ bias,
                     float* __restrict__ P, float* __restrict__ out, uint32_t drop_thr,
                     float drop_scale, uint64_t drop_seed) {
  constexpr int W = kFuseW, Wo = W - 2, H = kConvC;
  constexpr int64_t HD = (int64_t)H * W;
  __shared__ float s_in[kFuseCube];
  const int tid = threadIdx.x, lane = tid & 63, h = tid >> 6;
  const int lo = lane & 15, lk = lane >> 4;
  float wfr[27];
#pragma unroll
  for (int ks = 0; ks < 27; ++ks) wfr[ks] = lo < kConvO ? wgt[lo * 108 + 4 * ks + lk] : 0.f;
  float bo[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bo[r] = 4 * lk + r < kConvO ? bias[4 * lk + r] : 0.f;
  if (tid < 8) s_in[kConvC * kConvH * kConvLd + tid] = 0.f;
  const int64_t b0 = (int64_t)blockIdx.x * per_block, b1 = min(B, b0 + per_block);
  // head h's rows of molecule b: keys (the LayerNorm rows), p and v; the next molecule's are
  // loaded while this one's convolution runs
  float k[NT][kDkVpl], q[NT][kDkVpl], v[NT][kDkVpl];
  auto load = [&](int64_t b) {
    load_rows3(x + b * NT * ldx, ldx, lane, k);
    load_rows3(pv + b * NT * ld + (int64_t)h * W, ld, lane, q);
    load_rows3(pv + b * NT * ld + HD + (int64_t)h * W, ld, lane, v);
  };
  if (b0 < b1) load(b0);
  for (int64_t b = b0; b < b1; ++b) {
    __syncthreads();  // the previous molecule's convolution reads of the cube are done
    {
      float p[NT][NT];
      fold_scores(q, k, scale, p);
      fold_att_lds(p, v, s_in + h * NT * kConvLd, lane);
      if (lane < NT * NT) {
        float pvv = p[0][0];
#pragma unroll
        for (int e = 1; e < NT * NT; ++e) pvv = lane == e ? p[e / NT][e % NT] : pvv;
        P[(b * H + h) * NT * NT + lane] = pvv;
      }
    }
    if (b + 1 < b1) load(b + 1);
    __syncthreads();
    // Conv2d + bias + ReLU on the matrix cores (conv3_fwd3_kernel): wave h the column tiles
    // [32 h, 32 h + 32)
    f32x4_t acc[2];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) acc[ct] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 27; ++ks) {
      const int kk = 4 * ks + lk;
      const int koff = (kk / 3) * kConvLd + kk % 3;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const float bv = s_in[koff + 32 * h + 16 * ct + lo];  // columns >= Wo: discarded
        acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(wfr[ks], bv, acc[ct], 0, 0, 0);
      }
    }
    float* ob = out + b * (int64_t)(kConvO * Wo);
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const int xx = 32 * h + 16 * ct + lo;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = 4 * lk + r;
        if (o < kConvO && xx < Wo) {
          float y = fmaxf(acc[ct][r] + bo[r], 0.f);
          if (drop_thr)  // the Dropout after the ReLU (model.py:36), mvml_dropout_fwd's mask
            y = dropout_u32(drop_seed, b * (int64_t)(kConvO * Wo) + o * Wo + xx) >= drop_thr ? y * drop_scale
                                                                                               : 0.f;
          ob[o * Wo + xx] = y;
        }
      }
    }
  }
}

// Backward of attn_conv_fwd, one molecule per loop trip, its inputs prefetched one molecule
// ahead by LDS-DMA (global_load_lds_dwordx4: no registers, the loads of molecule b + 1 fly
// while molecule b computes):
//   (A) wait for molecule b's staged g_out / out / v / P, barrier;
//   (B) the cube recomputed as P v into LDS (wave h: head h);
//   (C) Conv2d weight gradient on the matrix cores (conv3_bwd2's MFMA steps, wave w the x-steps
//       [8 w, 8 w + 8)) and the bias row sums, g_pre = g_out (out > 0) read from the staged rows;
//   (D) the cube's gradient (conv3_bwd2's VALU loop; threads t and t + 384 the (c, dy) rows
//       [0, 18) / [18, 36) of column t) in registers; barrier, then the cube gradient is stored
//       over the cube, each wave moves its head's v / P rows to registers, molecule b + 1's
//       g_out / out start into their (now free) staging rows and the wave's query / key loads
//       are issued; barrier, then molecule b + 1's v / P start;
//   (E) the attention backward of head h (token_attn_fold_bwd): g_pv stores, the keys'
//       gradient partial over head h's own cube rows, then the twelve partials in head order.
// Staging (one __shared__ array): cube [36 x 385 + 8] | g_out [18 KB] | out [18 KB] | v [3 x
// 4608] | P [108 + pad], each region a whole number of 1-KB DMA pieces.
constexpr int kStG = 18;                       // 1-KB pieces of a molecule's g_out (4584 floats)
constexpr int kStV = 54;                       // v: 3 rows x 4608 floats
constexpr int kStVP = kStV + 1;                // + P (108 floats)
constexpr int kOffG = ((kFuseCube * 4 + 1023) / 1024) * 256;  // float offsets of the regions
constexpr int kOffO = kOffG + kStG * 256;
constexpr int kOffV = kOffO + kStG * 256;
constexpr int kOffP = kOffV + kStV * 256;
constexpr int kBwdLds = kOffP + 256;
static_assert(kBwdLds * 4 <= 160 * 1024, "backward staging fits the CU's LDS");
static_assert(kConvO * (kFuseW - 2) <= kStG * 256, "g_out rows fit their staging");

// a wave-uniform pointer held in SGPRs (so a global_load_lds takes the saddr + 32-bit lane
// offset form instead of a 64-bit address per lane)
__device__ __forceinline__ const float* uniform_ptr(const float* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return reinterpret_cast<const float*>(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ void glds16(const float* src, float* dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// molecule b's g_out and out rows (contiguous 4584-float blocks) into their staging rows:
// pieces h and h + 12 of each (18 pieces), lanes past the block re-read its last float4
__device__ __forceinline__ void stage_go(const float* __restrict__ g_out, const float* __restrict__ out,
                                         int64_t b, float* lds, int h, int lane) {
  constexpr int n = kConvO * (kFuseW - 2);
  const int64_t base = b * (int64_t)n;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int piece = h + kFuseWaves * k;
    if (piece < kStG) {
      const int off = min(piece * 256 + 4 * lane, n - 4);
      glds16(g_out + base + off, lds + kOffG + piece * 256);
      glds16(out + base + off, lds + kOffO + piece * 256);
    }
  }
}

// molecule b's v rows (3 x 4608 floats of pv at column H dk) and P (108 floats): wave h issues
// pieces 5 h .. 5 h + 4 of the 55; wave 11's five (and nothing else) repeat the P piece — every
// wave issues exactly five, so the compiler's wait for the query / key loads issued before them
// is vmcnt(5), not a drain of the next molecule's staging
__device__ __forceinline__ void stage_vp(const float* __restrict__ pv, int64_t ld,
                                         const float* __restrict__ P, int64_t b, float* lds, int h,
                                         int lane) {
  constexpr int64_t HD = (int64_t)kConvC * kFuseW;
  const float* pb = uniform_ptr(P + b * (kConvC * NT * NT)) + min(4 * lane, kConvC * NT * NT - 4);
#pragma unroll
  for (int k = 0; k < 5; ++k) {  // branch-free (selects): the wait counts stay exact
    const int piece = 5 * h + k;
    const int t = min(piece, kStV - 1) / 18;
    const float* vb = uniform_ptr(pv + (b * NT + t) * ld + HD + (min(piece, kStV - 1) % 18) * 256) + 4 * lane;
    const bool isv = piece < kStV;  // else the P piece (repeats write the same bytes)
    glds16(isv ? vb : pb, lds + (isv ? kOffV + piece * 256 : kOffP));
  }
}

__global__ void __launch_bounds__(kFuseThreads, 3)  // one workgroup per CU
attn_conv_bwd_kernel(int64_t B, int64_t per_block, const float* __restrict__ pv, int64_t ld,
                     const float* __restrict__ x, int64_t ldx, float scale,
                     const float* __restrict__ P, const float* __restrict__ wgt,
                     const float* __restrict__ out, const float* __restrict__ g_out, float g_scale,
                     float* __restrict__ gpv, int64_t ldg, float* __restrict__ gk, int64_t ldgk,
                     uint32_t* __restrict__ gpv_amax, float* __restrict__ part,
                     uint32_t* __restrict__ gpv_rows) {
  constexpr int W = kFuseW, Wo = W - 2, H = kConvC;
  constexpr int64_t HD = (int64_t)H * W;
  constexpr int kCD = kConvC * kConvH / 2;  // cube-gradient rows per thread
  __shared__ __attribute__((aligned(16))) float lds[kBwdLds];
  float* s_in = lds;
  const float* s_o = lds + kOffO;
  const float* s_v = lds + kOffV;   // [3][12 x 384]
  const float* s_p = lds + kOffP;   // [12][9]
  const int tid = threadIdx.x, lane = tid & 63;
  const int h = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches
  const int lo = lane & 15, lk = lane >> 4;
  if (tid < 8) s_in[kConvC * kConvH * kConvLd + tid] = 0.f;
  for (int i = tid; i < kConvC * kConvH * (kConvLd - W); i += kFuseThreads)  // pad columns: finite
    s_in[(i / (kConvLd - W)) * kConvLd + W + i % (kConvLd - W)] = 0.f;
  f32x4_t acc[kConvNT];
#pragma unroll
  for (int j = 0; j < kConvNT; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  int boff[kConvNT];
#pragma unroll
  for (int j = 0; j < kConvNT; ++j) {
    const int n = 16 * j + lo;
    boff[j] = n < 108 ? (n / 3) * kConvLd + n % 3 : (n == 108 ? -1 : -2);
  }
  // g_pre[o][x] (masked in place over the staged g_out rows at (A)); 0 outside [0, Wo), by
  // select on an always-in-range address (no branch around the LDS read)
  float* s_gp = lds + kOffG;
  auto gpre = [&](int o, int xx) -> float {
    const float v = s_gp[o * Wo + min(max(xx, 0), Wo - 1)];
    return (xx >= 0 && xx < Wo) ? v : 0.f;
  };
  float gmx = 0.f, pb = 0.f;
  // cube-gradient role; half is wave-uniform (W = 6 waves), so its weights are scalar loads
  const int xp = tid % W, half = __builtin_amdgcn_readfirstlane(tid / W);
  const int64_t b0 = (int64_t)blockIdx.x * per_block, b1 = min(B, b0 + per_block);
  if (b0 < b1) {
    stage_go(g_out, out, b0, lds, h, lane);
    stage_vp(pv, ld, P, b0, lds, h, lane);
  }
  for (int64_t b = b0; b < b1; ++b) {
    const bool next = b + 1 < b1;
    // (A) molecule b's staging landed (this wave's pieces; the barrier: everyone's); then
    // g_pre = g_out (out > 0) in place
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    for (int e = tid; e < kConvO * Wo; e += kFuseThreads)
      s_gp[e] = s_o[e] > 0.f ? (g_scale == 1.f ? s_gp[e] : s_gp[e] * g_scale) : 0.f;
    // (B) the cube rows of head h
    {
      float p[NT][NT], v[NT][kDkVpl];
#pragma unroll
      for (int e = 0; e < NT * NT; ++e) p[e / NT][e % NT] = s_p[h * NT * NT + e];
      load_rows3(s_v + (int64_t)h * W, HD, lane, v);
      fold_att_lds(p, v, s_in + h * NT * kConvLd, lane);
    }
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
    // (C) weight / bias gradient
#pragma unroll 2
    for (int ks = 8 * h; ks < 8 * h + 8; ++ks) {
      const int xx = 4 * ks + lk;
      const float av = lo < kConvO ? gpre(lo, xx) : 0.f;
#pragma unroll
      for (int j = 0; j < kConvNT; ++j) {
        const float bv = boff[j] >= 0 ? s_in[boff[j] + xx] : (boff[j] == -1 ? 1.f : 0.f);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[j], 0, 0, 0);
      }
    }
    {  // bias of channel h: this molecule's row sum, then the running sum (short chains)
      float sb = 0.f;
#pragma unroll
      for (int i = 0; i < kDkVpl; ++i) sb += gpre(h, lane + 64 * i);
      pb += wsum(sb);
    }
    __builtin_amdgcn_sched_barrier(0);  // phases stay apart (registers)
    // (D) the cube's gradient in registers
    float acc_in[kCD];
    {
      int xpl = xp;  // laundered per molecule: the 36 row addresses are not hoisted out of the loop
      asm volatile("" : "+v"(xpl));
#pragma unroll
      for (int i = 0; i < kCD; ++i) acc_in[i] = 0.f;
      // the weights as SCALAR loads (constant address space: s_load, K$-resident) issued per
      // molecule; laundering the pointer keeps the compiler from hoisting all 648 of them out of
      // the molecule loop (SGPR spills).  A generic pointer here compiles to flat vector loads,
      // each batch drained by vmcnt(0) lgkmcnt(0) — 25 full memory latencies per molecule.
      const float* wh = wgt + half * kCD * 3;
      asm volatile("" : "+s"(wh));
      const __attribute__((address_space(4))) float* wc =
          (const __attribute__((address_space(4))) float*)wh;
      // g_pre rows one output channel at a time (3 values live, not 36)
#pragma unroll 2
      for (int o = 0; o < kConvO; ++o) {  // (o, dx) order as conv3_bwd2_kernel
        const auto* w = wc + o * (kConvC * kConvH * 3);
        float g[3];
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) g[dx] = gpre(o, xpl - dx);
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
          for (int cd = 0; cd < kCD; ++cd) acc_in[cd] = fmaf(w[cd * 3 + dx], g[dx], acc_in[cd]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every staged-row / cube read done
#pragma unroll
    for (int cd = 0; cd < kCD; ++cd) s_in[(half * kCD + cd) * kConvLd + xp] = acc_in[cd];
    float v[NT][kDkVpl], p[NT][NT];
#pragma unroll
    for (int e = 0; e < NT * NT; ++e) p[e / NT][e % NT] = s_p[h * NT * NT + e];
    load_rows3(s_v + (int64_t)h * W, HD, lane, v);
    if (next) stage_go(g_out, out, b + 1, lds, h, lane);  // after the stores: registers
    // head h's query rows and the keys (plain loads: the compiler's wait at their first use
    // also covers the LDS-DMA pieces issued before it, so the next molecule's staging and these
    // loads share one memory latency)
    float q[NT][kDkVpl], k[NT][kDkVpl];
    load_rows3(pv + b * NT * ld + (int64_t)h * W, ld, lane, q);
    load_rows3(x + b * NT * ldx, ldx, lane, k);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // cube gradient stored; v / P read
    // unconditional (the last molecule re-stages its own v / P, already in registers): a fixed
    // count of DMA pieces per wave keeps the compiler's wait below at vmcnt(5)
    stage_vp(pv, ld, P, next ? b + 1 : b, lds, h, lane);
    __builtin_amdgcn_sched_barrier(0);
    // (E) attention backward of head h (token_attn_fold_bwd_kernel's order)
    {
      float g[NT][kDkVpl];
      load_rows3(s_in + h * NT * kConvLd, kConvLd, lane, g);
      float gs[NT][NT];
      fold_grad_scores(g, v, p, scale, gs);
      float rmx[NT];  // this wave's part of each token row's |max| (gpv_rows)
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        float* grow = gpv + (b * NT + c) * ldg + HD + (int64_t)h * W;
        rmx[c] = 0.f;
#pragma unroll
        for (int i = 0; i < kDkVpl; ++i) {
          float o = 0.f;
#pragma unroll
          for (int a = 0; a < NT; ++a) o = fmaf(p[a][c], g[a][i], o);
          grow[lane + 64 * i] = o;
          rmx[c] = fmaxf(rmx[c], fabsf(o));
        }
      }
      // the keys' gradient partial of head h goes over head h's own cube rows (read above by
      // this wave only)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        float* grow = gpv + (b * NT + t) * ldg + (int64_t)h * W;
#pragma unroll
        for (int i = 0; i < kDkVpl; ++i) {
          float oq = 0.f, ok = 0.f;
#pragma unroll
          for (int c = 0; c < NT; ++c) {
            oq = fmaf(gs[t][c], k[c][i], oq);
            ok = fmaf(gs[c][t], q[c][i], ok);
          }
          grow[lane + 64 * i] = oq;
          rmx[t] = fmaxf(rmx[t], fabsf(oq));
          s_in[(h * NT + t) * kConvLd + lane + 64 * i] = ok;
        }
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        gmx = fmaxf(gmx, rmx[t]);
        if (gpv_rows) {  // the twelve head waves' parts of the row: an order-free max
          const float m = wave_max(rmx[t]);
          if (lane == 0) atomicMax(gpv_rows + b * NT + t, __float_as_uint(m));
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    for (int e = tid; e < NT * W; e += kFuseThreads) {  // g_k = sum over heads in head order
      const int t = e / W, c = e % W;
      float s = 0.f;
#pragma unroll
      for (int hh = 0; hh < H; ++hh) s += s_in[(hh * NT + t) * kConvLd + c];
      gk[(b * NT + t) * ldgk + c] = s;
    }
  }
  if (gpv_amax) {  // one unsigned atomicMax of the float bits per wave
    gmx = wave_max(gmx);
    if (lane == 0) atomicMax(gpv_amax, __float_as_uint(gmx));
  }
  // fixed-order reduction of the twelve waves' 12 x 109 weight-gradient tiles (rows o < 12)
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  float* red = lds;  // 12 x 12 x 112 floats <= the LDS array
  static_assert(kFuseWaves * kConvO * 112 <= kBwdLds, "reduction fits the LDS");
#pragma unroll
  for (int j = 0; j < kConvNT; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * lk + r < kConvO) red[(h * kConvO + 4 * lk + r) * 112 + 16 * j + lo] = acc[j][r];
  __syncthreads();
  for (int i = tid; i < kConvO * 108; i += kFuseThreads) {
    const int o = i / 108, n = i % 108;
    float s = 0.f;
    for (int w = 0; w < kFuseWaves; ++w) s += red[(w * kConvO + o) * 112 + n];
    part[(int64_t)blockIdx.x * kConvPart + o * 108 + n] = s;
  }
  if (lane == 0) part[(int64_t)blockIdx.x * kConvPart + 2 * kConvWg + h] = pb;
}

// Fixed-order sum of the per-workgroup partials: out[i] = sum_blk sum_j<nsub
// part[blk * stride + j * sub_stride + i].
__global__ void partial_sum_kernel(int nblk, int count, int stride, int nsub, int sub_stride,
                                   const float* __restrict__ part, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  // eight independent partial sums keep eight loads in flight (the loop is latency-bound);
  // the fixed combination order keeps the result deterministic
  const int n = nblk * nsub;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto at = [&](int r) { return part[(int64_t)(r / nsub) * stride + (r % nsub) * sub_stride + i]; };
  int r = 0;
  for (; r + 8 <= n; r += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += at(r + u);
  }
  for (; r < n; ++r) a[0] += at(r);
  out[i] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// BCEWithLogitsLoss (mean over all B x C logits, main.py:91): per-element loss terms (summed by
// the caller) and dL/dz = (sigmoid(z) - y) / (B C).
__global__ void bce_logits_kernel(int64_t n, const float* __restrict__ z, const float* __restrict__ y,
                                  float* __restrict__ loss_terms, float* __restrict__ gz) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float zi = z[i], yi = y[i];
  // max(z, 0) - z y + log(1 + exp(-|z|)): torch's stable form
  loss_terms[i] = fmaxf(zi, 0.f) - zi * yi + log1pf(expf(-fabsf(zi)));
  gz[i] = (1.f / (1.f + expf(-zi)) - yi) / (float)n;
}

}  // namespace
}  // namespace mvml

using namespace mvml;

extern "C" int mvml_layernorm_fwd(int64_t rows, int D, const float* x, int64_t ldx,
                                  const float* gamma, const float* beta, float eps, float* y,
                                  int64_t ldy, float* mean, float* rstd, void* stream) {
  clear_error();
  MVML_REQUIRE(rows >= 0 && D > 0 && D <= 64 * kFuseMaxVpl && ldx >= D && ldy >= D,
               "layernorm_fwd: bad shape (D must be <= %d)", 64 * kFuseMaxVpl);
  if (rows == 0) return MVML_OK;
  layernorm_fwd_kernel<<<(unsigned)ceil_div(rows, 4), 256, 0, as_stream(stream)>>>(
      rows, D, x, ldx, gamma, beta, eps, y, ldy, mean, rstd);
  return check_launch("layernorm_fwd_kernel");
}

extern "C" int mvml_layernorm_bwd(int64_t rows, int D, const float* x, int64_t ldx,
                                  const float* gamma, const float* mean, const float* rstd,
                                  const float* g_y, int64_t ldgy, float* g_x, int64_t ldgx,
                                  float* g_y_xhat, void* stream) {
  clear_error();
  MVML_REQUIRE(rows >= 0 && D > 0 && D <= 64 * kFuseMaxVpl && ldx >= D && ldgy >= D && ldgx >= D,
               "layernorm_bwd: bad shape");
  if (rows == 0) return MVML_OK;
  layernorm_bwd_kernel<<<(unsigned)ceil_div(rows, 4), 256, 0, as_stream(stream)>>>(
      rows, D, x, ldx, gamma, mean, rstd, g_y, ldgy, g_x, ldgx, g_y_xhat);
  return check_launch("layernorm_bwd_kernel");
}

extern "C" int mvml_token_attn_fwd(int64_t B, int H, int dk, const float* qkv, int64_t ld,
                                   float scale, float* att, float* P, void* stream) {
  clear_error();
  MVML_REQUIRE(B >= 0 && H > 0 && dk == 64 * kDkVpl && ld >= 3 * (int64_t)H * dk,
               "token_attn_fwd: dk must be %d and ld >= 3*H*dk", 64 * kDkVpl);
  if (B == 0) return MVML_OK;
  token_attn_fwd_kernel<<<(unsigned)ceil_div(B * H, 4), 256, 0, as_stream(stream)>>>(
      B, H, dk, qkv, ld, scale, att, P);
  return check_launch("token_attn_fwd_kernel");
}

extern "C" int mvml_token_attn_bwd(int64_t B, int H, int dk, const float* qkv, int64_t ld,
                                   float scale, const float* P, const float* g_att,
                                   float* g_qkv, int64_t ldg, void* stream) {
  clear_error();
  MVML_REQUIRE(B >= 0 && H > 0 && dk == 64 * kDkVpl && ld >= 3 * (int64_t)H * dk &&
                   ldg >= 3 * (int64_t)H * dk,
               "token_attn_bwd: bad shape");
  if (B == 0) return MVML_OK;
  token_attn_bwd_kernel<<<(unsigned)ceil_div(B * H, 4), 256, 0, as_stream(stream)>>>(
      B, H, dk, qkv, ld, scale, P, g_att, g_qkv, ldg);
  return check_launch("token_attn_bwd_kernel");
}

extern "C" int mvml_token_attn_fold_fwd(int64_t B, int H, int dk, const float* pv, int64_t ld,
                                        const float* x, int64_t ldx, float scale, float* att,
                                        float* P, void* stream) {
  clear_error();
  MVML_REQUIRE(B >= 0 && H > 0 && dk == 64 * kDkVpl && ld >= 2 * (int64_t)H * dk && ldx >= dk,
               "token_attn_fold_fwd: dk must be %d, ld >= 2*H*dk", 64 * kDkVpl);
  if (B == 0) return MVML_OK;
  token_attn_fold_fwd_kernel<<<(unsigned)ceil_div(B, 4), 256, 0, as_stream(stream)>>>(
      B, H, dk, pv, ld, x, ldx, scale, att, P);
  return check_launch("token_attn_fold_fwd_kernel");
}

extern "C" int mvml_token_attn_fold_bwd(int64_t B, int H, int dk, const float* pv, int64_t ld,
                                        const float* x, int64_t ldx, float scale, const float* P,
                                        const float* g_att, float* g_pv, int64_t ldg, float* g_k,
                                        int64_t ldgk, uint32_t* gpv_amax, void* stream) {
  clear_error();
  MVML_REQUIRE(B >= 0 && H > 0 && dk == 64 * kDkVpl && ld >= 2 * (int64_t)H * dk && ldx >= dk &&
                   ldg >= 2 * (int64_t)H * dk && ldgk >= dk,
               "token_attn_fold_bwd: bad shape");
  if (B == 0) return MVML_OK;
  token_attn_fold_bwd_kernel<<<(unsigned)ceil_div(B, 4), 256, 0, as_stream(stream)>>>(
      B, H, dk, pv, ld, x, ldx, scale, P, g_att, g_pv, ldg, g_k, ldgk, gpv_amax);
  return check_launch("token_attn_fold_bwd_kernel");
}

static int64_t conv3_blocks(int64_t B) { return std::min<int64_t>(B, 512); }  // 2 per CU

extern "C" int mvml_conv3_fwd(int64_t B, int C, int O, int W, const float* in, const float* weight,
                              const float* bias, float* out, void* stream) {
  clear_error();
  MVML_REQUIRE(C == kConvC && O == kConvO && W >= 3 && W <= 384, "conv3_fwd: C = O = 12, 3 <= W <= 384");
  if (B == 0) return MVML_OK;
#ifndef MVML_CONV_V1
  const int64_t nblk = conv3_blocks(B), per = ceil_div(B, nblk);
  conv3_fwd3_kernel<<<(unsigned)ceil_div(B, per), kConvThreads, 0, as_stream(stream)>>>(
      B, W, per, in, weight, bias, out);
#else
  conv3_fwd_kernel<<<(unsigned)B, kConvThreads, 0, as_stream(stream)>>>(B, W, in, weight, bias, out);
#endif
  return check_launch("conv3_fwd_kernel");
}


extern "C" size_t mvml_conv3_bwd_workspace_size(int64_t B) {
  return carve_size((size_t)conv3_blocks(B > 0 ? B : 1) * kConvPart * sizeof(float));
}

extern "C" int mvml_conv3_bwd(int64_t B, int C, int O, int W, const float* in, const float* weight,
                              const float* out, const float* g_out, float* g_in, float* g_weight,
                              float* g_bias, void* workspace, size_t workspace_bytes,
                              void* stream) {
  clear_error();
  MVML_REQUIRE(C == kConvC && O == kConvO && W >= 3 && W <= 384, "conv3_bwd: C = O = 12, 3 <= W <= 384");
  if (B == 0) return MVML_OK;
  if (!workspace || workspace_bytes < mvml_conv3_bwd_workspace_size(B)) {
    set_error("conv3_bwd: workspace of mvml_conv3_bwd_workspace_size bytes required");
    return MVML_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const int64_t nblk = conv3_blocks(B), per = ceil_div(B, nblk);
  const int64_t used = ceil_div(B, per);
  float* part = static_cast<float*>(workspace);
#ifndef MVML_CONV_V1
  conv3_bwd2_kernel<<<(unsigned)used, kConvThreads, 0, st>>>(B, W, per, in, weight, out, g_out,
                                                             g_in, part);
  const int nsub = 1;  // partial row: the 1296 weight sums, then (at 2 * 1296) the 12 bias sums
#else
  conv3_bwd_kernel<<<(unsigned)used, kConvThreads, 0, st>>>(B, W, per, in, weight, out, g_out,
                                                            g_in, part);
  const int nsub = 2;  // partial row: two column halves of the 1296 weight sums, then the biases
#endif
  int rc = check_launch("conv3_bwd_kernel");
  if (rc) return rc;
  partial_sum_kernel<<<(unsigned)ceil_div(kConvWg, 256), 256, 0, st>>>(
      (int)used, kConvWg, kConvPart, nsub, kConvWg, part, g_weight);
  rc = check_launch("partial_sum_kernel(w)");
  if (rc) return rc;
  partial_sum_kernel<<<1, 64, 0, st>>>((int)used, kConvO, kConvPart, 1, 0, part + 2 * kConvWg, g_bias);
  return check_launch("partial_sum_kernel(b)");
}

static int64_t fused_blocks(int64_t B) { return std::min<int64_t>(B, 256); }  // 1 per CU

extern "C" int mvml_attn_conv_fwd(int64_t B, int H, int dk, const float* pv, int64_t ld,
                                  const float* x, int64_t ldx, float scale, const float* weight,
                                  const float* bias, float* P, float* out, double drop_p,
                                  int64_t drop_seed, void* stream) {
  clear_error();
  MVML_REQUIRE(B >= 0 && H == kConvC && dk == 64 * kDkVpl && ld >= 2 * (int64_t)H * dk && ldx >= dk,
               "attn_conv_fwd: H must be %d, dk %d, ld >= 2*H*dk, ldx >= dk", kConvC, 64 * kDkVpl);
  MVML_REQUIRE(drop_p >= 0.0 && drop_p < 1.0, "attn_conv_fwd: dropout p must be in [0, 1)");
  if (B == 0) return MVML_OK;
  const int64_t nblk = fused_blocks(B), per = ceil_div(B, nblk);
  attn_conv_fwd_kernel<<<(unsigned)ceil_div(B, per), kFuseThreads, 0, as_stream(stream)>>>(
      B, per, pv, ld, x, ldx, scale, weight, bias, P, out, drop_p > 0.0 ? dropout_threshold(drop_p) : 0u,
      dropout_scale(drop_p), (uint64_t)drop_seed);
  return check_launch("attn_conv_fwd_kernel");
}

extern "C" size_t mvml_attn_conv_bwd_workspace_size(int64_t B) {
  return carve_size((size_t)fused_blocks(B > 0 ? B : 1) * kConvPart * sizeof(float));
}

extern "C" int mvml_attn_conv_bwd(int64_t B, int H, int dk, const float* pv, int64_t ld,
                                  const float* x, int64_t ldx, float scale, const float* P,
                                  const float* weight, const float* out, const float* g_out,
                                  float g_scale, float* g_pv, int64_t ldg, float* g_k, int64_t ldgk,
                                  uint32_t* g_pv_amax, uint32_t* g_pv_rows, float* g_weight,
                                  float* g_bias, void* workspace, size_t workspace_bytes,
                                  void* stream) {
  clear_error();
  MVML_REQUIRE(B >= 0 && H == kConvC && dk == 64 * kDkVpl && ld >= 2 * (int64_t)H * dk &&
                   ldx >= dk && ldg >= 2 * (int64_t)H * dk && ldgk >= dk,
               "attn_conv_bwd: H must be %d, dk %d, ld / ldg >= 2*H*dk, ldx / ldgk >= dk", kConvC,
               64 * kDkVpl);
  if (B == 0) return MVML_OK;
  if (!workspace || workspace_bytes < mvml_attn_conv_bwd_workspace_size(B)) {
    set_error("attn_conv_bwd: workspace of mvml_attn_conv_bwd_workspace_size bytes required");
    return MVML_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const int64_t nblk = fused_blocks(B), per = ceil_div(B, nblk);
  const int64_t used = ceil_div(B, per);
  float* part = static_cast<float*>(workspace);
  attn_conv_bwd_kernel<<<(unsigned)used, kFuseThreads, 0, st>>>(
      B, per, pv, ld, x, ldx, scale, P, weight, out, g_out, g_scale, g_pv, ldg, g_k, ldgk, g_pv_amax,
      part, g_pv_rows);
  int rc = check_launch("attn_conv_bwd_kernel");
  if (rc) return rc;
  partial_sum_kernel<<<(unsigned)ceil_div(kConvWg, 256), 256, 0, st>>>(
      (int)used, kConvWg, kConvPart, 1, kConvWg, part, g_weight);
  rc = check_launch("partial_sum_kernel(w)");
  if (rc) return rc;
  partial_sum_kernel<<<1, 64, 0, st>>>((int)used, kConvO, kConvPart, 1, 0, part + 2 * kConvWg, g_bias);
  return check_launch("partial_sum_kernel(b)");
}

extern "C" int mvml_bce_logits(int64_t n, const float* z, const float* y, float* loss_terms,
                               float* g_z, void* stream) {
  clear_error();
  MVML_REQUIRE(n >= 0, "bce_logits: bad size");
  if (n == 0) return MVML_OK;
  bce_logits_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, as_stream(stream)>>>(n, z, y, loss_terms, g_z);
  return check_launch("bce_logits_kernel");
}
