// Fused GAT attention + aggregation (dgl 0.9.1 GATConv.forward after fc/res_fc) and its
// atomic-free backward.  One wavefront per destination atom (two for wide layers).
//
// Projection row layout (the plain fc / res_fc GEMM, see mvml_gat_fold_weights):
//   Y[n] = [ Z (H*F) | R (RW) ]            RW = H*F (flatten modes) or F (mean mode)
// In mean mode (dgllife's last GATLayer, agg 'mean') only the head-mean of the residual is ever
// used, so the GEMM produces R_mean = X * mean_h(W_res_h)^T directly (F columns instead of H*F).
//
// Forward, per destination v (rows of the in-CSR, in-edges in ascending edge id):
//   el[n,h] = <Z[n,h,:], attn_l[h,:]>, er[n,h] = <Z[n,h,:], attn_r[h,:]>   GATConv el / er, from
//             Z exactly like `(feat_src * attn_l).sum(-1)`; saved to elr[n] = [el | er]
//   s_e   = LeakyReLU(el[src_e] + er[v], slope)                apply_edges(u_add_v), leaky_relu
//   a_e   = exp(s_e - max_v s) / sum_v exp(s - max_v s)       edge_softmax (norm_by = dst)
//   rst_v = sum_e a_e * Z[src_e] + R[v] + bias                update_all(u_mul_e, sum), res, bias
//   out_v = ELU(rst_v.flatten) | mean_h(rst_v) | rst_v        dgllife GATLayer agg / activation
// Two launches: gat_logits_kernel streams Z once into the compact elr array, then the
// aggregation kernel gathers 16-B logits per in-edge for the softmax and the Z rows for the sum.
// (A single-pass variant that reduces el[u] from each gathered Z row with an online softmax was
// measured 2x slower: its per-edge shuffle -> exp -> rescale chain is latency-bound.)
//
// Backward (two passes, no float atomics):
//   A (per dst v):  g_a_e = <Z[src_e], g_rst[v]>_f per head; g_s = a*(g_a - sum_v a*g_a);
//                   g_pre = g_s * leaky'(s_e); d er[v] = sum_e g_pre; dR[v] = g_rst[v] (or
//                   g_out[v] for the head-mean residual)                 -> gpre_ws, gelr, gY
//   B (per src u):  dZ[u] = sum_{e: u->w} a_e * g_rst[w] + d el[u] attn_l + d er[u] attn_r,
//                   d el[u] = sum_{e: u->w} g_pre_e (gather over the out-CSR; out_inslot maps an
//                   out-edge to its in-CSR slot; g_rst[w] rows come back from gY's dR block)
//   dL/dattn_{l,r} = sum_n d{el,er}[n,h] Z[n,h,:]   (mvml_gat_attn_grad, directly over atoms)
//
// Workgroup -> atom mapping is XCD-aware (xcd_block): each XCD walks one contiguous range of
// atoms, so a molecule's neighbour rows are gathered from ONE XCD's L2.
#include "common.h"

namespace mvml {
namespace {

constexpr int kWavesPerBlock = 4;
#ifndef MVML_FWD_UNR
#define MVML_FWD_UNR 2  // neighbour rows in flight per gather step (forward)
#endif

__device__ __forceinline__ float rl(float x, int j) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), j));
}
__device__ __forceinline__ int rl(int x, int j) { return __builtin_amdgcn_readlane(x, j); }

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float leaky(float x, float slope) { return x > 0.f ? x : x * slope; }
__device__ __forceinline__ float elu(float x) { return x > 0.f ? x : expm1f(x); }

__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }
__device__ __forceinline__ float4 fma4(float a, float4 z, float4 c) {
  return make_float4(fmaf(a, z.x, c.x), fmaf(a, z.y, c.y), fmaf(a, z.z, c.z), fmaf(a, z.w, c.w));
}
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float dot4(float4 a, float4 b) {
  return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

template <int H>
__device__ __forceinline__ float pick(const float (&a)[H], int h) {
  float r = a[0];
#pragma unroll
  for (int k = 1; k < H; ++k) r = (h == k) ? a[k] : r;
  return r;
}
template <int H>
__device__ __forceinline__ void add_at(float (&a)[H], int h, float v) {
#pragma unroll
  for (int k = 0; k < H; ++k) a[k] += (h == k) ? v : 0.f;
}
// wave-uniform per-head values -> p[0..H): lane h stores a[h]
template <int H>
__device__ __forceinline__ void store_heads(float* p, const float (&a)[H], int lane) {
  if (lane < H) p[lane] = pick<H>(a, lane);
}

// All-reduce of H per-lane values over the 64 lanes in (H - 1) + (6 - log2 H) shuffles instead
// of 6 H: a butterfly that halves the value count per step (lanes with the mask bit set keep
// the upper half) and then finishes the single remaining value inside 64/H-lane groups.  After
// it, lane l holds the total of head ((l >> (6 - log2 H)) & (H - 1)); readlane broadcasts them.
template <int H>
struct HeadReduce {
  static constexpr int LOG = H == 1 ? 0 : H == 2 ? 1 : H == 4 ? 2 : 3;
  template <bool MAX>
  __device__ static __forceinline__ float op(float a, float b) { return MAX ? fmaxf(a, b) : a + b; }
  template <bool MAX>
  __device__ static __forceinline__ void all(float (&v)[H], int lane) {
    float w[H];
#pragma unroll
    for (int h = 0; h < H; ++h) w[h] = v[h];
    if constexpr (H >= 8) step<MAX, 8>(w, lane, 32);
    if constexpr (H >= 4) step<MAX, 4>(w, lane, 32 >> (LOG - 2));
    if constexpr (H >= 2) step<MAX, 2>(w, lane, 32 >> (LOG - 1));
#pragma unroll
    for (int m = 32 >> LOG; m >= 1; m >>= 1) w[0] = op<MAX>(w[0], __shfl_xor(w[0], m, 64));
#pragma unroll
    for (int h = 0; h < H; ++h)
      v[h] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w[0]), h << (6 - LOG)));
  }
  template <bool MAX, int N>
  __device__ static __forceinline__ void step(float (&w)[H], int lane, int mask) {
    const bool hi = (lane & mask) != 0;
#pragma unroll
    for (int i = 0; i < N / 2; ++i) {
      const float keep = hi ? w[i + N / 2] : w[i];
      const float send = hi ? w[i] : w[i + N / 2];
      w[i] = op<MAX>(keep, __shfl_xor(send, mask, 64));
    }
  }
};

// g_rst[v, col..col+3] (per-head gradient of rst) from the layer-output gradient.
__device__ __forceinline__ float4 grst_of(const float* __restrict__ g_out, const float* __restrict__ out,
                                          int64_t v, int col, int HF, int F, int H, int mode) {
  if (mode == 1) {  // mean over heads: torch mean backward = grad / H
    const float4 g = ld4(g_out + v * F + (col % F));
    const float inv = (float)H;
    return make_float4(g.x / inv, g.y / inv, g.z / inv, g.w / inv);
  }
  float4 g = ld4(g_out + v * HF + col);
  if (mode == 0) {  // ELU'(x) = 1 (x > 0) else exp(x) = out + 1 (torch elu_backward, is_result)
    const float4 o = ld4(out + v * HF + col);
    g.x *= o.x > 0.f ? 1.f : o.x + 1.f;
    g.y *= o.y > 0.f ? 1.f : o.y + 1.f;
    g.z *= o.z > 0.f ? 1.f : o.z + 1.f;
    g.w *= o.w > 0.f ? 1.f : o.w + 1.f;
  }
  return g;
}

// ---------------------------------------------------------------------------------- forward
// Logits: el[n,h] = <Z[n,h,:], attn_l[h,:]>, er likewise, one wave per atom (a streaming read of
// Z, 16-B slices per lane, butterfly head reduction).  elr[n] = [el | er] is a compact [N, 2H]
// array, so the aggregation gathers a neighbour's logits as one 16-B load instead of reaching
// into Y's wide rows.
template <int H, int VPL>
__global__ void __launch_bounds__(kWavesPerBlock * 64)
gat_logits_kernel(int64_t N, const float* __restrict__ Y, int64_t ldy, int F,
                  const float* __restrict__ attn_l, const float* __restrict__ attn_r,
                  float* __restrict__ elr) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t v = (int64_t)blockIdx.x * kWavesPerBlock + wid;
  if (v >= N) return;
  const int HF = H * F;
  const float* yv = Y + v * ldy;
  float el[H], er[H];
#pragma unroll
  for (int h = 0; h < H; ++h) { el[h] = 0.f; er[h] = 0.f; }
#pragma unroll
  for (int c = 0; c < VPL; ++c) {
    const int col = 4 * (lane + 64 * c);
    if (col < HF) {
      const float4 z = ld4(yv + col);
      const int h = col / F;
      add_at<H>(el, h, dot4(z, ld4(attn_l + col)));
      add_at<H>(er, h, dot4(z, ld4(attn_r + col)));
    }
  }
  HeadReduce<H>::template all<false>(el, lane);
  HeadReduce<H>::template all<false>(er, lane);
  store_heads<H>(elr + v * 2 * H, el, lane);
  store_heads<H>(elr + v * 2 * H + H, er, lane);
}

// Aggregation.  A wave owns a GROUP of 64 consecutive destination atoms (CS waves share a
// group, each owning F / CS columns of EVERY head, so a wave never needs another wave's data).
//  1. Prologue, lane i <-> atom v0 + i: the softmax statistics of the atom's in-edges (max,
//     then sum of exp, exactly dgl's edge_softmax) from the gathered logits, the first DC
//     logits cached in registers; the attention a_e is written (part-0 wave).  The dependent
//     rowptr -> in_src -> elr chains of 64 atoms are in flight together.
//  2. Edge stream: the group's in-edges are contiguous in the in-CSR, so the wave walks them
//     UNR at a time regardless of atom boundaries (source ids from a 64-edge register chunk via
//     readlane, no per-atom index round trip): UNR neighbour rows Z[u] (16-B column slices per
//     lane) and their logits are loaded together, a_e is recomputed bit-identically from the
//     atom's statistics, and an atom is finished (residual prefetched when it starts) as soon
//     as the stream passes its last edge.
//  3. Epilogue per atom: + residual + bias, then flatten+ELU / flatten, or the head mean
//     through a wave-private LDS transpose.
template <int H, int VPL, int CS, int UNR>
__global__ void __launch_bounds__(kWavesPerBlock * 64)
gat_agg_fwd_kernel(int64_t N, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ in_src,
                   const float* __restrict__ Y, int64_t ldy, int F, const float* __restrict__ elr,
                   const float* __restrict__ bias, float slope, int mode, float* __restrict__ out,
                   float* __restrict__ attn) {
  constexpr int DC = 4;  // logits cached per atom in the prologue
  __shared__ __attribute__((aligned(16))) float red[kWavesPerBlock][VPL * 256];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t wave = xcd_block(blockIdx.x, gridDim.x) * kWavesPerBlock + wid;
  const int part = (int)(wave % CS);
  const int64_t v0 = (wave / CS) * 64;
  if (v0 >= N) return;
  const int HF = H * F, FW = F / CS, HFW = HF / CS;

  // ---- 1. prologue: softmax statistics, lane per atom ----
  const int64_t vl = v0 + lane;
  const bool lv = vl < N;
  int beg_l = 0, end_l = 0;
  if (lv) { beg_l = rowptr[vl]; end_l = rowptr[vl + 1]; }
  float er_l[H], m_l[H], s_l[H], sc[DC][H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    er_l[h] = lv ? elr[vl * 2 * H + H + h] : 0.f;
    m_l[h] = -INFINITY;
    s_l[h] = 0.f;
  }
#pragma unroll
  for (int t = 0; t < DC; ++t) {
    const int j = beg_l + t;
    const float* eu = elr + (int64_t)(j < end_l ? in_src[j] : 0) * 2 * H;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      sc[t][h] = leaky(eu[h] + er_l[h], slope);
      if (j < end_l) m_l[h] = fmaxf(m_l[h], sc[t][h]);
    }
  }
  for (int j = beg_l + DC; j < end_l; ++j) {
    const float* eu = elr + (int64_t)in_src[j] * 2 * H;
#pragma unroll
    for (int h = 0; h < H; ++h) m_l[h] = fmaxf(m_l[h], leaky(eu[h] + er_l[h], slope));
  }
#pragma unroll
  for (int t = 0; t < DC; ++t)
    if (beg_l + t < end_l) {
#pragma unroll
      for (int h = 0; h < H; ++h) s_l[h] += expf(sc[t][h] - m_l[h]);
    }
  for (int j = beg_l + DC; j < end_l; ++j) {
    const float* eu = elr + (int64_t)in_src[j] * 2 * H;
#pragma unroll
    for (int h = 0; h < H; ++h) s_l[h] += expf(leaky(eu[h] + er_l[h], slope) - m_l[h]);
  }
  if (part == 0) {
#pragma unroll
    for (int t = 0; t < DC; ++t)
      if (beg_l + t < end_l) {
#pragma unroll
        for (int h = 0; h < H; ++h)
          attn[(int64_t)(beg_l + t) * H + h] = expf(sc[t][h] - m_l[h]) / s_l[h];
      }
    for (int j = beg_l + DC; j < end_l; ++j) {
      const float* eu = elr + (int64_t)in_src[j] * 2 * H;
#pragma unroll
      for (int h = 0; h < H; ++h)
        attn[(int64_t)j * H + h] = expf(leaky(eu[h] + er_l[h], slope) - m_l[h]) / s_l[h];
    }
  }

  // ---- column map of this lane: wave column j -> (head, f) -> global column ----
  int hc[VPL], gcol[VPL];
  bool okc[VPL];
  float4 bc[VPL];
#pragma unroll
  for (int c = 0; c < VPL; ++c) {
    const int j = 4 * (lane + 64 * c);
    okc[c] = j < HFW;
    hc[c] = okc[c] ? j / FW : 0;
    gcol[c] = okc[c] ? hc[c] * F + part * FW + j % FW : 0;
    bc[c] = okc[c] ? ld4(bias + gcol[c]) : f4(0.f);
  }

  // ---- 2./3. edge stream + per-atom epilogue ----
  const int nv = (int)min<int64_t>(64, N - v0);
  int k = 0, kend = 0;
  float M[H], S[H], ER[H];
  float4 r[VPL], acc[VPL];
  auto start_atom = [&](int kk) {
    kend = rl(end_l, kk);
#pragma unroll
    for (int h = 0; h < H; ++h) { M[h] = rl(m_l[h], kk); S[h] = rl(s_l[h], kk); ER[h] = rl(er_l[h], kk); }
    if (mode != 1) {
      const float* rv = Y + (v0 + kk) * ldy + HF;
#pragma unroll
      for (int c = 0; c < VPL; ++c) r[c] = okc[c] ? ld4(rv + gcol[c]) : f4(0.f);
    }
#pragma unroll
    for (int c = 0; c < VPL; ++c) acc[c] = f4(0.f);
  };
  auto finish_atom = [&](int kk) {
    const int64_t v = v0 + kk;
    if (mode == 1) {
      // head mean: rst + bias of every head -> LDS, then sum heads h = 0..H-1 per column
      float* rr = red[wid];
#pragma unroll
      for (int c = 0; c < VPL; ++c)
        if (okc[c]) st4(rr + 4 * (lane + 64 * c), add4(acc[c], bc[c]));
      wave_lds_sync();
      const float invh = (float)H;
      const float* rm_row = Y + v * ldy + HF + part * FW;  // head-mean residual
      for (int f = 4 * lane; f < FW; f += 256) {
        float4 s = ld4(rr + f);
#pragma unroll
        for (int h = 1; h < H; ++h) s = add4(s, ld4(rr + h * FW + f));
        const float4 rm = ld4(rm_row + f);
        st4(out + v * F + part * FW + f, make_float4(s.x / invh + rm.x, s.y / invh + rm.y,
                                                     s.z / invh + rm.z, s.w / invh + rm.w));
      }
      wave_lds_sync();
    } else {
#pragma unroll
      for (int c = 0; c < VPL; ++c)
        if (okc[c]) {
          float4 o = add4(add4(acc[c], r[c]), bc[c]);
          if (mode == 0) o = make_float4(elu(o.x), elu(o.y), elu(o.z), elu(o.w));
          st4(out + v * HF + gcol[c], o);
        }
    }
  };

  start_atom(0);
  const int E0 = rl(beg_l, 0), E1 = rl(end_l, nv - 1);
  for (int cb = E0; cb < E1; cb += 64) {
    const int cnt = min(64, E1 - cb);
    const int u_c = (lane < cnt) ? in_src[cb + lane] : 0;
    for (int i = 0; i < cnt; i += UNR) {
      float4 z[UNR][VPL];
      float el[UNR][H];
#pragma unroll
      for (int t = 0; t < UNR; ++t) {
        const int u = rl(u_c, min(i + t, cnt - 1));
        const float* zu = Y + (int64_t)u * ldy;
#pragma unroll
        for (int c = 0; c < VPL; ++c) z[t][c] = okc[c] ? ld4(zu + gcol[c]) : f4(0.f);
        const float* eu = elr + (int64_t)u * 2 * H;
#pragma unroll
        for (int h = 0; h < H; ++h) el[t][h] = eu[h];
      }
#pragma unroll
      for (int t = 0; t < UNR; ++t) {
        if (i + t < cnt) {
          while (cb + i + t >= kend) {  // the stream passed atom k's last edge
            finish_atom(k);
            start_atom(++k);
          }
          float a[H];
#pragma unroll
          for (int h = 0; h < H; ++h) a[h] = expf(leaky(el[t][h] + ER[h], slope) - M[h]) / S[h];
#pragma unroll
          for (int c = 0; c < VPL; ++c)
            if (okc[c]) acc[c] = fma4(pick<H>(a, hc[c]), z[t][c], acc[c]);
        }
      }
    }
  }
  // the last atom with edges and any trailing atoms without
  for (;;) {
    finish_atom(k);
    if (++k >= nv) break;
    start_atom(k);
  }
}

// --------------------------------------------------------------------------------- backward
// Pass A: one wave per destination v.
template <int H, int VPL>
__global__ void __launch_bounds__(kWavesPerBlock * 64)
gat_agg_bwd_dst_kernel(int64_t N, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ in_src,
                       const float* __restrict__ Y, int64_t ldy, const float* __restrict__ elr,
                       const float* __restrict__ attn, const float* __restrict__ out,
                       const float* __restrict__ g_out, int F, float slope, int mode,
                       float* __restrict__ gpre, float* __restrict__ gY, int64_t ldgy,
                       float* __restrict__ gelr) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t v = xcd_block(blockIdx.x, gridDim.x) * kWavesPerBlock + wid;
  if (v >= N) return;
  const int HF = H * F;
  const int beg = rowptr[v], end = rowptr[v + 1];
  const int deg = end - beg;
  int hc[VPL];
  bool okc[VPL];
  float4 gr[VPL];
#pragma unroll
  for (int c = 0; c < VPL; ++c) {
    const int col = 4 * (lane + 64 * c);
    okc[c] = col < HF;
    hc[c] = okc[c] ? col / F : 0;
    gr[c] = okc[c] ? grst_of(g_out, out, v, col, HF, F, H, mode) : f4(0.f);
  }
  // dR[v]: per-head g_rst (flatten modes) or g_out (head-mean residual).  Written here so the
  // source pass can gather finished g_rst rows from gY instead of re-deriving them per edge.
  float* gyv = gY + v * ldgy;
#pragma unroll
  for (int c = 0; c < VPL; ++c) {
    const int col = 4 * (lane + 64 * c);
    if (mode != 1) {
      if (okc[c]) st4(gyv + HF + col, gr[c]);
    } else if (col < F) {
      st4(gyv + HF + col, ld4(g_out + v * F + col));
    }
  }
  float er[H];
#pragma unroll
  for (int h = 0; h < H; ++h) er[h] = elr[v * 2 * H + H + h];

  float dots[H];  // sum_e a_e * g_a_e per head
#pragma unroll
  for (int h = 0; h < H; ++h) dots[h] = 0.f;
  float ga_l[H], a_l[H];
  for (int base = 0; base < deg; base += 64) {
    const int cnt = min(64, deg - base);
    const int u_l = (base + lane < deg) ? in_src[beg + base + lane] : 0;
#pragma unroll
    for (int h = 0; h < H; ++h) ga_l[h] = 0.f;
    for (int j = 0; j < cnt; ++j) {
      const float* zu = Y + (int64_t)rl(u_l, j) * ldy;
      float part[H];
#pragma unroll
      for (int h = 0; h < H; ++h) part[h] = 0.f;
#pragma unroll
      for (int c = 0; c < VPL; ++c)
        if (okc[c]) add_at<H>(part, hc[c], dot4(ld4(zu + 4 * (lane + 64 * c)), gr[c]));
      HeadReduce<H>::template all<false>(part, lane);
#pragma unroll
      for (int h = 0; h < H; ++h) ga_l[h] = (lane == j) ? part[h] : ga_l[h];
    }
    const bool valid = base + lane < deg;
    float ag[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      a_l[h] = valid ? attn[(int64_t)(beg + base + lane) * H + h] : 0.f;
      ag[h] = a_l[h] * ga_l[h];
    }
    HeadReduce<H>::template all<false>(ag, lane);
#pragma unroll
    for (int h = 0; h < H; ++h) dots[h] += ag[h];
    if (deg > 64 && valid) {  // keep g_a for the second sweep
#pragma unroll
      for (int h = 0; h < H; ++h) gpre[(int64_t)(beg + base + lane) * H + h] = ga_l[h];
    }
  }
  float ger[H];
#pragma unroll
  for (int h = 0; h < H; ++h) ger[h] = 0.f;
  for (int base = 0; base < deg; base += 64) {
    const bool valid = base + lane < deg;
    const int64_t slot = beg + base + lane;
    float gp[H];
    if (valid) {
      const float* el_u = elr + (int64_t)in_src[slot] * 2 * H;
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const float a = (deg > 64) ? attn[slot * H + h] : a_l[h];
        const float ga = (deg > 64) ? gpre[slot * H + h] : ga_l[h];
        const float gs = a * (ga - dots[h]);
        gp[h] = (el_u[h] + er[h]) > 0.f ? gs : gs * slope;
        gpre[slot * H + h] = gp[h];
      }
    } else {
#pragma unroll
      for (int h = 0; h < H; ++h) gp[h] = 0.f;
    }
    HeadReduce<H>::template all<false>(gp, lane);
#pragma unroll
    for (int h = 0; h < H; ++h) ger[h] += gp[h];
  }
  store_heads<H>(gelr + v * 2 * H + H, ger, lane);
}

// Pass B: one wave per source u (out-CSR gather).
template <int H, int VPL>
__global__ void __launch_bounds__(kWavesPerBlock * 64)
gat_agg_bwd_src_kernel(int64_t N, const int32_t* __restrict__ out_rowptr,
                       const int32_t* __restrict__ out_dst, const int32_t* __restrict__ out_inslot,
                       const float* __restrict__ attn, const float* __restrict__ gpre,
                       const float* __restrict__ attn_l, const float* __restrict__ attn_r,
                       const float* __restrict__ out, const float* __restrict__ g_out, int F,
                       int mode, float* __restrict__ gY, int64_t ldgy, float* __restrict__ gelr) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t u = xcd_block(blockIdx.x, gridDim.x) * kWavesPerBlock + wid;
  if (u >= N) return;
  const int HF = H * F;
  const int beg = out_rowptr[u], end = out_rowptr[u + 1];
  const int deg = end - beg;
  int hc[VPL];
  bool okc[VPL];
  float4 gz[VPL];
#pragma unroll
  for (int c = 0; c < VPL; ++c) {
    const int col = 4 * (lane + 64 * c);
    okc[c] = col < HF;
    hc[c] = okc[c] ? col / F : 0;
    gz[c] = f4(0.f);
  }
  float gel[H];
#pragma unroll
  for (int h = 0; h < H; ++h) gel[h] = 0.f;
  for (int base = 0; base < deg; base += 64) {
    const int cnt = min(64, deg - base);
    int w_l = 0;
    float a_l[H], gp_l[H];
    if (base + lane < deg) {
      w_l = out_dst[beg + base + lane];
      const int64_t js = out_inslot[beg + base + lane];
#pragma unroll
      for (int h = 0; h < H; ++h) { a_l[h] = attn[js * H + h]; gp_l[h] = gpre[js * H + h]; }
    } else {
#pragma unroll
      for (int h = 0; h < H; ++h) { a_l[h] = 0.f; gp_l[h] = 0.f; }
    }
    HeadReduce<H>::template all<false>(gp_l, lane);
#pragma unroll
    for (int h = 0; h < H; ++h) gel[h] += gp_l[h];
    for (int j = 0; j < cnt; ++j) {
      const int w = rl(w_l, j);
      float a[H];
#pragma unroll
      for (int h = 0; h < H; ++h) a[h] = rl(a_l[h], j);
      const float* gw = gY + (int64_t)w * ldgy + HF;  // g_rst row written by the dst pass
#pragma unroll
      for (int c = 0; c < VPL; ++c)
        if (okc[c]) {
          const int col = 4 * (lane + 64 * c);
          const float4 g = (mode == 1) ? grst_of(g_out, out, w, col, HF, F, H, mode) : ld4(gw + col);
          gz[c] = fma4(pick<H>(a, hc[c]), g, gz[c]);
        }
    }
  }
  // + the el / er paths: Z also feeds el = <Z, attn_l> and er = <Z, attn_r>
  float ger[H];
#pragma unroll
  for (int h = 0; h < H; ++h) ger[h] = gelr[u * 2 * H + H + h];
  float* gyu = gY + u * ldgy;
#pragma unroll
  for (int c = 0; c < VPL; ++c)
    if (okc[c]) {
      const int col = 4 * (lane + 64 * c);
      float4 g = fma4(pick<H>(gel, hc[c]), ld4(attn_l + col), gz[c]);
      g = fma4(pick<H>(ger, hc[c]), ld4(attn_r + col), g);
      st4(gyu + col, g);
    }
  store_heads<H>(gelr + u * 2 * H, gel, lane);
}

template <int H, int VPL>
int launch_fwd(int64_t N, const int32_t* rp, const int32_t* src, const float* Y, int64_t ldy, int F,
               const float* al, const float* ar, const float* bias, float slope, int mode, float* out,
               float* attn, float* elr, hipStream_t st) {
  gat_logits_kernel<H, VPL><<<(unsigned)ceil_div(N, kWavesPerBlock), kWavesPerBlock * 64, 0, st>>>(
      N, Y, ldy, F, al, ar, elr);
  int rc = check_launch("gat_logits_kernel");
  if (rc) return rc;
  // Wide layers (more than 4 float4 slices per lane) split every head's columns over 2 waves.
  if constexpr (VPL > 4) {
    constexpr int CS = 2, V2 = (VPL + 1) / 2;
    if (F % 8 != 0) {
      set_error("gat_agg_fwd: H*F > 1024 needs out_feats divisible by 8");
      return MVML_ERR_INVALID;
    }
    const unsigned blocks = (unsigned)ceil_div(ceil_div(N, 64) * CS, kWavesPerBlock);
    gat_agg_fwd_kernel<H, V2, CS, (V2 <= 3 ? MVML_FWD_UNR : 2)><<<blocks, kWavesPerBlock * 64, 0, st>>>(
        N, rp, src, Y, ldy, F, elr, bias, slope, mode, out, attn);
  } else {
    const unsigned blocks = (unsigned)ceil_div(ceil_div(N, 64), kWavesPerBlock);
    gat_agg_fwd_kernel<H, VPL, 1, (VPL <= 3 ? MVML_FWD_UNR : 2)><<<blocks, kWavesPerBlock * 64, 0, st>>>(
        N, rp, src, Y, ldy, F, elr, bias, slope, mode, out, attn);
  }
  return check_launch("gat_agg_fwd_kernel");
}

template <int H, int VPL>
int launch_bwd(int64_t N, const int32_t* rp, const int32_t* src, const int32_t* orp,
               const int32_t* odst, const int32_t* oslot, const float* Y, int64_t ldy,
               const float* elr, const float* attn, const float* al, const float* ar,
               const float* out, const float* g_out, int F, float slope, int mode, float* gpre,
               float* gY, int64_t ldgy, float* gelr, hipStream_t st) {
  const unsigned blocks = (unsigned)ceil_div(N, kWavesPerBlock);
  gat_agg_bwd_dst_kernel<H, VPL><<<blocks, kWavesPerBlock * 64, 0, st>>>(
      N, rp, src, Y, ldy, elr, attn, out, g_out, F, slope, mode, gpre, gY, ldgy, gelr);
  int rc = check_launch("gat_agg_bwd_dst_kernel");
  if (rc) return rc;
  gat_agg_bwd_src_kernel<H, VPL><<<blocks, kWavesPerBlock * 64, 0, st>>>(
      N, orp, odst, oslot, attn, gpre, al, ar, out, g_out, F, mode, gY, ldgy, gelr);
  return check_launch("gat_agg_bwd_src_kernel");
}

#define MVML_VPL_CASES(FN, H, ...)                 \
  switch (vpl) {                                   \
    case 1: return FN<H, 1>(__VA_ARGS__);          \
    case 2: return FN<H, 2>(__VA_ARGS__);          \
    case 3: return FN<H, 3>(__VA_ARGS__);          \
    case 4: return FN<H, 4>(__VA_ARGS__);          \
    case 5: return FN<H, 5>(__VA_ARGS__);          \
    case 6: return FN<H, 6>(__VA_ARGS__);          \
    case 7: return FN<H, 7>(__VA_ARGS__);          \
    case 8: return FN<H, 8>(__VA_ARGS__);          \
    default: break;                                \
  }

int check_shapes(int H, int F, int mode, int64_t ldy, const void* Y, const char* who) {
  MVML_REQUIRE(H == 1 || H == 2 || H == 4 || H == 8, "%s: num_heads must be 1, 2, 4 or 8 (got %d)", who, H);
  MVML_REQUIRE(F > 0 && F % 4 == 0, "%s: out_feats must be a positive multiple of 4 (got %d)", who, F);
  MVML_REQUIRE(H * F <= 2048, "%s: H*F must be <= 2048 (got %d)", who, H * F);
  MVML_REQUIRE(mode >= 0 && mode <= 2, "%s: bad mode %d", who, mode);
  const int64_t need = (int64_t)mvml_gat_proj_cols(H, F, mode == 1);
  MVML_REQUIRE(ldy >= need && ldy % 4 == 0, "%s: leading dimension %lld < %lld or not a multiple of 4",
               who, (long long)ldy, (long long)need);
  MVML_REQUIRE(((uintptr_t)Y & 15) == 0, "%s: tensors must be 16-byte aligned", who);
  return MVML_OK;
}

// ------------------------------------------------------------------ parameter-side helpers
// dL/dattn_l[h,f] = sum_n d el[n,h] * Z[n,h,f] (likewise attn_r with d er), summed directly over
// atoms as autograd does.  Stage 1: each thread owns one Z column over a chunk of atoms.
__global__ void attn_grad_partial_kernel(int64_t N, int H, int F, const float* __restrict__ Y,
                                         int64_t ldy, const float* __restrict__ gelr,
                                         int64_t rows_per, float* __restrict__ part) {
  const int HF = H * F;
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= HF) return;
  const int h = col / F;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per, r1 = min(N, r0 + rows_per);
  float sl[4] = {0.f, 0.f, 0.f, 0.f}, sr[4] = {0.f, 0.f, 0.f, 0.f};
  int64_t r = r0;
  for (; r + 4 <= r1; r += 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float z = Y[(r + j) * ldy + col];
      const float* g = gelr + (r + j) * 2 * H;
      sl[j] = fmaf(g[h], z, sl[j]);
      sr[j] = fmaf(g[H + h], z, sr[j]);
    }
  }
  for (; r < r1; ++r) {
    const float z = Y[r * ldy + col];
    const float* g = gelr + r * 2 * H;
    sl[0] = fmaf(g[h], z, sl[0]);
    sr[0] = fmaf(g[H + h], z, sr[0]);
  }
  part[((int64_t)blockIdx.y * 2 + 0) * HF + col] = (sl[0] + sl[1]) + (sl[2] + sl[3]);
  part[((int64_t)blockIdx.y * 2 + 1) * HF + col] = (sr[0] + sr[1]) + (sr[2] + sr[3]);
}

__global__ void attn_grad_final_kernel(int HF, int S, const float* __restrict__ part,
                                       float* __restrict__ g_al, float* __restrict__ g_ar) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // over 2*HF
  if (i >= 2 * HF) return;
  const int side = i / HF, col = i % HF;
  float s = 0.f;
  for (int z = 0; z < S; ++z) s += part[((int64_t)z * 2 + side) * HF + col];
  (side ? g_ar : g_al)[col] = s;
}

int attn_grad_splits(int64_t N, int HF) {
  const int64_t colblocks = ceil_div(HF, 256);
  int64_t s = ceil_div(2048, colblocks);
  s = std::min<int64_t>(s, ceil_div(N, 256));
  return (int)std::max<int64_t>(1, s);
}

// Wcat rows: [0,HF) fc.weight | [HF,HF+RW) res_fc.weight (RW = HF) or its head mean (RW = F);
// columns Fin..ldw-1 are zero.
__global__ void fold_weights_kernel(const float* __restrict__ fc_w, const float* __restrict__ res_w,
                                    int H, int F, int Fin, int ldw, int mean_res,
                                    float* __restrict__ Wcat) {
  const int HF = H * F;
  const int RW = mean_res ? F : HF;
  const int64_t total = (int64_t)(HF + RW) * ldw;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)(e / ldw), k = (int)(e % ldw);
    float v;
    if (k >= Fin) {
      v = 0.f;
    } else if (row < HF) {
      v = fc_w[(int64_t)row * Fin + k];
    } else {
      const int r = row - HF;
      if (mean_res) {
        float s = 0.f;
        for (int h = 0; h < H; ++h) s += res_w[(int64_t)(h * F + r) * Fin + k];
        v = s / (float)H;
      } else {
        v = res_w[(int64_t)r * Fin + k];
      }
    }
    Wcat[e] = v;
  }
}

// dL/dfc.weight = gWcat[0:HF];  dL/dres_fc.weight[hF+f] = gWcat[HF+hF+f] or gWcat[HF+f] / H.
__global__ void unfold_w_kernel(const float* __restrict__ gW, int H, int F, int Fin, int ldg,
                                int mean_res, float* __restrict__ g_fc, float* __restrict__ g_res) {
  const int HF = H * F;
  const int64_t total = (int64_t)HF * Fin;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)(e / Fin), k = (int)(e % Fin);
    g_fc[e] = gW[(int64_t)row * ldg + k];
    g_res[e] = mean_res ? gW[(int64_t)(HF + row % F) * ldg + k] / (float)H
                        : gW[(int64_t)(HF + row) * ldg + k];
  }
}

}  // namespace
}  // namespace mvml

using namespace mvml;

extern "C" int mvml_gat_proj_cols(int H, int F, int mean_residual) {
  return H * F + (mean_residual ? F : H * F);
}

extern "C" int mvml_gat_agg_fwd(int64_t num_nodes, const int32_t* in_rowptr, const int32_t* in_src,
                                const float* Y, int64_t ldy, int H, int F, const float* attn_l,
                                const float* attn_r, const float* bias, float slope, int mode,
                                float* out, float* attn, float* elr, void* stream) {
  clear_error();
  int rc = check_shapes(H, F, mode, ldy, Y, "gat_agg_fwd");
  if (rc) return rc;
  MVML_REQUIRE(((uintptr_t)out & 15) == 0 && ((uintptr_t)bias & 15) == 0 &&
               ((uintptr_t)attn_l & 15) == 0 && ((uintptr_t)attn_r & 15) == 0,
               "gat_agg_fwd: out / bias / attention vectors must be 16-byte aligned");
  MVML_REQUIRE(attn != nullptr && elr != nullptr, "gat_agg_fwd: attn and elr outputs are required");
  if (num_nodes == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  const int vpl = (int)ceil_div(H * F, 256);
  switch (H) {
    case 1: { MVML_VPL_CASES(launch_fwd, 1, num_nodes, in_rowptr, in_src, Y, ldy, F, attn_l, attn_r, bias, slope, mode, out, attn, elr, st) break; }
    case 2: { MVML_VPL_CASES(launch_fwd, 2, num_nodes, in_rowptr, in_src, Y, ldy, F, attn_l, attn_r, bias, slope, mode, out, attn, elr, st) break; }
    case 4: { MVML_VPL_CASES(launch_fwd, 4, num_nodes, in_rowptr, in_src, Y, ldy, F, attn_l, attn_r, bias, slope, mode, out, attn, elr, st) break; }
    case 8: { MVML_VPL_CASES(launch_fwd, 8, num_nodes, in_rowptr, in_src, Y, ldy, F, attn_l, attn_r, bias, slope, mode, out, attn, elr, st) break; }
  }
  set_error("gat_agg_fwd: unsupported shape");
  return MVML_ERR_INVALID;
}

extern "C" size_t mvml_gat_agg_bwd_workspace_size(int64_t num_edges, int H) {
  return carve_size((size_t)num_edges * H * sizeof(float));
}

extern "C" int mvml_gat_agg_bwd(int64_t num_nodes, const int32_t* in_rowptr, const int32_t* in_src,
                                const int32_t* out_rowptr, const int32_t* out_dst,
                                const int32_t* out_inslot, const float* Y, int64_t ldy,
                                const float* elr, const float* attn, const float* attn_l,
                                const float* attn_r, const float* out, const float* g_out, int H,
                                int F, float slope, int mode, float* gY, int64_t ldgy, float* gelr,
                                void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  int rc = check_shapes(H, F, mode, ldy, Y, "gat_agg_bwd");
  if (rc) return rc;
  MVML_REQUIRE(ldgy >= mvml_gat_proj_cols(H, F, mode == 1) && ldgy % 4 == 0, "gat_agg_bwd: bad ldgy");
  MVML_REQUIRE(attn != nullptr && elr != nullptr && gelr != nullptr,
               "gat_agg_bwd: attn / elr from the forward and the gelr output are required");
  MVML_REQUIRE(mode != 0 || out != nullptr, "gat_agg_bwd: mode 0 needs the forward output");
  if (num_nodes == 0) return MVML_OK;
  if (!workspace || workspace_bytes == 0) {
    set_error("gat_agg_bwd: workspace of mvml_gat_agg_bwd_workspace_size(E, H) bytes required");
    return MVML_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  float* gpre = static_cast<float*>(workspace);
  const int vpl = (int)ceil_div(H * F, 256);
  switch (H) {
    case 1: { MVML_VPL_CASES(launch_bwd, 1, num_nodes, in_rowptr, in_src, out_rowptr, out_dst, out_inslot, Y, ldy, elr, attn, attn_l, attn_r, out, g_out, F, slope, mode, gpre, gY, ldgy, gelr, st) break; }
    case 2: { MVML_VPL_CASES(launch_bwd, 2, num_nodes, in_rowptr, in_src, out_rowptr, out_dst, out_inslot, Y, ldy, elr, attn, attn_l, attn_r, out, g_out, F, slope, mode, gpre, gY, ldgy, gelr, st) break; }
    case 4: { MVML_VPL_CASES(launch_bwd, 4, num_nodes, in_rowptr, in_src, out_rowptr, out_dst, out_inslot, Y, ldy, elr, attn, attn_l, attn_r, out, g_out, F, slope, mode, gpre, gY, ldgy, gelr, st) break; }
    case 8: { MVML_VPL_CASES(launch_bwd, 8, num_nodes, in_rowptr, in_src, out_rowptr, out_dst, out_inslot, Y, ldy, elr, attn, attn_l, attn_r, out, g_out, F, slope, mode, gpre, gY, ldgy, gelr, st) break; }
  }
  set_error("gat_agg_bwd: unsupported shape");
  return MVML_ERR_INVALID;
}

extern "C" size_t mvml_gat_attn_grad_workspace_size(int64_t num_nodes, int H, int F) {
  return carve_size((size_t)attn_grad_splits(num_nodes, H * F) * 2 * H * F * sizeof(float));
}

extern "C" int mvml_gat_attn_grad(int64_t num_nodes, int H, int F, const float* Y, int64_t ldy,
                                  const float* gelr, float* g_attn_l, float* g_attn_r,
                                  void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  MVML_REQUIRE(H > 0 && F > 0 && num_nodes >= 0 && ldy >= (int64_t)H * F, "gat_attn_grad: bad shape");
  if (!workspace || workspace_bytes < mvml_gat_attn_grad_workspace_size(num_nodes, H, F)) {
    set_error("gat_attn_grad: workspace too small");
    return MVML_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const int HF = H * F;
  const int S = attn_grad_splits(num_nodes, HF);
  const int64_t rows_per = ceil_div(num_nodes > 0 ? num_nodes : 1, S);
  float* part = static_cast<float*>(workspace);
  dim3 g1((unsigned)ceil_div(HF, 256), (unsigned)S);
  attn_grad_partial_kernel<<<g1, 256, 0, st>>>(num_nodes, H, F, Y, ldy, gelr, rows_per, part);
  attn_grad_final_kernel<<<(unsigned)ceil_div(2 * HF, 256), 256, 0, st>>>(HF, S, part, g_attn_l, g_attn_r);
  return check_launch("attn_grad");
}

extern "C" int mvml_gat_fold_weights(const float* fc_w, const float* res_fc_w, int H, int F, int Fin,
                                     int ldw, int mean_residual, float* Wcat, void* stream) {
  clear_error();
  MVML_REQUIRE(H > 0 && F > 0 && Fin > 0 && ldw >= Fin, "gat_fold_weights: bad shape");
  hipStream_t st = as_stream(stream);
  const int64_t total = (int64_t)mvml_gat_proj_cols(H, F, mean_residual) * ldw;
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(total, 256), 8192);
  fold_weights_kernel<<<blocks, 256, 0, st>>>(fc_w, res_fc_w, H, F, Fin, ldw, mean_residual, Wcat);
  return check_launch("fold_weights_kernel");
}

extern "C" int mvml_gat_unfold_grads(const float* gWcat, int H, int F, int Fin, int ldg,
                                     int mean_residual, float* g_fc_w, float* g_res_fc_w,
                                     void* stream) {
  clear_error();
  MVML_REQUIRE(H > 0 && F > 0 && Fin > 0 && ldg >= Fin, "gat_unfold_grads: bad shape");
  hipStream_t st = as_stream(stream);
  const int64_t total = (int64_t)H * F * Fin;
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(total, 256), 8192);
  unfold_w_kernel<<<blocks, 256, 0, st>>>(gWcat, H, F, Fin, ldg, mean_residual, g_fc_w, g_res_fc_w);
  return check_launch("unfold_w_kernel");
}
