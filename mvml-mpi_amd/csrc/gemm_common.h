// Shared pieces of the split-fp16 GEMM kernels (gemm_f32.hip, gemm_planes.hip): operand types,
// the scaled split-fp16 split, operand / per-row maxima, and the LDS epilogue of a wave's 32x32
// accumulator tiles (bias, beta, ReLU / ELU / ELU', LSTM cell, folded output maxima).
#pragma once
#include <type_traits>
#include <utility>

#include "common.h"

namespace mvml {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Scaled split-fp16 (NP = 2): an operand scaled by a power of two s (its |max| lands in
// [2^14, 2^15)) is split into x s = h + l, h = f16(x s), l = f16(x s - h): 2 x 11 significant
// bits, representation error <= 2^-22 |x s| (plus 2^-25 absolute in scaled units for values
// 2^18 below the operand's max, where l is subnormal).  The product keeps h_a h_b + h_a l_b +
// l_a h_b (dropped l_a l_b < 2^-22 relative); fp16 products are exact in fp32, so the result has
// the accuracy of an fp32 GEMM at 3 MFMAs per fragment pair instead of 6.  The epilogue
// multiplies by 1/(s_a s_b) (exact).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// l = f16(x s - h) of a pair: v_fma_mix{lo,hi}_f16 forms -h * 1 + x s from the f16 h and the
// f32 x s with one rounding (the difference is exact in f32, so this is f16(x s - f32(h))) —
// 2 VALU per pair instead of 2 converts, a packed subtract and a packed convert.
__device__ __forceinline__ uint32_t lo_pair(f16x2 h, f32x2 xs) {
  uint32_t r;
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(r)
      : "v"(h), "v"(xs.x), "v"(xs.y));
  return r;
}
__device__ __forceinline__ void split2h(const float4& v, float s, uint2& p0, uint2& p1) {
  const f32x2 u = {v.x * s, v.y * s}, w = {v.z * s, v.w * s};
  const f16x2 hu = __builtin_convertvector(u, f16x2), hw = __builtin_convertvector(w, f16x2);
  p0.x = __builtin_bit_cast(uint32_t, hu);
  p0.y = __builtin_bit_cast(uint32_t, hw);
  p1.x = lo_pair(hu, u);
  p1.y = lo_pair(hw, w);
}

// Eight values (two float4, k order) -> the two scaled fp16 planes of split2h, as MFMA operands.
__device__ __forceinline__ void split2h8(const float4& lo, const float4& hi, float s, bf16x8& h,
                                         bf16x8& l) {
  uint2 h0, l0, h1, l1;
  split2h(lo, s, h0, l0);
  split2h(hi, s, h1, l1);
  const u32x4 hv = {h0.x, h0.y, h1.x, h1.y}, lv = {l0.x, l0.y, l1.x, l1.y};
  h = __builtin_bit_cast(bf16x8, hv);
  l = __builtin_bit_cast(bf16x8, lv);
}

// Scale of an operand from its |max| bits (non-negative float bits order as integers): 2^k with
// k = 141 - biased exponent, so |max| s < 2^15 (fp16 max 65504); k clamped to [-100, 100] (zero
// / tiny operands: any scale works; a NaN max gives NaN results either way).
__device__ __forceinline__ int amax_shift(uint32_t bits) {
  const int k = 141 - (int)((bits >> 23) & 0xff);
  return k < -100 ? -100 : (k > 100 ? 100 : k);
}
__device__ __forceinline__ float pow2f(int k) { return __uint_as_float((uint32_t)(k + 127) << 23); }

// Split-fp16 operand maxima: bits of max |A| and max |B| (device pointers, may alias).
// Per-row A maxima (a_rows, M entries, K-contiguous A only): every A row gets its own scale,
// so a row's split — and with it the row of the product — depends on that row alone, not on the
// largest row of the batch: per-row fp32 accuracy however far a row sits below the operand's
// max, and results that do not change with the batch a row is computed in.
struct AmaxPtrs {
  const uint32_t* a = nullptr;
  const uint32_t* b = nullptr;
  int64_t b_plane = 0;  // BPS: elements from B's high fp16 plane to its low plane
  const uint32_t* a_rows = nullptr;
  // gemm_f32_kernel<..., RS = true> (k-major A): fp32 sums over k of every op(A) row, as
  // [2 S][M] partials (split s, wave column half h -> row 2 s + h); mvml_gemm_f16x2_amax_colsum
  float* a_rowsum = nullptr;
};

// Scale shift of A row `row` (clamped into range: clamped rows feed outputs never stored).
__device__ __forceinline__ int row_shift(const AmaxPtrs& am, int64_t row, int64_t M) {
  return amax_shift(am.a_rows[row < M ? row : M - 1]);
}


// LSTM cell in the GEMM epilogue (D > 0): the product is the gate pre-activation block of D
// units with the weight rows INTERLEAVED (column 4 j + q = gate q of unit j), so a lane's
// row-contiguous float4 is one unit's (i, f, g, o); it adds b_ih + b_hh (gate-major, as
// nn.LSTM stores them), runs lstm_cell_fwd_kernel's arithmetic in its order and writes c, h
// (twice), and the activations act[row][q D + j] (gate-major) instead of the gates.
struct CellEpi {
  const float* b_ih = nullptr;
  const float* b_hh = nullptr;
  const float* c_prev = nullptr;  // [M][D] or null (zero state)
  float* c_out = nullptr;         // [M][D]
  float* h_out = nullptr;         // row stride ldh
  float* h_out2 = nullptr;        // row stride ldh2, or null
  float* act = nullptr;           // [M][4 D]
  int64_t ldh = 0, ldh2 = 0;
  int D = 0;
  const float* gx = nullptr;  // [M][4 D] gate-major addend (a BiLSTM step's input projection), or null
  int64_t ldgx = 0;
};

__device__ __forceinline__ float sigm_epi(float x) { return 1.f / (1.f + expf(-x)); }

// Extra epilogue work of the 256x256 split-fp16 tile (mvml_gemm_f16x2_ex):
//  * act 2: ELU (dgllife GATLayer's flatten activation, x > 0 ? x : expm1(x)) after the bias;
//    act 3: the ELU backward with the layer output as aux, v *= aux > 0 ? 1 : aux + 1 (torch's
//    elu_backward on the result) — the layer-2 data gradient leaves as layer 1's g_rst;
//  * c_amax: unsigned atomicMax of max |stored value| bits (one slot per product);
//  * c_rows: per-row |max| bits of the stored values, slot (column / rows_cols) of row r at
//    c_rows[slot * rows_stride + r] (rows_cols = 0: one slot per row), atomicMax so that column
//    tiles and batch products fold into the same word (host: rows_cols % 64 == 0);
//  * strided batch: product z adds z * bias_z to bias, z * rows_z to the per-row A maxima and
//    z * crows_z to c_rows.
struct EpiX {
  const float* aux = nullptr;
  int64_t ld_aux = 0;
  uint32_t* c_amax = nullptr;
  uint32_t* c_rows = nullptr;
  int64_t rows_stride = 0;
  int rows_cols = 0;
  int64_t bias_z = 0, rows_z = 0, crows_z = 0;
};
__device__ __forceinline__ float elu_epi(float x) { return x > 0.f ? x : expm1f(x); }
__device__ __forceinline__ float elu_grad_epi(float o) { return o > 0.f ? 1.f : o + 1.f; }

constexpr int kEpiLd = 68;  // floats per LDS row (64 + 4: the column writes hit distinct banks)

// Epilogue of the 256x256 kernel through LDS: a wave's 128 x 64 accumulator block goes out in
// four 32-row passes; each pass writes the 32x32 MFMA layout (lane = column, 16 rows per lane)
// into a wave-private LDS tile and reads it back as whole-row float4s, so C (or the split-K
// slab) is stored with 16-B row-contiguous stores instead of 4-B column scatters — the
// epilogue of an output-bound GEMM (L2 forward: 13.5 GB of C) is store-issue-bound otherwise.
// Rows / columns outside C and unaligned C fall back to guarded scalar stores per element.
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// A wave's FM x 2 accumulator tiles (rows r0 .. r0 + 32 FM, 64 columns) through its 32-row LDS
// window: FM = 4 in the 256x256 kernels, 2 in the 128x128 one.
// One float4 of an output row through the EpiX epilogue (bias, beta, act 0-3), stored; returns
// max |stored value| (columns past N neither stored nor counted).
__device__ __forceinline__ float epix_store4(const float* src, float* __restrict__ out, int64_t ld,
                                            int64_t N, int64_t row, int64_t col, float ua,
                                            bool hb, const float (&bv)[4], float beta, int act,
                                            const float* __restrict__ aux, int64_t ld_aux, bool vec) {
  const float4 t = *reinterpret_cast<const float4*>(src);
  float e0 = t.x * ua, e1 = t.y * ua, e2 = t.z * ua, e3 = t.w * ua;
  float* cp = out + row * ld + col;
  const bool full = col + 3 < N;
  // act 3: the four aux values of a full, 16-B aligned piece in one load (ld_aux % 4 == 0 and
  // aux 16-B aligned: col is a multiple of 4)
  float ax[4] = {0.f, 0.f, 0.f, 0.f};
  if (act == 3) {
    const float* ap = aux + row * ld_aux + col;
    if (full && vec && (ld_aux & 3) == 0 && ((uintptr_t)aux & 15) == 0) {
      const float4 a4 = *reinterpret_cast<const float4*>(ap);
      ax[0] = a4.x; ax[1] = a4.y; ax[2] = a4.z; ax[3] = a4.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) ax[u] = col + u < N ? ap[u] : 0.f;
    }
  }
  auto fin = [&](float x, int u) __attribute__((always_inline)) -> float {
    if (hb) x += bv[u];
    if (beta != 0.f) x += beta * cp[u];
    if (act == 1) x = fmaxf(x, 0.f);
    if (act == 2) x = elu_epi(x);
    if (act == 3) x *= elu_grad_epi(ax[u]);
    return x;
  };
  e0 = fin(e0, 0);
  if (full || col + 1 < N) e1 = fin(e1, 1);
  if (full || col + 2 < N) e2 = fin(e2, 2);
  if (full) e3 = fin(e3, 3);
  float m = fabsf(e0);
  if (full && vec) {
    *reinterpret_cast<float4*>(cp) = make_float4(e0, e1, e2, e3);
    m = fmaxf(fmaxf(m, fabsf(e1)), fmaxf(fabsf(e2), fabsf(e3)));
  } else {
    cp[0] = e0;
    if (col + 1 < N) { cp[1] = e1; m = fmaxf(m, fabsf(e1)); }
    if (col + 2 < N) { cp[2] = e2; m = fmaxf(m, fabsf(e2)); }
    if (col + 3 < N) { cp[3] = e3; m = fmaxf(m, fabsf(e3)); }
  }
  return m;
}

// The EpiX tile pass: the accumulators of each 32-row block through the wave's LDS rows (as
// epilogue_lds), then stores through epix_store4, per-row maxima (a row's 16 lanes reduce, one
// atomicMax per row slot) and the tile's |max| (one atomicMax per wave).  The row blocks are
// unrolled by construction (a fold over the block index) so the accumulators stay in registers;
// the store loop inside is not unrolled.  The bias of the lane's four columns (the same for every
// row it stores) is loaded once.  s_rm (LDS, the wave's rows of the tile): the per-row maxima
// are folded there (LDS atomics) and the kernel commits one global atomicMax per row and
// workgroup after the epilogue, instead of one per row and wave.
template <int... Is, typename Fn>
__device__ __forceinline__ void static_for_x(std::integer_sequence<int, Is...>, Fn&& fn) {
  (fn(std::integral_constant<int, Is>{}), ...);
}
template <int FM>
__device__ __forceinline__ void epix_tile(const f32x16 (&acc)[FM][2], float* wl, int64_t M, int64_t N,
                                          int64_t r0, int64_t c0, int lane,
                                          const float* __restrict__ bias, float beta, int act,
                                          float* __restrict__ out, int64_t ld, bool vec, const int* rs,
                                          const EpiX& ex, uint32_t* s_rm) {
  const int li = lane & 31, lk = lane >> 5;
  float am = 0.f;
  float bv[4];
  {
    const int64_t cb = c0 + (lane & 15) * 4;
#pragma unroll
    for (int u = 0; u < 4; ++u) bv[u] = (bias && cb + u < N) ? bias[cb + u] : 0.f;
  }
  static_for_x(std::make_integer_sequence<int, FM>{}, [&](auto I) __attribute__((always_inline)) {
    constexpr int i = decltype(I)::value;
    if (i > 0) wave_sync_lds();
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        wl[((r & 3) + 8 * (r >> 2) + 4 * lk) * kEpiLd + 32 * j + li] = acc[i][j][r];
    wave_sync_lds();
#pragma nounroll
    for (int q = 0; q < 8; ++q) {
      const int idx = q * 64 + lane, rr = idx >> 4, c4 = (idx & 15) * 4;
      const int64_t row = r0 + 32 * i + rr, col = c0 + c4;
      float rm = 0.f;
      if (row < M && col < N)
        rm = epix_store4(wl + rr * kEpiLd + c4, out, ld, N, row, col, rs ? pow2f(-rs[32 * i + rr]) : 1.f,
                         bias != nullptr, bv, beta, act, ex.aux, ex.ld_aux, vec);
      am = fmaxf(am, rm);
      if (ex.c_rows) {  // (uniform) the row's 16 lanes reduce together
#pragma unroll
        for (int o = 8; o >= 1; o >>= 1) rm = fmaxf(rm, __shfl_xor(rm, o, 64));
        if ((lane & 15) == 0 && row < M) {
          if (s_rm) {
            atomicMax(s_rm + 32 * i + rr, __float_as_uint(rm));
          } else {
            const int64_t slot = ex.rows_cols > 0 ? c0 / ex.rows_cols : 0;
            atomicMax(ex.c_rows + blockIdx.z * ex.crows_z + slot * ex.rows_stride + row, __float_as_uint(rm));
          }
        }
      }
    }
  });
  if (ex.c_amax) {  // (uniform) one atomic per wave
    am = wave_max(am);
    if (lane == 0) atomicMax(ex.c_amax, __float_as_uint(am));
  }
}

template <int FM, bool EX = false>
__device__ __forceinline__ void epilogue_lds(const f32x16 (&acc)[FM][2], float* wl, int64_t M,
                                                 int64_t N, int64_t r0, int64_t c0, int lane,
                                                 const float* __restrict__ bias, float beta, int act,
                                                 float* __restrict__ C, int64_t ldc,
                                                 float* __restrict__ slab, const CellEpi& cep = CellEpi{},
                                                 const int* rs = nullptr, const EpiX& ex = EpiX{},
                                                 uint32_t* s_rm = nullptr) {
  // rs (per-row A maxima): rs[32 i + rr] = the scale shift of row r0 + 32 i + rr, undone here as
  // each row leaves (acc already carries B's)
  const int li = lane & 31, lk = lane >> 5;
  float* out = slab ? slab + (int64_t)blockIdx.y * M * N : C;
  const int64_t ld = slab ? N : ldc;
  const bool vec = (ld % 4 == 0) && (((uintptr_t)out & 15) == 0);
  // LSTM cell, four units per lane (16 columns of a row): every load and store of the cell is a
  // float4 (c, h, h2, the four activation rows, the biases, c_prev, the input projection)
  // instead of seven dword stores per unit — the cell epilogue was store-issue-bound.  Same
  // arithmetic per unit, so bitwise the per-unit path's results (kept for unaligned operands).
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  // EpiX work (act 2 / 3, folded maxima): its own tile pass, never with split-K or the cell
  if constexpr (EX) {
    if (!slab && cep.D == 0 && (act >= 2 || ex.c_amax || ex.c_rows)) {
      epix_tile<FM>(acc, wl, M, N, r0, c0, lane, bias, beta, act, out, ld, vec, rs, ex, s_rm);
      return;
    }
  }
  const bool cell4 = cep.D > 0 && cep.D % 4 == 0 && al16(cep.b_ih) && al16(cep.b_hh) &&
                     al16(cep.c_prev) && al16(cep.c_out) && al16(cep.h_out) && al16(cep.h_out2) &&
                     al16(cep.act) && cep.ldh % 4 == 0 && cep.ldh2 % 4 == 0 && al16(cep.gx) &&
                     cep.ldgx % 4 == 0;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    if (i > 0) wave_sync_lds();  // the previous pass's reads are done
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        wl[((r & 3) + 8 * (r >> 2) + 4 * lk) * kEpiLd + 32 * j + li] = acc[i][j][r];
    wave_sync_lds();
    if (cell4) {  // (host: N = 4 D, no split-K; N % 16 == 0, so a 4-unit group never straddles N)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int idx = q * 64 + lane, rr = idx >> 2, u = idx & 3;
        const int64_t row = r0 + 32 * i + rr, col = c0 + 16 * u;
        if (row >= M || col >= N) continue;
        const int D = cep.D;
        const int64_t j = col >> 2;  // units j .. j + 3
        float4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = *reinterpret_cast<const float4*>(wl + rr * kEpiLd + 16 * u + 4 * k);
        if (rs) {
          const float ua = pow2f(-rs[32 * i + rr]);
#pragma unroll
          for (int k = 0; k < 4; ++k) { v[k].x *= ua; v[k].y *= ua; v[k].z *= ua; v[k].w *= ua; }
        }
        auto ld4 = [](const float* p) { return *reinterpret_cast<const float4*>(p); };
        auto el = [](const float4& f, int k) { return k == 0 ? f.x : k == 1 ? f.y : k == 2 ? f.z : f.w; };
        if (cep.gx) {
          const float* gxr = cep.gx + row * cep.ldgx + j;
          const float4 xi = ld4(gxr), xf = ld4(gxr + D), xg = ld4(gxr + 2 * D), xo = ld4(gxr + 3 * D);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            v[k].x += el(xi, k); v[k].y += el(xf, k); v[k].z += el(xg, k); v[k].w += el(xo, k);
          }
        }
        const float4 bii = ld4(cep.b_ih + j), bif = ld4(cep.b_ih + D + j), big = ld4(cep.b_ih + 2 * D + j),
                     bio = ld4(cep.b_ih + 3 * D + j);
        const float4 bhi = ld4(cep.b_hh + j), bhf = ld4(cep.b_hh + D + j), bhg = ld4(cep.b_hh + 2 * D + j),
                     bho = ld4(cep.b_hh + 3 * D + j);
        const float4 cp4 = cep.c_prev ? ld4(cep.c_prev + row * D + j) : make_float4(0.f, 0.f, 0.f, 0.f);
        float cv[4], hv[4], iv[4], fv[4], gv[4], ov[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float gi = v[k].x + el(bii, k) + el(bhi, k);
          const float gf = v[k].y + el(bif, k) + el(bhf, k);
          const float gg = v[k].z + el(big, k) + el(bhg, k);
          const float go = v[k].w + el(bio, k) + el(bho, k);
          iv[k] = sigm_epi(gi); fv[k] = sigm_epi(gf); gv[k] = tanhf(gg); ov[k] = sigm_epi(go);
          cv[k] = __fmaf_rn(fv[k], el(cp4, k), __fmul_rn(iv[k], gv[k]));  // lstm_cell_fwd_kernel's rounding
          hv[k] = __fmul_rn(ov[k], tanhf(cv[k]));
        }
        auto st4 = [](float* p, const float (&a)[4]) { *reinterpret_cast<float4*>(p) = make_float4(a[0], a[1], a[2], a[3]); };
        st4(cep.c_out + row * D + j, cv);
        st4(cep.h_out + row * cep.ldh + j, hv);
        if (cep.h_out2) st4(cep.h_out2 + row * cep.ldh2 + j, hv);
        float* a = cep.act + row * 4 * (int64_t)D + j;
        st4(a, iv);
        st4(a + D, fv);
        st4(a + 2 * D, gv);
        st4(a + 3 * D, ov);
      }
      continue;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int idx = q * 64 + lane, rr = idx >> 4, c4 = (idx & 15) * 4;
      const int64_t row = r0 + 32 * i + rr, col = c0 + c4;
      if (row >= M || col >= N) continue;
      float4 v = *reinterpret_cast<const float4*>(wl + rr * kEpiLd + c4);
      if (rs) {
        const float ua = pow2f(-rs[32 * i + rr]);
        v.x *= ua; v.y *= ua; v.z *= ua; v.w *= ua;
      }
      if (cep.D > 0) {  // LSTM cell (host: N = 4 D, no split-K): one unit's four gates
        const int D = cep.D;
        const int64_t j = col >> 2;
        if (cep.gx) {  // (h W^T + x W_ih^T) first, as the GEMM's beta = 1 onto the projection
          const float* gxr = cep.gx + row * cep.ldgx + j;
          v.x += gxr[0]; v.y += gxr[D]; v.z += gxr[2 * D]; v.w += gxr[3 * D];
        }
        const float gi = v.x + cep.b_ih[j] + cep.b_hh[j];
        const float gf = v.y + cep.b_ih[D + j] + cep.b_hh[D + j];
        const float gg = v.z + cep.b_ih[2 * D + j] + cep.b_hh[2 * D + j];
        const float go = v.w + cep.b_ih[3 * D + j] + cep.b_hh[3 * D + j];
        const float ig = sigm_epi(gi), fg = sigm_epi(gf), gt = tanhf(gg), og = sigm_epi(go);
        const float cpv = cep.c_prev ? cep.c_prev[row * D + j] : 0.f;
        const float c = __fmaf_rn(fg, cpv, __fmul_rn(ig, gt));  // lstm_cell_fwd_kernel's rounding
        const float h = __fmul_rn(og, tanhf(c));
        cep.c_out[row * D + j] = c;
        cep.h_out[row * cep.ldh + j] = h;
        if (cep.h_out2) cep.h_out2[row * cep.ldh2 + j] = h;
        float* a = cep.act + row * 4 * (int64_t)D + j;
        a[0] = ig;
        a[D] = fg;
        a[2 * D] = gt;
        a[3 * D] = og;
        continue;
      }
      float* cp = out + row * ld + col;
      if (vec && col + 3 < N) {
        if (!slab) {
          if (bias) {
            const float4 b = *reinterpret_cast<const float4*>(bias + col);
            v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
          }
          if (beta != 0.f) {
            const float4 o = *reinterpret_cast<const float4*>(cp);
            v.x += beta * o.x; v.y += beta * o.y; v.z += beta * o.z; v.w += beta * o.w;
          }
          if (act == 1) {
            v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
          }
        }
        *reinterpret_cast<float4*>(cp) = v;
      } else {
        const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (col + u >= N) break;
          float x = e[u];
          if (!slab) {
            if (bias) x += bias[col + u];
            if (beta != 0.f) x += beta * cp[u];
            if (act == 1) x = fmaxf(x, 0.f);
          }
          cp[u] = x;
        }
      }
    }
  }
}

typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

}  // namespace
}  // namespace mvml
