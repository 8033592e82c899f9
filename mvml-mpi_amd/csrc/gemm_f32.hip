// Dense fp32 GEMM on CDNA4 matrix cores (v_mfma_f32_32x32x2_f32) + column sums.
//
// Used for every dense product of the view: GATConv fc/res_fc (+ the folded el/er columns),
// their backward (dX = dY * W, dW = dY^T * X), the Set2Set LSTM gate GEMMs and
// GNNModule.fc (model.py:86-87).  f32-input MFMA is exact f32 (a k-ordered fmaf chain), so
// results match a CPU fp32 GEMM to rounding.
//
// Tiling: 128x128 output tile per 256-thread workgroup (4 waves as 2x2, 64x64 per wave =
// 2x2 MFMA 32x32 tiles), K staged 32 deep through a 2-stage LDS ring filled by LDS-DMA
// (global_load_lds_dwordx4) one stage ahead, one raw s_barrier per stage, two workgroups/CU.
// The K order inside a 32-deep stage is permuted so that one ds_read_b128 yields a lane's
// operand for four consecutive MFMA steps: step s of k-group g pairs k = 8g+s (lanes 0-31) with
// k = 8g+4+s (lanes 32-63) for BOTH operands, so the sum is unchanged.
// Small-output / long-K products (the weight gradients, K = atoms in the batch) split K over
// workgroups into fp32 slabs that a second kernel sums in fixed order — deterministic, no
// float atomics.
//
// Split-bf16 variant (X3): the same tiles and LDS pipeline, but every fp32 operand fragment is
// split in registers into three bf16 terms, x = x0 + x1 + x2 (x0 = bf16(x), x1 = bf16(x - x0),
// x2 = bf16(x - x0 - x1): 3 x 8 significant bits = fp32's 24, exact for normal values), and
// the product is the six bf16 MFMAs (v_mfma_f32_32x32x16_bf16, fp32 accumulate)
//   a0b0 + a0b1 + a1b0 + a0b2 + a1b1 + a2b0,
// dropping only a1b2 + a2b1 + a2b2 (< 2^-25 relative per product).  Products of bf16 are exact
// in fp32, so the result carries fp32 GEMM accuracy (tests/test_gpu_parity.py compares both
// variants against fp64) at 6 bf16 MFMAs per 16 k instead of 8 f32 MFMAs at 1/16 the rate.
#include <cstdlib>
#include <type_traits>
#include <utility>
#include <vector>

#include "common.h"
#include "gemm_common.h"

namespace mvml {
namespace {


// Two fp32 -> packed bf16 pair (v_cvt_pk_bf16_f32, round-to-nearest-even) and the two exact
// fp32 residuals x - bf16(x), unpacked with one shift / one mask: 5 VALU per pair.
__device__ __forceinline__ uint32_t split_pair(float& a, float& b) {
  const f32x2 v = {a, b};
  const uint32_t p = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
  a -= __builtin_bit_cast(float, p << 16);
  b -= __builtin_bit_cast(float, p & 0xffff0000u);
  return p;
}

// fp32 x 8 -> three bf16 x 8 terms (round-to-nearest each; the residuals are exact in fp32):
// 11 VALU per pair of values.
__device__ __forceinline__ void split3(const float4& lo, const float4& hi, bf16x8& p0, bf16x8& p1,
                                       bf16x8& p2) {
  float x[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  u32x4 q0, q1, q2;
#pragma unroll
  for (int i = 0; i < 4; ++i) q0[i] = split_pair(x[2 * i], x[2 * i + 1]);
#pragma unroll
  for (int i = 0; i < 4; ++i) q1[i] = split_pair(x[2 * i], x[2 * i + 1]);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x2 v = {x[2 * i], x[2 * i + 1]};
    q2[i] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
  }
  p0 = __builtin_bit_cast(bf16x8, q0);
  p1 = __builtin_bit_cast(bf16x8, q1);
  p2 = __builtin_bit_cast(bf16x8, q2);
}

// acc += (a0 + a1 + a2)(b0 + b1 + b2) to fp32 accuracy: the six significant cross terms.
__device__ __forceinline__ f32x16 mfma_x3(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}


// NP = 3: the split-bf16 product above; NP = 2: scaled split-fp16; NP = 1: one bf16 MFMA (bf16
// operands, fp32 accumulate).
template <int NP>
__device__ __forceinline__ f32x16 mfma_np(const bf16x8 (&a)[NP], const bf16x8 (&b)[NP], f32x16 acc) {
  if constexpr (NP == 3) {
    return mfma_x3(a, b, acc);
  } else if constexpr (NP == 2) {
    const f16x8 a0 = __builtin_bit_cast(f16x8, a[0]), a1 = __builtin_bit_cast(f16x8, a[1]);
    const f16x8 b0 = __builtin_bit_cast(f16x8, b[0]), b1 = __builtin_bit_cast(f16x8, b[1]);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, acc, 0, 0, 0);
  } else {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  }
}

constexpr int BM = 128, BN = 128, BKT = 32, kThreads = 256;
constexpr int kTileFloats = 128 * BKT;  // one operand tile in LDS (16 KB)

// ---- operand staging ---------------------------------------------------------------------
// An operand tile is 128 rows (M for A, N for B) x 32 k.
//  * K-contiguous operands (A stored [M][K], B stored [N][K]) live in LDS as [row][32 k] with
//    the 16-B chunk index XOR-swizzled by (row >> 1) & 7, so that the ds_read_b128 fragment
//    reads below are bank-conflict free.
//  * K-major operands (stored [K][rows]) live in LDS as [k][128], read by ds_read_b32.
// Each wave-instruction fills 1 KB (64 lanes x 16 B) of LDS; a 16 KB tile is 16 instructions,
// 4 per wave.  The same lane -> (row, chunk) map serves the LDS-DMA path (global_load_lds, the
// per-lane SOURCE carries the swizzle) and the guarded register path (tails / unaligned).
template <bool KMAJ>
struct Stager {
  __device__ static __forceinline__ int swz(int row) { return (row >> 1) & 7; }

  // Global element offset (row, k) of this lane's 16-B piece for wave-instruction `inst`,
  // and the LDS float offset it lands at.
  __device__ static __forceinline__ void piece(int inst, int lane, int& row, int& kk) {
    if (!KMAJ) {
      row = inst * 8 + (lane >> 3);
      kk = 4 * ((lane & 7) ^ swz(row));
    } else {
      kk = inst * 2 + (lane >> 5);
      row = 4 * (lane & 31);
    }
  }

  __device__ static __forceinline__ void issue_lds_dma(const float* __restrict__ P, int64_t ld,
                                                       int64_t r0, int64_t rows, int64_t k0,
                                                       float* lds_tile, int wid, int lane) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int inst = wid * 4 + it;
      int row, kk;
      piece(inst, lane, row, kk);
      const float* src;
      if (!KMAJ) {
        const int64_t gr = min(r0 + row, rows - 1);  // rows past the edge are never stored
        src = P + gr * ld + k0 + kk;
      } else {  // rows % 4 == 0 here: a piece past the edge re-reads the last in-range piece
        src = P + (k0 + kk) * ld + min(r0 + row, rows - 4);
      }
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(lds_tile + inst * 256),
                                       16, 0, 0);
    }
  }

  // Guarded register path: zero-fills k >= kend and rows >= rows; same LDS image.  Split into
  // a load (issued before the MFMAs) and a store (after them) so the latency overlaps compute.
  __device__ static __forceinline__ void load_guarded(const float* __restrict__ P, int64_t ld,
                                                      int64_t r0, int64_t rows, int64_t k0,
                                                      int64_t kend, bool vec, int wid, int lane,
                                                      float4 (&v)[4]) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int inst = wid * 4 + it;
      int row, kk;
      piece(inst, lane, row, kk);
      float e[4] = {0.f, 0.f, 0.f, 0.f};
      if (!KMAJ) {
        const int64_t gr = r0 + row, gk = k0 + kk;
        if (gr < rows) {
          const float* p = P + gr * ld + gk;
          if (vec && gk + 3 < kend) {
            const float4 t = *reinterpret_cast<const float4*>(p);
            e[0] = t.x; e[1] = t.y; e[2] = t.z; e[3] = t.w;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (gk + j < kend) e[j] = p[j];
          }
        }
      } else {
        const int64_t gk = k0 + kk, gr = r0 + row;
        if (gk < kend) {
          const float* p = P + gk * ld + gr;
          if (vec && gr + 3 < rows) {
            const float4 t = *reinterpret_cast<const float4*>(p);
            e[0] = t.x; e[1] = t.y; e[2] = t.z; e[3] = t.w;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (gr + j < rows) e[j] = p[j];
          }
        }
      }
      v[it] = make_float4(e[0], e[1], e[2], e[3]);
    }
  }

  __device__ static __forceinline__ void store_guarded(float* lds_tile, int wid, int lane,
                                                       const float4 (&v)[4]) {
#pragma unroll
    for (int it = 0; it < 4; ++it)
      *reinterpret_cast<float4*>(lds_tile + (wid * 4 + it) * 256 + lane * 4) = v[it];
  }

  // Inline-asm fragment read (the compiler does not see it, so it cannot insert a vmcnt(0)
  // that would drain the LDS-DMA prefetch in flight).  The caller waits lgkmcnt and places a
  // sched_barrier before using the result.  tile_b = LDS byte address of the operand tile.
  template <int G>
  __device__ static __forceinline__ void frag_asm(uint32_t tile_b, int row, int h, float4& out) {
    if (!KMAJ) {
      const uint32_t addr = tile_b + row * (BKT * 4) + 16 * ((2 * G + h) ^ swz(row));
      asm volatile("ds_read_b128 %0, %1" : "=v"(out) : "v"(addr) : "memory");
    } else {
      const uint32_t addr = tile_b + ((8 * G + 4 * h) * 128 + row) * 4;
      asm volatile(
          "ds_read_b32 %0, %4\n\t"
          "ds_read_b32 %1, %4 offset:512\n\t"
          "ds_read_b32 %2, %4 offset:1024\n\t"
          "ds_read_b32 %3, %4 offset:1536"
          : "=&v"(out.x), "=&v"(out.y), "=&v"(out.z), "=&v"(out.w)
          : "v"(addr)
          : "memory");
    }
  }

  // Split-bf16 operand fragment of one 32x32x16 MFMA: the lane's 8 consecutive k values
  // k = 8g .. 8g+7 of k-group g (g = 2 t + (lane >> 5) for 16-k step t), as two float4.
  // Inline asm for the same reason as frag_asm; the caller waits lgkmcnt.
  __device__ static __forceinline__ void frag8_asm(uint32_t tile_b, int row, int g, float4& lo,
                                                   float4& hi) {
    if (!KMAJ) {
      const uint32_t base = tile_b + row * (BKT * 4);
      const uint32_t a0 = base + 16 * ((2 * g) ^ swz(row)), a1 = base + 16 * ((2 * g + 1) ^ swz(row));
      asm volatile("ds_read_b128 %0, %1" : "=v"(lo) : "v"(a0) : "memory");
      asm volatile("ds_read_b128 %0, %1" : "=v"(hi) : "v"(a1) : "memory");
    } else {
      const uint32_t addr = tile_b + ((8 * g) * 128 + row) * 4;
      asm volatile(
          "ds_read_b32 %0, %8\n\t"
          "ds_read_b32 %1, %8 offset:512\n\t"
          "ds_read_b32 %2, %8 offset:1024\n\t"
          "ds_read_b32 %3, %8 offset:1536\n\t"
          "ds_read_b32 %4, %8 offset:2048\n\t"
          "ds_read_b32 %5, %8 offset:2560\n\t"
          "ds_read_b32 %6, %8 offset:3072\n\t"
          "ds_read_b32 %7, %8 offset:3584"
          : "=&v"(lo.x), "=&v"(lo.y), "=&v"(lo.z), "=&v"(lo.w), "=&v"(hi.x), "=&v"(hi.y),
            "=&v"(hi.z), "=&v"(hi.w)
          : "v"(addr)
          : "memory");
    }
  }

  // Fragment of k-group g (8 k values): element s of the result is the operand value at
  // row `row`, k = 8g + 4h + s, where h = lane >> 5 — the k order both operands share.
  __device__ static __forceinline__ float4 frag(const float* lds_tile, int row, int g, int h) {
    if (!KMAJ) {
      const int slot = (2 * g + h) ^ swz(row);
      return *reinterpret_cast<const float4*>(lds_tile + row * BKT + slot * 4);
    } else {
      const float* p = lds_tile + (8 * g + 4 * h) * 128 + row;
      return make_float4(p[0], p[128], p[256], p[384]);
    }
  }
};

__device__ __forceinline__ float comp(const float4& v, int s) {
  return s == 0 ? v.x : (s == 1 ? v.y : (s == 2 ? v.z : v.w));
}

// Optional GAT-projection epilogue (EPI_LOGW >= 0, W = 1 << EPI_LOGW columns per partial):
// for every W-column group g of the first ep_cols output columns (Z = X fc^T), the per-row
// partial logits
//   part[g][0][row] = sum_{c in g} C[row][c] * attn_l[c],  part[g][1][row] = ... attn_r[c]
// (attn_l / attn_r = ep_vec[0 : ep_cols] / ep_vec[ep_cols : 2 ep_cols]; W divides F so a group
// never straddles two heads), so GATConv's el = (feat * attn_l).sum(-1) needs no second pass
// over Z: mvml_gat_proj_fwd sums a head's groups in fixed order.  In a 32x32 accumulator tile
// the lane holds a column and 16 rows: a halving butterfly over the W lanes of a group
// (values 32 -> 32/W, masks W/2 .. 1) leaves lane li with the values of index
// ((li & (W-1)) << (5 - EPI_LOGW)) | t, index = side * 16 + row register.
// Strided batch (blockIdx.z): product z reads A + z a, B + z b and writes C + z c (floats).

struct BatchStrides {
  int64_t a = 0, b = 0, c = 0;
};

// A second, independent product in the same launch (blockIdx.z == 1): its own A, B, row count,
// split-K slab, B maximum and LSTM-cell epilogue pointers; K, the leading dimensions and the
// column count are shared.  Both directions of a BiLSTM step run as one launch this way.
struct DualPtrs {
  const float* a = nullptr;
  const float* b = nullptr;
  float* slab = nullptr;
  const uint32_t* amax_b = nullptr;
  int64_t m = 0;
  CellEpi cep;
  const uint32_t* amax_a = nullptr;  // null: the first product's A maximum
};

struct ProjEpi {
  const float* vec;  // [2][cols]
  int cols;          // H*F
  float* part;       // [cols / W][2][M]: a wave's stores for one (group, side) are 32 rows, contiguous
};


// Epilogue of a wave's FM x FN 32x32 accumulators (rows r0 + 32 i .., columns c0 + 32 j ..):
// optional GAT logit partials, then bias / beta*C / ReLU, or the raw split-K slab.
template <int EPI_LOGW, int FM = 2, int FN = 2, bool STORE_C = true>
__device__ __forceinline__ void tile_epilogue(const f32x16 (&acc)[FM][FN], int64_t M, int64_t N,
                                              int64_t r0, int64_t c0, int lane,
                                              const float* __restrict__ bias, float beta, int act,
                                              float* __restrict__ C, int64_t ldc,
                                              float* __restrict__ slab, const ProjEpi& epi,
                                              int64_t split = -1) {
  const int li = lane & 31, lk = lane >> 5;
  if (split < 0) split = blockIdx.y;  // the split-K slab's block: the grid's y unless remapped
  // Epilogue. C/D map of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
  if constexpr (EPI_LOGW >= 0) {
    constexpr int W = 1 << EPI_LOGW, NV = 32 >> EPI_LOGW;
  #pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int64_t cb0 = c0 + j * 32;  // first column of this 32-column block
        if (cb0 >= epi.cols) continue;             // wave-uniform
        const int64_t c = cb0 + li;
        const float al = c < epi.cols ? epi.vec[c] : 0.f;
        const float ar = c < epi.cols ? epi.vec[epi.cols + c] : 0.f;
        float v[32];  // [side][row register]
#pragma unroll
        for (int r = 0; r < 16; ++r) { v[r] = acc[i][j][r] * al; v[16 + r] = acc[i][j][r] * ar; }
#pragma unroll
        for (int st = 0; st < EPI_LOGW; ++st) {
          const int half = 16 >> st, mask = (W / 2) >> st;
          const bool hi = (lane & mask) != 0;
#pragma unroll
          for (int t = 0; t < half; ++t) {
            // the empty asm pins both values in registers first: otherwise the selects fold
            // into a dynamically indexed v[], lowered as a 32-way compare chain
            float lo = v[t], up = v[t + half];
            asm volatile("" : "+v"(lo), "+v"(up));
            const float keep = hi ? up : lo;
            const float send = hi ? lo : up;
            v[t] = keep + __shfl_xor(send, mask, 64);
          }
        }
        const int64_t gc = cb0 + (li & ~(W - 1));  // first column of the lane's group
        if (gc < epi.cols) {
#pragma unroll
          for (int t = 0; t < NV; ++t) {
            const int idx = ((li & (W - 1)) << (5 - EPI_LOGW)) | t;
            const int side = idx >> 4, r = idx & 15;
            const int64_t row = r0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
            if (row < M) epi.part[((gc / W) * 2 + side) * M + row] = v[t];
          }
        }
      }
  }
  if constexpr (!STORE_C) return;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int64_t col = c0 + j * 32 + li;
      if (col >= N) continue;
      const float bcol = (bias && !slab) ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = r0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row >= M) continue;
        float v = acc[i][j][r];
        if (slab) {
          slab[(split * M + row) * N + col] = v;
        } else {
          v += bcol;
          float* cp = C + row * ldc + col;
          if (beta != 0.f) v += beta * (*cp);
          if (act == 1) v = fmaxf(v, 0.f);
          *cp = v;
        }
      }
    }
}


// Undo the split-fp16 operand scales of a 128x128 tile's 2 x 2 accumulators (exact: powers of
// two).  Per-row A maxima: lane li scaled A rows 32 i + li of its wave's 64 (shift ka0 / ka1);
// accumulator register r of block i holds row 32 i + (r & 3) + 8 (r >> 2) + 4 (lane >> 5), whose
// shift comes from the lane that staged it.
__device__ __forceinline__ void unscale_rows(f32x16 (&acc)[2][2], bool per_row, int ka, int ka0,
                                             int ka1, int kb, int lane) {
  const float ub = pow2f(-kb);
  if (!per_row) {
    const float ua = pow2f(-ka);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = acc[i][j][r] * ua * ub;
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int src = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const float ua = pow2f(-__shfl(i ? ka1 : ka0, src, 64));
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j][r] = acc[i][j][r] * ua * ub;
    }
}

// X3: fp32-accurate products from split fp32 fragments — H2 = false: split-bf16 (six MFMAs per
// fragment pair); H2 = true: scaled split-fp16 (three; operand scales from amax, as the 256x256
// kernel's NP = 2), the skinny products' plan when the algorithm is f16x2.
// BPS (H2, K-contiguous B only): B is the interleaved pre-split of the operand
// (split_f16x2_il_kernel), so the B fragments need no split.
__device__ __forceinline__ float hsum8(const float4& a, const float4& b) {
  return ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w));
}

// RS (split-fp16, k-major A): the fp32 A fragments the waves read anyway are also summed over k
// per A row (a weight gradient's A = gY^T: the bias gradient's column sums of gY come out of
// the product's own reads).  Waves of column half wn sum 16-k step wn of every 32-k stage, the
// two k halves of a row (lanes l, l + 32) are added once at the end, and every workgroup of the
// first N tile writes its rows' partials to amax.a_rowsum[2 split + wn][row].
template <bool AK, bool BKM, int EPI_LOGW = -1, bool X3 = false, bool H2 = false, bool BPS = false,
          bool RS = false>
__global__ void __launch_bounds__(kThreads, 2)
gemm_f32_kernel(int64_t M, int64_t N, int64_t K, const float* __restrict__ A, int64_t lda,
                const float* __restrict__ B, int64_t ldb, const float* __restrict__ bias,
                float beta, int act, float* __restrict__ C, int64_t ldc, int64_t k_split,
                float* __restrict__ slab, int a_vec, int b_vec, ProjEpi epi = ProjEpi{},
                BatchStrides bst = BatchStrides{}, AmaxPtrs amax = AmaxPtrs{},
                CellEpi cep = CellEpi{}, DualPtrs dual = DualPtrs{}) {
  static_assert(!H2 || X3, "split-fp16 is a split product");
  static_assert(!BPS || (H2 && !BKM), "pre-split B: split-fp16, K-contiguous B");
  static_assert(!RS || (H2 && AK), "row sums: split-fp16, k-major A");
  if (blockIdx.z) {  // strided batch
    A += blockIdx.z * bst.a;
    B += blockIdx.z * bst.b;
    C += blockIdx.z * bst.c;
  }
  if (blockIdx.z == 1 && dual.a) {  // the second product of a dual launch (gemm_x3w_kernel's)
    A = dual.a;
    B = dual.b;
    M = dual.m;
    slab = dual.slab;
    cep = dual.cep;
    amax.b = dual.amax_b;
    if (dual.amax_a) amax.a = dual.amax_a;
    amax.a_rows = nullptr;  // (host: dual launches use operand-wide maxima)
  }
  using SA = Stager<AK>;
  using SB = Stager<BKM>;
  // [stage][A tile | B tile], one __shared__ object (a second one can de-pipeline glds waits).
  __shared__ __attribute__((aligned(16))) float lds[2 * 2 * kTileFloats];

  // XCD-aware tile order: each XCD walks a contiguous range of tiles, N fastest, so the
  // workgroups sharing an A row-panel share one L2.  Split-K grids (no batch): the (split,
  // tile) pairs in split-major order, each XCD a contiguous range of them (xcd_block over the
  // dispatch order, XCD = L % 8), so the tiles of one K split run on one XCD back to back and
  // the K chunk of the operand they all read (the skinny weight gradients' B, e.g. the layer-1
  // atom features under every 128-row tile of the 1544 gradient rows) is fetched from HBM once
  // into that XCD's L2 instead of once per XCD (a split straddling two XCDs: twice).
  const int64_t tiles_n = ceil_div(N, BN);
  int64_t tile, split;
  if (gridDim.y > 1 && gridDim.z == 1) {
    const unsigned L = blockIdx.x + blockIdx.y * gridDim.x;
    const int64_t pair = xcd_block(L, gridDim.x * gridDim.y);
    split = pair / gridDim.x;
    tile = pair % gridDim.x;
  } else {
    tile = xcd_block(blockIdx.x, gridDim.x);
    split = blockIdx.y;
  }
  const int64_t m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  if (m0 >= M) return;  // a dual launch's shorter product (grid sized for the longer one)
  const int64_t kbeg = split * k_split;
  const int64_t kend = min(K, kbeg + k_split);

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int li = lane & 31, lk = lane >> 5;
  const bool rs_on = RS && amax.a_rowsum && gridDim.z == 1 && (tile % tiles_n) == 0;
  float rs0 = 0.f, rs1 = 0.f;  // RS: this lane's k-half sums of A rows ra0 / ra1

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  int ka = 0, kb = 0;  // H2: operand scales 2^ka, 2^kb from the |max| bits
  int ka0 = 0, ka1 = 0;  // H2 with per-row A maxima: the scales of this lane's two A rows
  if constexpr (H2) {
    kb = amax_shift(*amax.b);
    if (amax.a_rows) {
      ka0 = row_shift(amax, m0 + wm * 64 + li, M);
      ka1 = row_shift(amax, m0 + wm * 64 + li + 32, M);
    } else {
      ka = ka0 = ka1 = amax_shift(*amax.a);
    }
  }
  const float s_a0 = pow2f(ka0), s_a1 = pow2f(ka1), s_b = pow2f(kb);

  // LDS-DMA needs 16-B aligned pieces; a k-major operand's edge tile also needs rows % 4 == 0
  // (no piece straddles the edge), otherwise the guarded register path fills the stage.
  const bool dma = a_vec && b_vec && (!AK || M % 4 == 0 || m0 + BM <= M) &&
                   (!BKM || N % 4 == 0 || n0 + BN <= N);
  const int64_t nfull = (kend > kbeg) ? (kend - kbeg) / BKT : 0;       // whole 32-deep tiles
  const int64_t ntiles = (kend > kbeg) ? ceil_div(kend - kbeg, BKT) : 0;

  auto stage_ptr = [&](int st) { return lds + st * 2 * kTileFloats; };

  // Single-barrier pipeline.  Iteration t: wait for tile t (vmcnt(0) / lgkmcnt(0)) and barrier
  // (which also proves every wave finished reading the other stage), immediately start
  // filling the other stage with tile t+1 (LDS-DMA; a synchronous guarded fill for tails), then
  // run the 4 k-groups x 16 MFMAs with the next group's fragments read (inline-asm ds_read,
  // double-buffered registers) under the current group's MFMAs.
  const uint32_t lds_b = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds;
  const int ra0 = wm * 64 + li, ra1 = ra0 + 32, rb0 = wn * 64 + li, rb1 = rb0 + 32;
  if (ntiles > 0) {
    float* sa = stage_ptr(0);
    if (dma && nfull > 0) {
      SA::issue_lds_dma(A, lda, m0, M, kbeg, sa, wid, lane);
      SB::issue_lds_dma(B, ldb, n0, N, kbeg, sa + kTileFloats, wid, lane);
    } else {
      float4 ra[4], rb[4];
      SA::load_guarded(A, lda, m0, M, kbeg, kend, a_vec, wid, lane, ra);
      SB::load_guarded(B, ldb, n0, N, kbeg, kend, b_vec, wid, lane, rb);
      SA::store_guarded(sa, wid, lane, ra);
      SB::store_guarded(sa + kTileFloats, wid, lane, rb);
    }
  }
  for (int64_t t = 0; t < ntiles; ++t) {
    const int cur = (int)(t & 1);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const bool next = t + 1 < ntiles;
    const int64_t k1 = kbeg + (t + 1) * BKT;
    float* na = stage_ptr(cur ^ 1);
    if (next && dma && t + 1 < nfull) {
      SA::issue_lds_dma(A, lda, m0, M, k1, na, wid, lane);
      SB::issue_lds_dma(B, ldb, n0, N, k1, na + kTileFloats, wid, lane);
    } else if (next) {  // tails / unaligned operands: synchronous guarded fill
      float4 ra[4], rb[4];
      SA::load_guarded(A, lda, m0, M, k1, kend, a_vec, wid, lane, ra);
      SB::load_guarded(B, ldb, n0, N, k1, kend, b_vec, wid, lane, rb);
      SA::store_guarded(na, wid, lane, ra);
      SB::store_guarded(na + kTileFloats, wid, lane, rb);
    }
    const uint32_t sa_b = lds_b + (uint32_t)(cur * 2 * kTileFloats * 4);
    const uint32_t sb_b = sa_b + kTileFloats * 4;
    if constexpr (H2) {
      // the same two 16-k steps, each fragment split into its two scaled fp16 planes; 4
      // sub-tiles x 3 fp16 MFMAs per step
      float4 f[2][4][2];  // [step][a0, a1, b0, b1][lo, hi]
      bf16x8 pa[2][2], pb[2][2];
#pragma unroll
      for (int T = 0; T < 2; ++T) {
        SA::frag8_asm(sa_b, ra0, 2 * T + lk, f[T][0][0], f[T][0][1]);
        SA::frag8_asm(sa_b, ra1, 2 * T + lk, f[T][1][0], f[T][1][1]);
        SB::frag8_asm(sb_b, rb0, 2 * T + lk, f[T][2][0], f[T][2][1]);
        SB::frag8_asm(sb_b, rb1, 2 * T + lk, f[T][3][0], f[T][3][1]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (RS) {
        if (rs_on) {  // wave-uniform: column half wn takes 16-k step wn
          if (wn == 0) {
            rs0 += hsum8(f[0][0][0], f[0][0][1]);
            rs1 += hsum8(f[0][1][0], f[0][1][1]);
          } else {
            rs0 += hsum8(f[1][0][0], f[1][0][1]);
            rs1 += hsum8(f[1][1][0], f[1][1][1]);
          }
        }
      }
#pragma unroll
      for (int T = 0; T < 2; ++T) {
        split2h8(f[T][0][0], f[T][0][1], s_a0, pa[0][0], pa[0][1]);
        split2h8(f[T][1][0], f[T][1][1], s_a1, pa[1][0], pa[1][1]);
        if constexpr (BPS) {
          pb[0][0] = __builtin_bit_cast(bf16x8, f[T][2][0]);
          pb[0][1] = __builtin_bit_cast(bf16x8, f[T][2][1]);
          pb[1][0] = __builtin_bit_cast(bf16x8, f[T][3][0]);
          pb[1][1] = __builtin_bit_cast(bf16x8, f[T][3][1]);
        } else {
          split2h8(f[T][2][0], f[T][2][1], s_b, pb[0][0], pb[0][1]);
          split2h8(f[T][3][0], f[T][3][1], s_b, pb[1][0], pb[1][1]);
        }
        acc[0][0] = mfma_np<2>(pa[0], pb[0], acc[0][0]);
        acc[0][1] = mfma_np<2>(pa[0], pb[1], acc[0][1]);
        acc[1][0] = mfma_np<2>(pa[1], pb[0], acc[1][0]);
        acc[1][1] = mfma_np<2>(pa[1], pb[1], acc[1][1]);
      }
      __builtin_amdgcn_sched_barrier(0);
    } else if constexpr (X3) {
      // two 16-k steps; the fp32 fragments of step 1 are read under step 0's MFMAs and split
      // there (VALU beside the matrix pipe); 4 sub-tiles x 6 bf16 MFMAs per step
      float4 f[2][4][2];  // [step][a0, a1, b0, b1][lo, hi]
      bf16x8 pa[2][3], pb[2][3];
#define MVML_FRAGS8(T)                                                          \
      SA::frag8_asm(sa_b, ra0, 2 * (T) + lk, f[T][0][0], f[T][0][1]);           \
      SA::frag8_asm(sa_b, ra1, 2 * (T) + lk, f[T][1][0], f[T][1][1]);           \
      SB::frag8_asm(sb_b, rb0, 2 * (T) + lk, f[T][2][0], f[T][2][1]);           \
      SB::frag8_asm(sb_b, rb1, 2 * (T) + lk, f[T][3][0], f[T][3][1]);
#define MVML_SPLIT(T)                                                           \
      split3(f[T][0][0], f[T][0][1], pa[0][0], pa[0][1], pa[0][2]);             \
      split3(f[T][1][0], f[T][1][1], pa[1][0], pa[1][1], pa[1][2]);             \
      split3(f[T][2][0], f[T][2][1], pb[0][0], pb[0][1], pb[0][2]);             \
      split3(f[T][3][0], f[T][3][1], pb[1][0], pb[1][1], pb[1][2]);
#define MVML_MFMAS3()                                                           \
      acc[0][0] = mfma_x3(pa[0], pb[0], acc[0][0]);                             \
      acc[0][1] = mfma_x3(pa[0], pb[1], acc[0][1]);                             \
      acc[1][0] = mfma_x3(pa[1], pb[0], acc[1][0]);                             \
      acc[1][1] = mfma_x3(pa[1], pb[1], acc[1][1]);
      MVML_FRAGS8(0)
      MVML_FRAGS8(1)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      MVML_SPLIT(0)
      MVML_MFMAS3()
      MVML_SPLIT(1)
      MVML_MFMAS3()
      __builtin_amdgcn_sched_barrier(0);
#undef MVML_FRAGS8
#undef MVML_SPLIT
#undef MVML_MFMAS3
    } else {
    float4 fa0[2], fa1[2], fb0[2], fb1[2];  // [register set] x (sub-tile 0 / 1)
#define MVML_FRAGS(G, SET)                                  \
    SA::template frag_asm<G>(sa_b, ra0, lk, fa0[SET]);      \
    SA::template frag_asm<G>(sa_b, ra1, lk, fa1[SET]);      \
    SB::template frag_asm<G>(sb_b, rb0, lk, fb0[SET]);      \
    SB::template frag_asm<G>(sb_b, rb1, lk, fb1[SET]);
#define MVML_MFMAS(SET)                                                                                      \
    _Pragma("unroll") for (int s = 0; s < 4; ++s) {                                                          \
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(comp(fa0[SET], s), comp(fb0[SET], s), acc[0][0], 0, 0, 0); \
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(comp(fa0[SET], s), comp(fb1[SET], s), acc[0][1], 0, 0, 0); \
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(comp(fa1[SET], s), comp(fb0[SET], s), acc[1][0], 0, 0, 0); \
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(comp(fa1[SET], s), comp(fb1[SET], s), acc[1][1], 0, 0, 0); \
    }
#define MVML_WAIT_LDS()                                  \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   \
    __builtin_amdgcn_sched_barrier(0);
    MVML_FRAGS(0, 0)
    MVML_WAIT_LDS()
    MVML_FRAGS(1, 1)
    MVML_MFMAS(0)
    MVML_WAIT_LDS()
    MVML_FRAGS(2, 0)
    MVML_MFMAS(1)
    MVML_WAIT_LDS()
    MVML_FRAGS(3, 1)
    MVML_MFMAS(0)
    MVML_WAIT_LDS()
    MVML_MFMAS(1)
    __builtin_amdgcn_sched_barrier(0);
#undef MVML_FRAGS
#undef MVML_MFMAS
#undef MVML_WAIT_LDS
    }
  }

  if constexpr (RS) {
    if (rs_on) {
      rs0 += __shfl_xor(rs0, 32, 64);  // + the other k half of the same rows
      rs1 += __shfl_xor(rs1, 32, 64);
      if (lk == 0) {
        float* dst = amax.a_rowsum + (split * 2 + wn) * M;
        const int64_t r = m0 + wm * 64 + li;
        if (r < M) dst[r] = rs0;
        if (r + 32 < M) dst[r + 32] = rs1;
      }
    }
  }
  if constexpr (H2) unscale_rows(acc, amax.a_rows != nullptr, ka, ka0, ka1, kb, lane);
  if constexpr (H2 && EPI_LOGW < 0) {
    if (cep.D > 0) {  // LSTM cell epilogue through LDS (host: N = 4 D, no split-K)
      __syncthreads();  // every wave is done reading the last stage
      epilogue_lds(acc, lds + wid * 32 * kEpiLd, M, N, m0 + wm * 64, n0 + wn * 64, lane, bias, beta,
                   act, C, ldc, slab, cep);
      return;
    }
  }
  tile_epilogue<EPI_LOGW>(acc, M, N, m0 + wm * 64, n0 + wn * 64, lane, bias, beta, act, C, ldc,
                          slab, epi, split);
}

// ---- split-bf16 GEMM with the split done once per workgroup, at staging -------------------
// The fp32 tile is loaded into registers (one tile ahead), split into its three bf16 terms and
// written to LDS as three bf16 planes per operand; the waves then read ready-made MFMA operand
// fragments (ds_read_b128), so an element is split once per workgroup instead of once per wave
// that reads it (half the VALU of splitting fragments).
// LDS image per operand: 3 planes x 128 rows x 32 k bf16 (64-B rows); the 16-B chunk (8 k) is
// XOR-swizzled by (row >> 2) & 3, so 8 consecutive rows read at one chunk hit 8 distinct 16-B
// bank groups.  48 KB per workgroup, two workgroups per CU.
constexpr int kPlaneBytes = 128 * 64;
constexpr int kOpBytes = 3 * kPlaneBytes;

__device__ __forceinline__ uint32_t plane_off(int plane, int row, int chunk) {
  return (uint32_t)(plane * kPlaneBytes + row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4));
}

// 4 fp32 -> three bf16 x 4 terms (two dwords each).
__device__ __forceinline__ void split4(float a, float b, float c, float d, uint2& p0, uint2& p1,
                                       uint2& p2) {
  p0.x = split_pair(a, b);
  p0.y = split_pair(c, d);
  p1.x = split_pair(a, b);
  p1.y = split_pair(c, d);
  const f32x2 u = {a, b}, w = {c, d};
  p2.x = __builtin_bit_cast(uint32_t, __builtin_convertvector(u, bf16x2));
  p2.y = __builtin_bit_cast(uint32_t, __builtin_convertvector(w, bf16x2));
}

// A thread's 16 values of a 128 x 32 operand tile.
//  * K-contiguous ([rows][K]): row = tid >> 1, k = 16 (tid & 1) + 4 i + [0, 4) in v[i].
//  * K-major ([K][rows]): rows 4 (tid & 31) + [0, 4) in v[i].{x,y,z,w}, k = 4 (tid >> 5) + i.
template <bool KMAJ>
struct SplitStager {
  __device__ static __forceinline__ void load(const float* __restrict__ P, int64_t ld, int64_t r0,
                                              int64_t rows, int64_t k0, int64_t kend, bool fast,
                                              int tid, float4 (&v)[4]) {
    if (!KMAJ) {
      const int64_t row = r0 + (tid >> 1), kb = k0 + 16 * (tid & 1);
      if (fast) {
        const float* p = P + row * ld + kb;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = *reinterpret_cast<const float4*>(p + 4 * i);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float e[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int64_t k = kb + 4 * i + j;
            e[j] = (row < rows && k < kend) ? P[row * ld + k] : 0.f;
          }
          v[i] = make_float4(e[0], e[1], e[2], e[3]);
        }
      }
    } else {
      const int64_t rb = r0 + 4 * (tid & 31), kb = k0 + 4 * (tid >> 5);
      if (fast) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = *reinterpret_cast<const float4*>(P + (kb + i) * ld + rb);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float e[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int64_t k = kb + i, r = rb + j;
            e[j] = (r < rows && k < kend) ? P[k * ld + r] : 0.f;
          }
          v[i] = make_float4(e[0], e[1], e[2], e[3]);
        }
      }
    }
  }

  // Scaled split-fp16 (two planes; the 256x256 kernel's split2h): same LDS image, planes 0 / 1.
  __device__ static __forceinline__ void split_store_h2(uint8_t* op, int tid, const float4 (&v)[4],
                                                        float s) {
    if (!KMAJ) {
      const int row = tid >> 1;
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        bf16x8 h, l;
        split2h8(v[2 * g], v[2 * g + 1], s, h, l);
        const int chunk = 2 * (tid & 1) + g;
        *reinterpret_cast<bf16x8*>(op + plane_off(0, row, chunk)) = h;
        *reinterpret_cast<bf16x8*>(op + plane_off(1, row, chunk)) = l;
      }
    } else {
      const int rb = 4 * (tid & 31), kk = 4 * (tid >> 5);
      const int chunk = kk >> 3, half = (kk >> 2) & 1;
      const float* f = reinterpret_cast<const float*>(v);  // f[4 i + j]: k = kk + i, row rb + j
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint2 h, l;
        split2h(make_float4(f[j], f[4 + j], f[8 + j], f[12 + j]), s, h, l);
        const int row = rb + j;
        *reinterpret_cast<uint2*>(op + plane_off(0, row, chunk) + 8 * half) = h;
        *reinterpret_cast<uint2*>(op + plane_off(1, row, chunk) + 8 * half) = l;
      }
    }
  }

  __device__ static __forceinline__ void split_store(uint8_t* op, int tid, const float4 (&v)[4]) {
    if (!KMAJ) {
      const int row = tid >> 1;
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        bf16x8 p0, p1, p2;
        split3(v[2 * g], v[2 * g + 1], p0, p1, p2);
        const int chunk = 2 * (tid & 1) + g;
        *reinterpret_cast<bf16x8*>(op + plane_off(0, row, chunk)) = p0;
        *reinterpret_cast<bf16x8*>(op + plane_off(1, row, chunk)) = p1;
        *reinterpret_cast<bf16x8*>(op + plane_off(2, row, chunk)) = p2;
      }
    } else {
      const int rb = 4 * (tid & 31), kk = 4 * (tid >> 5);
      const int chunk = kk >> 3, half = (kk >> 2) & 1;
      const float* f = reinterpret_cast<const float*>(v);  // f[4 i + j]: k = kk + i, row rb + j
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint2 p0, p1, p2;
        split4(f[j], f[4 + j], f[8 + j], f[12 + j], p0, p1, p2);
        const int row = rb + j;
        *reinterpret_cast<uint2*>(op + plane_off(0, row, chunk) + 8 * half) = p0;
        *reinterpret_cast<uint2*>(op + plane_off(1, row, chunk) + 8 * half) = p1;
        *reinterpret_cast<uint2*>(op + plane_off(2, row, chunk) + 8 * half) = p2;
      }
    }
  }
};

#ifndef MVML_X3S_WAVES
#define MVML_X3S_WAVES 2
#endif
// H2: scaled split-fp16 planes (two per operand, three fp16 MFMAs per fragment pair; scales from
// amax) instead of split-bf16 (three planes, six MFMAs) — the skinny plan of the f16x2 algorithm.
template <bool AK, bool BKM, int EPI_LOGW = -1, bool H2 = false>
__global__ void __launch_bounds__(kThreads, MVML_X3S_WAVES)  // 2 workgroups per CU
gemm_x3s_kernel(int64_t M, int64_t N, int64_t K, const float* __restrict__ A, int64_t lda,
                const float* __restrict__ B, int64_t ldb, const float* __restrict__ bias,
                float beta, int act, float* __restrict__ C, int64_t ldc, int64_t k_split,
                float* __restrict__ slab, int a_vec, int b_vec, ProjEpi epi = ProjEpi{},
                BatchStrides bst = BatchStrides{}, AmaxPtrs amax = AmaxPtrs{}) {
  if (blockIdx.z) {  // strided batch
    A += blockIdx.z * bst.a;
    B += blockIdx.z * bst.b;
    C += blockIdx.z * bst.c;
  }
  using SA = SplitStager<AK>;
  using SB = SplitStager<BKM>;
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * kOpBytes];
  const int64_t tiles_n = ceil_div(N, BN);
  const int64_t tile = xcd_block(blockIdx.x, gridDim.x);
  const int64_t m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int64_t kbeg = (int64_t)blockIdx.y * k_split;
  const int64_t kend = min(K, kbeg + k_split);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int li = lane & 31, lk = lane >> 5;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  int ka = 0, kb = 0;  // H2: operand scales 2^ka, 2^kb from the |max| bits
  int ka0 = 0, ka1 = 0, kst = 0;  // per-row A maxima: this lane's fragment rows, its staged row
  if constexpr (H2) {
    kb = amax_shift(*amax.b);
    if (amax.a_rows) {  // (host: K-contiguous A)
      ka0 = row_shift(amax, m0 + wm * 64 + li, M);
      ka1 = row_shift(amax, m0 + wm * 64 + li + 32, M);
      kst = row_shift(amax, m0 + (tid >> 1), M);
    } else {
      ka = ka0 = ka1 = kst = amax_shift(*amax.a);
    }
  }
  const float s_a = pow2f(kst), s_b = pow2f(kb);
  const int64_t ntiles = (kend > kbeg) ? ceil_div(kend - kbeg, BKT) : 0;
  // unguarded 16-B loads when the whole tile is in range and rows are 16-B aligned
  const bool a_in = a_vec && (AK ? m0 + BM <= M : m0 + BM <= M);
  const bool b_in = b_vec && (BKM ? n0 + BN <= N : n0 + BN <= N);
  float4 va[4], vb[4];
  auto load_tile = [&](int64_t k0) {
    const bool kin = k0 + BKT <= kend;
    SA::load(A, lda, m0, M, k0, kend, a_in && kin, tid, va);
    SB::load(B, ldb, n0, N, k0, kend, b_in && kin, tid, vb);
  };
  if (ntiles > 0) load_tile(kbeg);
  const int ra0 = wm * 64 + li, ra1 = ra0 + 32, rb0 = wn * 64 + li, rb1 = rb0 + 32;
  for (int64_t t = 0; t < ntiles; ++t) {
    if (t > 0) __syncthreads();  // every wave is done reading the previous tile
    if constexpr (H2) {
      SA::split_store_h2(lds, tid, va, s_a);
      SB::split_store_h2(lds + kOpBytes, tid, vb, s_b);
    } else {
      SA::split_store(lds, tid, va);
      SB::split_store(lds + kOpBytes, tid, vb);
    }
    __syncthreads();
    if (t + 1 < ntiles) load_tile(kbeg + (t + 1) * BKT);  // in flight under the MFMAs
    constexpr int NPL = H2 ? 2 : 3;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int chunk = 2 * st + lk;
      bf16x8 pa[2][NPL], pb[2][NPL];
#pragma unroll
      for (int p = 0; p < NPL; ++p) {
        pa[0][p] = *reinterpret_cast<const bf16x8*>(lds + plane_off(p, ra0, chunk));
        pa[1][p] = *reinterpret_cast<const bf16x8*>(lds + plane_off(p, ra1, chunk));
        pb[0][p] = *reinterpret_cast<const bf16x8*>(lds + kOpBytes + plane_off(p, rb0, chunk));
        pb[1][p] = *reinterpret_cast<const bf16x8*>(lds + kOpBytes + plane_off(p, rb1, chunk));
      }
      acc[0][0] = mfma_np<NPL>(pa[0], pb[0], acc[0][0]);
      acc[0][1] = mfma_np<NPL>(pa[0], pb[1], acc[0][1]);
      acc[1][0] = mfma_np<NPL>(pa[1], pb[0], acc[1][0]);
      acc[1][1] = mfma_np<NPL>(pa[1], pb[1], acc[1][1]);
    }
  }
  if constexpr (H2) unscale_rows(acc, amax.a_rows != nullptr, ka, ka0, ka1, kb, lane);
  tile_epilogue<EPI_LOGW>(acc, M, N, m0 + wm * 64, n0 + wn * 64, lane, bias, beta, act, C, ldc,
                          slab, epi);
}

// ---- 256x256 split-bf16 GEMM, one workgroup per CU ---------------------------------------
// 512 threads = 8 waves as 2 (M) x 4 (N); a wave owns 128 x 64 outputs = 4 x 2 accumulators of
// 32x32 (48 MFMAs per 16-deep k step: 4x the MFMAs per staged element of the 128x128 kernels,
// so the per-element split and LDS writes are a quarter of the cost).  K is staged 16 deep: the
// next fp32 tile (8 values per thread per operand) is loaded into registers one stage ahead,
// split into three bf16 terms and written into the free half of a double-buffered LDS image
// while the current stage's MFMAs run; one barrier per stage.
//  * K-contiguous operands ([rows][K]) live as [row][16 k] bf16 planes (32-B rows; the 16-B
//    chunk XOR-ed with row bit 3), read as 32x32x16 fragments by one ds_read_b128 per plane
//    (conflict-free over the instruction's 16-lane groups).
//  * K-major operands ([K][rows]) live as [k][256 rows] bf16 planes (k-row pitch 576 B: the four
//    k rows of a transposed read land on four different bank quarters) and are read by two
//    ds_read_b64_tr_b16 per plane — the hardware transpose delivers a lane its row's 8
//    consecutive k — so both layouts are staged with contiguous, conflict-free writes.
constexpr int XBM = 256, XBN = 256, XBK = 16, kXThreads = 512;
constexpr int kXKmajPitch = 576;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <bool KMAJ, int NP = 3, int NTH = kXThreads>
struct XOp {
  static constexpr int kPlane = KMAJ ? XBK * kXKmajPitch : 256 * 32;
  static constexpr int kBytes = NP * kPlane;  // NP = 3 split-bf16 planes, 1 = plain bf16
  // float4 pieces per thread of a 256 x 16 tile (1024 pieces), the K-contiguous row stride
  static constexpr int NI = 1024 / NTH, RS = NTH / 4;

  // This thread's 8 values of a 256 x 16 operand tile (rows r0.., k0..):
  //  K-contiguous: rows (tid >> 2) + 128 i, k = 4 (tid & 3) + [0, 4) in v[i] (16 rows x 64 B per
  //  wave-instruction); K-major: k = 2 (tid >> 6) + i, rows 4 (tid & 63) + [0, 4) in v[i] (1 KB
  //  contiguous per wave-instruction).  Guarded path zero-fills rows >= rows, k >= kend.
  __device__ static __forceinline__ void load(const float* __restrict__ P, int64_t ld, int64_t r0,
                                              int64_t rows, int64_t k0, int64_t kend, bool fast,
                                              int tid, float4 (&v)[NI]) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (!KMAJ) {
        const int64_t row = r0 + (tid >> 2) + RS * i, k = k0 + 4 * (tid & 3);
        if (fast) {
          v[i] = *reinterpret_cast<const float4*>(P + row * ld + k);
        } else {
          float e[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) e[j] = (row < rows && k + j < kend) ? P[row * ld + k + j] : 0.f;
          v[i] = make_float4(e[0], e[1], e[2], e[3]);
        }
      } else {
        const int64_t k = k0 + NI * (tid >> 6) + i, row = r0 + 4 * (tid & 63);
        if (fast) {
          v[i] = *reinterpret_cast<const float4*>(P + k * ld + row);
        } else {
          float e[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) e[j] = (k < kend && row + j < rows) ? P[k * ld + row + j] : 0.f;
          v[i] = make_float4(e[0], e[1], e[2], e[3]);
        }
      }
    }
  }

  // Fast path: this thread's two source pointers, rows clamped into range (a clamped row only
  // feeds output rows / columns that are never stored; K-major needs rows % 4 == 0 or a full
  // tile so that no float4 straddles the edge), advanced by kStep floats per stage.
  __device__ static __forceinline__ void ptrs(const float* __restrict__ P, int64_t ld, int64_t r0,
                                              int64_t rows, int64_t k0, int tid,
                                              const float* (&p)[NI]) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (!KMAJ) {
        const int64_t row = min(r0 + (tid >> 2) + RS * i, rows - 1);
        p[i] = P + row * ld + k0 + 4 * (tid & 3);
      } else {
        const int64_t row = min(r0 + 4 * (tid & 63), rows - 4);
        p[i] = P + (k0 + NI * (tid >> 6) + i) * ld + row;
      }
    }
  }
  __device__ static __forceinline__ int64_t kstep(int64_t ld) { return KMAJ ? XBK * ld : XBK; }


  __device__ static __forceinline__ void split_store(uint8_t* op, int tid, const float4 (&v)[NI],
                                                     float s = 1.f) {
    float sv[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) sv[i] = s;
    split_store(op, tid, v, sv);
  }
  // s[i]: the scale of piece i (split-fp16; per-row A maxima give the pieces' rows their own)
  __device__ static __forceinline__ void split_store(uint8_t* op, int tid, const float4 (&v)[NI],
                                                     const float (&s)[NI]) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      uint2 p0, p1, p2;
      if constexpr (NP == 3) {
        split4(v[i].x, v[i].y, v[i].z, v[i].w, p0, p1, p2);
      } else if constexpr (NP == 2) {
        split2h(v[i], s[i], p0, p1);
      } else {  // bf16 operands: round-to-nearest-even, one plane
        const f32x2 u = {v[i].x, v[i].y}, w = {v[i].z, v[i].w};
        p0.x = __builtin_bit_cast(uint32_t, __builtin_convertvector(u, bf16x2));
        p0.y = __builtin_bit_cast(uint32_t, __builtin_convertvector(w, bf16x2));
      }
      uint32_t off;
      if (!KMAJ) {
        const int row = (tid >> 2) + RS * i, q = tid & 3;
        off = row * 32 + (((q >> 1) ^ ((row >> 3) & 1)) << 4) + 8 * (q & 1);
      } else {
        off = (NI * (tid >> 6) + i) * kXKmajPitch + 8 * (tid & 63);
      }
      *reinterpret_cast<uint2*>(op + off) = p0;
      if constexpr (NP >= 2) *reinterpret_cast<uint2*>(op + kPlane + off) = p1;
      if constexpr (NP == 3) *reinterpret_cast<uint2*>(op + 2 * kPlane + off) = p2;
    }
  }

  // pre-split operand (BPS): v[i] carries the piece's high plane bits in .x .y and its low plane
  // bits in .z .w (loaded from the fp16 planes of mvml_split_f16x2); same LDS image as split_store
  __device__ static __forceinline__ void store_planes(uint8_t* op, int tid, const float4 (&v)[NI]) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const uint2 p0 = make_uint2(__float_as_uint(v[i].x), __float_as_uint(v[i].y));
      const uint2 p1 = make_uint2(__float_as_uint(v[i].z), __float_as_uint(v[i].w));
      uint32_t off;
      if (!KMAJ) {
        const int row = (tid >> 2) + RS * i, q = tid & 3;
        off = row * 32 + (((q >> 1) ^ ((row >> 3) & 1)) << 4) + 8 * (q & 1);
      } else {
        off = (NI * (tid >> 6) + i) * kXKmajPitch + 8 * (tid & 63);
      }
      *reinterpret_cast<uint2*>(op + off) = p0;
      *reinterpret_cast<uint2*>(op + kPlane + off) = p1;
    }
  }

  // 32x32x16 operand fragment of tile rows R0 .. R0+31, plane p: lane l holds row R0 + (l & 31),
  // k = 8 (l >> 5) + [0, 8).
  __device__ static __forceinline__ bf16x8 frag(const uint8_t* op, int p, int R0, int lane) {
    const uint8_t* pl = op + p * kPlane;
    if (!KMAJ) {
      const int row = R0 + (lane & 31);
      return *reinterpret_cast<const bf16x8*>(pl + row * 32 + (((lane >> 5) ^ ((row >> 3) & 1)) << 4));
    } else {
      // ds_read_b64_tr_b16: 16-lane group g reads k rows k0 .. k0+3, columns mb .. mb+15; lane
      // 4q+p of the group addresses row q, columns 4p .. 4p+3 and receives column (lane & 15)
      const int g = lane >> 4, i = lane & 15;
      const int mb = R0 + 16 * (g & 1), k0 = 8 * (g >> 1);
      const uint8_t* a = pl + (k0 + (i >> 2)) * kXKmajPitch + 2 * (mb + 4 * (i & 3));
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 4 * kXKmajPitch));
      const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, r);
    }
  }
};


#ifndef MVML_X3W_WAVES
#define MVML_X3W_WAVES 2
#endif
#ifndef MVML_X3W_LDSEPI
#define MVML_X3W_LDSEPI 1
#endif
#ifndef MVML_X3W_SGB
#define MVML_X3W_SGB 0
#endif
#ifndef MVML_X3W_PF2
#define MVML_X3W_PF2 0
#endif
#ifndef MVML_X3W_STAGGER
#define MVML_X3W_STAGGER 0
#endif
#ifndef MVML_X3W_SGB_V
#define MVML_X3W_SGB_V 3
#endif
#ifndef MVML_H2_SGB
#define MVML_H2_SGB 1
#endif
#ifndef MVML_H2_KS
#define MVML_H2_KS (MVML_H2_SGB ? 1 : 2)
#endif
#ifndef MVML_X3W_SGB_V2
#define MVML_X3W_SGB_V2 3
#endif
// FAST (host-checked: both operands 16-B aligned rows, K-major row counts % 4 == 0): whole
// stages by unguarded loads from clamped rows, the K tail as one guarded stage; !FAST: every
// stage guarded.
// NP = 3: fp32-accurate split-bf16 (six MFMAs per fragment pair); NP = 1: bf16 operands
// (one MFMA per pair, fp32 accumulate) — the bf16 projection of BASELINE config 4.
// BPS = 2 (split-fp16, FAST only): B points at the interleaved split image of the operand
// (mvml_split_f16x2_il4: [4 high | 4 low] fp16 per 16-B piece) instead of fp32 values: a B
// piece is one 16-B load stored to the LDS planes unsplit — the weights are split once per
// step instead of once per tile.
// ROWS (split-fp16, K-contiguous A): per-row A maxima (amax.a_rows), a scale per A row; a
// separate instantiation so that the operand-wide kernels keep their register allocation (one
// spill reload inside the main loop costs a vmcnt drain per stage).
template <bool AK, bool BKM, int EPI_LOGW = -1, bool FAST = true, int NP = 3, int BPS = 0,
          bool ROWS = false, bool EX = false>
__global__ void __launch_bounds__(kXThreads, MVML_X3W_WAVES)  // one workgroup per CU
gemm_x3w_kernel(int64_t M, int64_t N, int64_t K, const float* __restrict__ A, int64_t lda,
                const float* __restrict__ B, int64_t ldb, const float* __restrict__ bias,
                float beta, int act, float* __restrict__ C, int64_t ldc, int64_t k_split,
                float* __restrict__ slab, int a_vec, int b_vec, ProjEpi epi = ProjEpi{},
                BatchStrides bst = BatchStrides{}, CellEpi cep = CellEpi{},
                AmaxPtrs amax = AmaxPtrs{}, DualPtrs dual = DualPtrs{}, EpiX ex = EpiX{}) {
  if (blockIdx.z) {  // strided batch
    A += blockIdx.z * bst.a;
    B += blockIdx.z * bst.b;
    C += blockIdx.z * bst.c;
    if constexpr (EX) {
      if (bias) bias += blockIdx.z * ex.bias_z;
      if (amax.a_rows) amax.a_rows += blockIdx.z * ex.rows_z;
    }
  }
  if (blockIdx.z == 1 && dual.a) {  // the second product of a dual launch
    A = dual.a;
    B = dual.b;
    M = dual.m;
    slab = dual.slab;
    cep = dual.cep;
    amax.b = dual.amax_b;
    if (dual.amax_a) amax.a = dual.amax_a;
  }
  using OA = XOp<AK, NP>;
  using OB = XOp<BKM, NP>;
  static_assert(!BPS || (NP == 2 && FAST), "pre-split B: split-fp16 fast path only");
  // B piece at float-indexed address p: fp32 values, or
  // (BPS 2) the interleaved image's 16-B piece [4 high | 4 low] (mvml_split_f16x2_il4: the same
  // float indexing as the fp32 operand, one load per piece like fp32)
  auto ldb4 = [&](const float* p) -> float4 {
    if constexpr (BPS == 2) {
      return *reinterpret_cast<const float4*>(p);
    } else {
      return *reinterpret_cast<const float4*>(p);
    }
  };
  // NP = 2: operand scales from the |max| bits of A and B (per-row A maxima: amax.a_rows, a
  // shift per A row of the tile in rsh — host: K-contiguous A)
  static_assert(!ROWS || (NP == 2 && !AK), "per-row A maxima: split-fp16, K-contiguous A");
  int ka = 0, kb = 0;
  if constexpr (NP == 2) {
    if constexpr (!ROWS) ka = amax_shift(*amax.a);
    kb = amax_shift(*amax.b);
  }
  const float s_a = pow2f(ka), s_b = pow2f(kb);
  __shared__ int rsh[ROWS ? XBM : 1];
  // EX: per-row maxima of the tile folded in LDS, committed once per row (rows_cols 0 or whole
  // tiles: one slot per row of the workgroup)
  __shared__ uint32_t s_rmax[EX ? XBM : 1];
  const bool lds_rows = EX && ex.c_rows && !slab && cep.D == 0 && (ex.rows_cols == 0 || ex.rows_cols % XBN == 0);
  // KS 16-deep sub-stages per barrier (split-fp16: 2, so a stage carries as many MFMAs as the
  // split-bf16 one); a sub-stage's LDS image is exactly the KS = 1 stage layout
  // (round 4) products whose B comes pre-split (BPS: the il4 weight image) only split A in the
  // loop: the sched_group_barrier interleave, placed for the split of both operands, measured
  // slower there than two plain sub-stages per barrier (L2 forward 17.5 -> 16.8 ms, dX 15.7 ->
  // 15.5, LSTM gates 0.523 -> 0.514; profiles/r04_gemm_schedule_variants.txt), so it is kept
  // for the in-loop split of both operands only
  constexpr bool H2SGB = MVML_H2_SGB && BPS == 0;
  constexpr int KS = (NP == 2) ? (H2SGB ? MVML_H2_KS : 2) : 1;
  constexpr int kSub = OA::kBytes + OB::kBytes;
  constexpr int kStage = KS * kSub;
  // double-buffered stages; the LDS epilogue reuses the space (8 waves x 32 rows x kEpiLd)
  constexpr int kLdsBytes = 2 * kStage > 8 * 32 * kEpiLd * 4 ? 2 * kStage : 8 * 32 * kEpiLd * 4;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  const int64_t tiles_n = ceil_div(N, XBN);
  // Tile loop (persistent when the host launches fewer workgroups than tiles): XCD x = the
  // blocks b with b % 8 == x walks ONE contiguous range of tiles (the xcd_block partition),
  // its cnt blocks interleaved, so the tiles in flight on an XCD share A row panels in its L2.
  // A workgroup's next tile starts while its last tile's C stores drain.
  const int64_t n_tiles = ceil_div(M, XBM) * tiles_n;
  const unsigned xq = n_tiles / 8, xr = n_tiles % 8, bx = blockIdx.x % 8;
  const int64_t t_beg = (bx < xr) ? bx * (xq + 1) : xr * (xq + 1) + (bx - xr) * xq;
  const int64_t t_end = t_beg + xq + (bx < xr ? 1 : 0);
  const unsigned bq = gridDim.x / 8, br = gridDim.x % 8;
  int64_t t_first = t_beg + blockIdx.x / 8, t_stop = t_end;
  int64_t t_step = bq + (bx < br ? 1 : 0);  // blocks on this XCD
  // Split-K grids (one workgroup per (tile, split), never persistent): the pairs in split-major
  // order, each XCD a contiguous range (xcd_block over the dispatch order), so all tiles of a K
  // split run on one XCD together and its K chunk of both operands streams from HBM once into
  // that L2 (tile-major, every XCD re-read all of the operand its tiles do not own: the layer-2
  // weight gradient's 5.4 GB of X eight times).  The slab pointer is shifted so the epilogue's
  // blockIdx.y-indexed store lands in this pair's split.
  int64_t split = blockIdx.y;
  if (gridDim.y > 1) {
    const unsigned L = blockIdx.x + blockIdx.y * gridDim.x;
    const int64_t pair = xcd_block(L, gridDim.x * gridDim.y);
    split = pair / gridDim.x;
    t_first = pair % gridDim.x;
    t_stop = t_first + 1;
    t_step = 1;
    if (t_first >= n_tiles) return;
    if (slab) slab += (split - (int64_t)blockIdx.y) * M * N;
  }
  for (int64_t tile = t_first; tile < t_stop; tile += t_step) {
  if (tile != t_first) __syncthreads();  // the previous tile's epilogue LDS reads
  const int64_t m0 = (tile / tiles_n) * XBM, n0 = (tile % tiles_n) * XBN;
  const int64_t kbeg = split * k_split;
  const int64_t kend = min(K, kbeg + k_split);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  // ROWS: the scales of this thread's staged A pieces (rows (tid >> 2) + 128 i)
  float sa_i[OA::NI];
#pragma unroll
  for (int i = 0; i < OA::NI; ++i) sa_i[i] = s_a;
  if constexpr (ROWS) {
#pragma unroll
    for (int i = 0; i < OA::NI; ++i) sa_i[i] = pow2f(row_shift(amax, m0 + (tid >> 2) + OA::RS * i, M));
    // every row's shift for the epilogue (read after the K loop's barriers)
    if (tid < XBM) rsh[tid] = row_shift(amax, m0 + tid, M);
  }
  if constexpr (EX) {
    if (lds_rows && tid < XBM) s_rmax[tid] = 0u;  // (read after the K loop's barriers)
  }

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int64_t ntiles = (kend > kbeg) ? ceil_div(kend - kbeg, XBK * KS) : 0;
  const float* pa[2];
  const float* pb[2];
  OA::ptrs(A, lda, m0, M, kbeg, tid, pa);
  OB::ptrs(B, ldb, n0, N, kbeg, tid, pb);
  const int64_t sa_step = OA::kstep(lda), sb_step = OB::kstep(ldb);  // per 16-deep sub-stage
  float4 va[KS][2], vb[KS][2];
  auto load_fast = [&]() {
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        va[s][i] = *reinterpret_cast<const float4*>(pa[i] + s * sa_step);
        vb[s][i] = ldb4(pb[i] + s * sb_step);
      }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      pa[i] += KS * sa_step;
      pb[i] += KS * sb_step;
    }
  };
  // fast load of a stage that may be the K tail: addresses clamped to k < kend (host: kend %
  // 4 == 0), A's values at k >= kend zeroed, so B's clamped (finite) values add nothing
  auto load_masked_into = [&](int64_t t, float4 (&xa)[2], float4 (&xb)[2]) {
    const int64_t k0 = kbeg + t * XBK;  // t counts 16-deep sub-stages here
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int64_t ka, kb_;  // this thread's k for operand A / B piece i
      const float* qa;
      const float* qb;
      if (!AK) {
        ka = k0 + 4 * (tid & 3);
        qa = pa[i] + (min(ka, kend - 4) - ka);
      } else {
        ka = k0 + 2 * (tid >> 6) + i;
        qa = pa[i] + (min(ka, kend - 1) - ka) * lda;
      }
      if (!BKM) {
        kb_ = k0 + 4 * (tid & 3);
        qb = pb[i] + (min(kb_, kend - 4) - kb_);
      } else {
        kb_ = k0 + 2 * (tid >> 6) + i;
        qb = pb[i] + (min(kb_, kend - 1) - kb_) * ldb;
      }
      const float4 a = *reinterpret_cast<const float4*>(qa);
      xa[i] = ka < kend ? a : make_float4(0.f, 0.f, 0.f, 0.f);
      xb[i] = ldb4(qb);
      pa[i] += sa_step;
      pb[i] += sb_step;
    }
  };
  auto load_masked = [&](int64_t t) {  // stage t (KS sub-stages), each masked at kend
#pragma unroll
    for (int s = 0; s < KS; ++s) load_masked_into(t * KS + s, va[s], vb[s]);  // advances pa / pb
  };
  auto load_guarded = [&](int64_t t) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int64_t k0 = kbeg + (t * KS + s) * XBK;
      const bool kin = k0 + XBK <= kend;
      OA::load(A, lda, m0, M, k0, kend, a_vec && m0 + XBM <= M && kin, tid, va[s]);
      OB::load(B, ldb, n0, N, k0, kend, b_vec && n0 + XBN <= N && kin, tid, vb[s]);
    }
  };
  auto stage = [&](int buf) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      uint8_t* op = lds + buf * kStage + s * kSub;
      if constexpr (ROWS)
        OA::split_store(op, tid, va[s], sa_i);
      else
        OA::split_store(op, tid, va[s], s_a);
      if constexpr (BPS)
        OB::store_planes(op + OA::kBytes, tid, vb[s]);
      else
        OB::split_store(op + OA::kBytes, tid, vb[s], s_b);
    }
  };
#ifndef MVML_X3W_PRIO
#define MVML_X3W_PRIO 1
#endif
  // One 16-deep stage: fragments of stage t from LDS buffer t & 1; with STAGE, split + store
  // stage t+1 (in va / vb) into the other buffer; LOAD: 0 none, 1 fast, 2 guarded load of t+2.
  // Each (STAGE, LOAD) is its own straight-line body: no control flow around the accumulators.
  auto body = [&](int64_t t, auto STAGE, auto LOAD) {
#if MVML_X3W_SGB || MVML_H2_SGB
    const uint8_t* sa = lds + (t & 1) * kStage;
    const uint8_t* sb = sa + OA::kBytes;
    bf16x8 fb[2][NP];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int p = 0; p < NP; ++p) fb[j][p] = OB::frag(sb, p, wn * 64 + 32 * j, lane);
    if constexpr (MVML_X3W_SGB && decltype(STAGE)::value && NP == 3) {
      // Interleaved schedule: every fragment of stage t is read from LDS FIRST (so the split's
      // LDS writes into the other buffer, which the compiler cannot prove disjoint, do not pin
      // the reads behind them), then the split of stage t+1 (VALU + LDS writes) and the global
      // loads of stage t+2 ride in the MFMA stream of stage t (an MFMA leaves 24 of its 32 issue
      // cycles to other instructions), instead of running as a VALU-only phase in front of it
      // while the SIMD's matrix pipe idles (both waves of a SIMD reach that phase together).
      bf16x8 fa[4][NP];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int p = 0; p < NP; ++p) fa[i][p] = OA::frag(sa, p, wm * 128 + 32 * i, lane);
      stage((t + 1) & 1);
      if constexpr (decltype(LOAD)::value == 1) load_fast();
      if constexpr (decltype(LOAD)::value == 2) load_guarded(t + 2);
      if constexpr (decltype(LOAD)::value == 3) load_masked(t + 2);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma_np<NP>(fa[i], fb[j], acc[i][j]);
      // 0x8 MFMA, 0x2 VALU, 0x100 DS read, 0x200 DS write, 0x20 VMEM read
      __builtin_amdgcn_sched_group_barrier(0x100, 6 * NP, 0);  // fb + fa[0] + fa[1]
#pragma unroll
      for (int k = 0; k < 24; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x2, MVML_X3W_SGB_V, 0);
        if (k % 4 == 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        if (k == 2) __builtin_amdgcn_sched_group_barrier(0x100, 2 * NP, 0);  // fa[2] + fa[3]
      }
      __builtin_amdgcn_sched_group_barrier(0x20, 4, 0);  // next stage's global loads
#pragma unroll
      for (int k = 0; k < 24; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x2, 1, 0);
      }
      __syncthreads();
      return;
    }
    if constexpr (H2SGB && decltype(STAGE)::value && NP == 2 && KS == 1) {
      // the same interleave for split-fp16 (default): 24 MFMAs carry the 32 split VALU (8 per
      // float4: 2 pk_mul, 2 cvt_pk, 4 fma_mix), 8 LDS plane writes and the 4 global loads —
      // measured +3 / +7 / +3 % on the L2 forward / dX / dW shapes over two sub-stages per
      // barrier without the interleave (tools/gemm_bench.py)
      bf16x8 fa[4][NP];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int p = 0; p < NP; ++p) fa[i][p] = OA::frag(sa, p, wm * 128 + 32 * i, lane);
      stage((t + 1) & 1);
      if constexpr (decltype(LOAD)::value == 1) load_fast();
      if constexpr (decltype(LOAD)::value == 2) load_guarded(t + 2);
      if constexpr (decltype(LOAD)::value == 3) load_masked(t + 2);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma_np<NP>(fa[i], fb[j], acc[i][j]);
      __builtin_amdgcn_sched_group_barrier(0x100, 4 * NP, 0);  // fb + fa[0]
#pragma unroll
      for (int k = 0; k < 24; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x2, MVML_X3W_SGB_V2, 0);
        if (k % 3 == 2) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        if (k == 1 || k == 4 || k == 7) __builtin_amdgcn_sched_group_barrier(0x100, NP, 0);  // fa[1..3]
        if (k == 12) __builtin_amdgcn_sched_group_barrier(0x20, 4, 0);
      }
      __syncthreads();
      return;
    }
#endif
    auto stage_and_load = [&]() {
      if constexpr (decltype(STAGE)::value) stage((t + 1) & 1);
      if constexpr (decltype(LOAD)::value == 1) load_fast();
      if constexpr (decltype(LOAD)::value == 2) load_guarded(t + 2);
      if constexpr (decltype(LOAD)::value == 3) load_masked(t + 2);
    };
#if MVML_X3W_STAGGER
    // Stagger: waves 0-3 (one per SIMD) split stage t+1 BEFORE their MFMAs of stage t, waves
    // 4-7 (the SIMD partners) AFTER theirs, so each SIMD's matrix pipe runs one wave's MFMAs
    // while its partner does the VALU split, instead of both splitting together behind the
    // barrier.  The branches are wave-uniform and leave the accumulators alone.
    if (wid < 4) stage_and_load();
#else
    stage_and_load();
#endif
    // s_setprio around the MFMA block: measured +1-3 % slower for split-fp16 (NP = 2), kept for
    // the split-bf16 / bf16 instantiations
    constexpr bool kPrio = MVML_X3W_PRIO && NP != 2;
    if (kPrio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const uint8_t* sa = lds + (t & 1) * kStage + s * kSub;
      const uint8_t* sb = sa + OA::kBytes;
      bf16x8 fb[2][NP];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int p = 0; p < NP; ++p) fb[j][p] = OB::frag(sb, p, wn * 64 + 32 * j, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bf16x8 fa[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) fa[p] = OA::frag(sa, p, wm * 128 + 32 * i, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma_np<NP>(fa, fb[j], acc[i][j]);
      }
    }
    if (kPrio) __builtin_amdgcn_s_setprio(0);
#if MVML_X3W_STAGGER
    if (wid >= 4) stage_and_load();
#endif
    __syncthreads();
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  using L0 = std::integral_constant<int, 0>;
  using L1 = std::integral_constant<int, 1>;
  using L2 = std::integral_constant<int, 2>;
#if MVML_X3W_PF2
  if constexpr (FAST && KS == 1 && BPS == 0) {
    // Prefetch distance 2: tile k's fp32 values live in register set k % 2 from their load (in
    // body k - 3) to their split (in body k - 1), so a global load has two whole stages to land
    // instead of one (the loads of a stage are issued right after the split that frees the set).
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    using LM = std::integral_constant<int, 3>;
    float4 ra[2][2], rb[2][2];
    auto ldf = [&](auto SET) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ra[decltype(SET)::value][i] = *reinterpret_cast<const float4*>(pa[i]);
        rb[decltype(SET)::value][i] = *reinterpret_cast<const float4*>(pb[i]);
        pa[i] += sa_step;
        pb[i] += sb_step;
      }
    };
    auto ldm = [&](auto SET, int64_t k) {  // tile k, the K tail: as load_masked
      load_masked_into(k, ra[decltype(SET)::value], rb[decltype(SET)::value]);
    };
    auto stg = [&](auto SET, int buf) {
      OA::split_store(lds + buf * kStage, tid, ra[decltype(SET)::value], sa_i);
      OB::split_store(lds + buf * kStage + OA::kBytes, tid, rb[decltype(SET)::value], s_b);
    };
    auto body2 = [&](int64_t t, auto SET, auto STAGE, auto LOAD) {
      const uint8_t* sa = lds + (t & 1) * kStage;
      const uint8_t* sb = sa + OA::kBytes;
      bf16x8 fb[2][NP];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int p = 0; p < NP; ++p) fb[j][p] = OB::frag(sb, p, wn * 64 + 32 * j, lane);
      if constexpr (decltype(STAGE)::value) stg(SET, (int)((t + 1) & 1));
      if constexpr (decltype(LOAD)::value == 1) ldf(SET);
      if constexpr (decltype(LOAD)::value == 3) ldm(SET, t + 3);
      if (MVML_X3W_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bf16x8 fa[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) fa[p] = OA::frag(sa, p, wm * 128 + 32 * i, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma_np<NP>(fa, fb[j], acc[i][j]);
      }
      if (MVML_X3W_PRIO) __builtin_amdgcn_s_setprio(0);
      __syncthreads();
    };
    if (ntiles >= 1) { if (ntiles == 1) ldm(S0{}, 0); else ldf(S0{}); }
    if (ntiles >= 2) { if (ntiles == 2) ldm(S1{}, 1); else ldf(S1{}); }
    if (ntiles >= 1) stg(S0{}, 0);
    if (ntiles >= 3) { if (ntiles == 3) ldm(S0{}, 2); else ldf(S0{}); }
    __syncthreads();
    int64_t t = 0;
    for (; t + 5 < ntiles; t += 2) {  // body t loads tile t + 3 (a whole stage: t + 4 < ntiles)
      body2(t, S1{}, T_{}, L1{});
      body2(t + 1, S0{}, T_{}, L1{});
    }
    for (; t < ntiles; ++t) {  // at most 5 bodies: runtime parity / stage / load kind
      const bool st = t + 1 < ntiles;
      const int lk = (t + 4 < ntiles) ? 1 : (t + 4 == ntiles ? 3 : 0);
      auto tail = [&](auto SET) {
        if (!st) body2(t, SET, F_{}, L0{});
        else if (lk == 1) body2(t, SET, T_{}, L1{});
        else if (lk == 3) body2(t, SET, T_{}, LM{});
        else body2(t, SET, T_{}, L0{});
      };
      if ((t & 1) == 0) tail(S1{});
      else tail(S0{});
    }
  } else
#endif
  if constexpr (FAST) {
    using LM = std::integral_constant<int, 3>;
    if (ntiles >= 3) {
      load_fast();
      stage(0);
      load_fast();
      __syncthreads();
      int64_t t = 0;
      for (; t + 3 < ntiles; ++t) body(t, T_{}, L1{});  // loads stages t+2 < ntiles-1: whole
      body(t, T_{}, LM{});                             // loads the last stage (maybe the tail)
      body(t + 1, T_{}, L0{});
      body(t + 2, F_{}, L0{});
    } else if (ntiles == 2) {
      load_masked(0);
      stage(0);
      load_masked(1);
      __syncthreads();
      body(0, T_{}, L0{});
      body(1, F_{}, L0{});
    } else if (ntiles == 1) {
      load_masked(0);
      stage(0);
      __syncthreads();
      body(0, F_{}, L0{});
    }
  } else if (ntiles > 0) {  // generic guarded pipeline (unaligned / ragged K-major operands)
    load_guarded(0);
    stage(0);
    __syncthreads();
    for (int64_t t = 0; t < ntiles; ++t) {
      if (t + 1 < ntiles) load_guarded(t + 1);
      body(t, F_{}, L0{});
      if (t + 1 < ntiles) {
        stage((t + 1) & 1);
        __syncthreads();
      }
    }
  }
  if constexpr (NP == 2) {  // undo the operand scales (exact: powers of two)
    const float ub = pow2f(-kb);
    if constexpr (ROWS) {  // B's scale here, each row's own in the LDS epilogue (rsh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = acc[i][j][r] * ub;
    } else {
      const float ua = pow2f(-ka);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = acc[i][j][r] * ua * ub;
    }
  }
#if MVML_X3W_LDSEPI
  // the projection's logit partials straight from the accumulators, then C through LDS (every
  // K loop ends with a workgroup barrier, so the staging buffers are free)
  if constexpr (EPI_LOGW >= 0)
    tile_epilogue<EPI_LOGW, 4, 2, false>(acc, M, N, m0 + wm * 128, n0 + wn * 64, lane, bias, beta,
                                         act, C, ldc, slab, epi);
  epilogue_lds<4, EX>(acc, reinterpret_cast<float*>(lds) + wid * 32 * kEpiLd, M, N, m0 + wm * 128,
                      n0 + wn * 64, lane, bias, beta, act, C, ldc, slab, cep,
                      (ROWS && ntiles > 0) ? rsh + wm * 128 : nullptr, ex,
                      lds_rows ? s_rmax + wm * 128 : nullptr);
  if constexpr (EX) {
    if (lds_rows) {  // (uniform) one global atomicMax per row of the tile
      __syncthreads();
      const int64_t slot = ex.rows_cols > 0 ? n0 / ex.rows_cols : 0;
      if (tid < XBM && m0 + tid < M && s_rmax[tid] != 0u)
        atomicMax(ex.c_rows + blockIdx.z * ex.crows_z + slot * ex.rows_stride + m0 + tid, s_rmax[tid]);
    }
  }
#else
  static_assert(NP != 2, "per-row A maxima need the LDS epilogue");
  tile_epilogue<EPI_LOGW, 4, 2>(acc, M, N, m0 + wm * 128, n0 + wn * 64, lane, bias, beta, act, C,
                                ldc, slab, epi);
#endif
  }  // tile loop
}

// Host check for gemm_x3w_kernel<FAST = true>: aligned rows; a K-major operand's row count
// % 4 == 0 (its clamped float4 never straddles the edge); K % 4 == 0 when an operand is
// K-contiguous (the K tail's clamped float4 stays inside the row).
bool x3w_fast(bool ak, bool bk, int64_t M, int64_t N, int64_t K, int av, int bv) {
  return av && bv && ((ak && bk) || K % 4 == 0) && (!ak || M % 4 == 0) && (!bk || N % 4 == 0);
}

// Sum S split-K slabs in fixed order: C = act(sum_z slab[z] + bias + beta*C).
__global__ void splitk_reduce_kernel(int64_t M, int64_t N, int S, const float* __restrict__ slab,
                                     const float* __restrict__ bias, float beta, int act,
                                     float* __restrict__ C, int64_t ldc) {
  const int64_t total = M * N;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = e / N, col = e - row * N;
    float v = 0.f;
    for (int z = 0; z < S; ++z) v += slab[(int64_t)z * total + e];
    if (bias) v += bias[col];
    float* cp = C + row * ldc + col;
    if (beta != 0.f) v += beta * (*cp);
    if (act == 1) v = fmaxf(v, 0.f);
    *cp = v;
  }
}

// Split-K policy for small-output / long-K products (the weight gradients): pick the split
// count that fills whole rounds of resident workgroups (256 CUs x 2) best, keeping >= 1024 K
// per split so the slab reduction stays negligible.
// Split-K count for `tiles` output tiles over `slots` concurrent workgroups: the count that
// best fills whole waves of workgroups, keeping >= 1024 k per split.
int choose_splits_t(int64_t tiles, int64_t K, int64_t slots) {
  if (tiles >= 2 * slots || K < 2048) return 1;
  int best = 1;
  double best_eff = (double)tiles / (double)(ceil_div(tiles, slots) * slots);
  for (int s = 2; s <= 64; ++s) {
    if (K / s < 1024) break;
    const int64_t tot = tiles * s;
    const double eff = (double)tot / (double)(ceil_div(tot, slots) * slots);
    if (eff > best_eff + 1e-9) { best_eff = eff; best = s; }
  }
  return best;
}

// Kernel plan of a product: the 256x256 split-bf16 kernel (one workgroup per CU) whenever its
// tiles x splits fill the chip, the 128x128 kernels (two per CU) otherwise.  Option
// MVML_OPT_GEMM_TILE = 128 / 256 forces a tile size (tests).
struct GemmPlan {
  bool wide;
  int S;
};
constexpr int kPrecF32 = 0, kPrecX3 = 1, kPrecBf16 = 2, kPrecF16x2 = 3;  // = MVML_GEMM_* ids
GemmPlan plan_gemm(int prec, int64_t M, int64_t N, int64_t K) {
  const int force = option(MVML_OPT_GEMM_TILE);
  if (prec == kPrecBf16) {  // bf16 operands exist only in the 256x256 kernel
    const int64_t tw = ceil_div(M, XBM) * ceil_div(N, XBN);
    return {true, choose_splits_t(tw, K, 256)};
  }
  // split-fp16 exists only in the 256x256 kernel; its 128x128 fallback is the split-bf16 plan
  if (prec == kPrecX3 || prec == kPrecF16x2) {
    const int64_t tw = ceil_div(M, XBM) * ceil_div(N, XBN);
    const int Sw = choose_splits_t(tw, K, 256);
    // skinny outputs (N = 76 / 384 columns of weight gradients): the 256x256 tile computes
    // mostly padding; prefer 128x128 when it wastes clearly less (measured: L1 dW N=76 7.3 ->
    // 4.8 ms, LSTM dW N=384 2.52 -> 2.46 ms, tools/gemm_bench.py)
    const double u256 = (double)M * N / ((double)tw * XBM * XBN);
    const double u128 = (double)M * N / ((double)ceil_div(M, BM) * ceil_div(N, BN) * BM * BN);
    const bool skinny = u128 > 1.3 * u256;
    if (force == 256 || (force != 128 && !skinny && tw * Sw >= 192)) return {true, Sw};
  }
  return {false, choose_splits_t(ceil_div(M, BM) * ceil_div(N, BN), K, 512)};
}
int choose_splits(int64_t M, int64_t N, int64_t K) {  // the larger of the two plans' counts
  return std::max(choose_splits_t(ceil_div(M, XBM) * ceil_div(N, XBN), K, 256),
                  choose_splits_t(ceil_div(M, BM) * ceil_div(N, BN), K, 512));
}

int64_t k_chunk(int64_t K, int S) { return ceil_div(ceil_div(K, S), BKT) * BKT; }

// Workgroups of a 256x256 launch: option MVML_OPT_GEMM_PERSIST = P > 0 (default 256, one per CU)
// caps a launch without split-K at P workgroups that loop over their XCD's tiles.  Round 2
// measured it neutral; since the per-row / pre-split-B kernels (round 4) it is 1-9 % faster on
// every shape of the step (L1 projection 4.73 -> 4.29 ms, L2 forward 16.9 -> 16.3 ms; the step
// +1 %, profiles/r04_gemm_persist.txt); P = 0 gives one workgroup per tile.
unsigned x3w_grid_x(int64_t tiles, int S) {
  // the persistent kernels give XCD x (the workgroups b % 8 == x) one tile range each, so the
  // cap is rounded up to a multiple of 8: every XCD gets a workgroup and every range is walked
  int persist = option(MVML_OPT_GEMM_PERSIST);
  if (S > 1 || persist <= 0) return (unsigned)tiles;
  persist = (persist + 7) / 8 * 8;
  if (tiles <= persist) return (unsigned)tiles;
  return (unsigned)persist;
}

// Column sums, stage 1: each thread owns one column of a row chunk; eight independent partial
// sums keep eight loads in flight per lane (the loop is otherwise latency-bound).
__global__ void colsum_partial_kernel(int64_t M, int64_t N, const float* __restrict__ X,
                                      int64_t ldx, int64_t rows_per, float* __restrict__ part) {
  const int64_t col = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= N) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int64_t r = r0;
  for (; r + 8 <= r1; r += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += X[(r + j) * ldx + col];
  }
  for (; r < r1; ++r) s[0] += X[r * ldx + col];
  part[(int64_t)blockIdx.y * N + col] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

// out[col] = beta out[col] + alpha sum_z part[z ld + col]: a workgroup per 16 columns, 16 stripes of
// the S partials per column (four accumulators each, loads in flight), a fixed-order LDS tree —
// deterministic.  (A thread per column walking all S ~ 1024 partials took 20-70 us.)
__global__ void __launch_bounds__(256) colsum_final_kernel(int64_t N, int S, const float* __restrict__ part,
                                                           int64_t ld, float alpha, float beta,
                                                           float* __restrict__ out) {
  const int c = threadIdx.x & 15, stripe = threadIdx.x >> 4;
  const int64_t col = (int64_t)blockIdx.x * 16 + c;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (col < N) {
    int z = stripe;
    for (; z + 48 < S; z += 64) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += part[(int64_t)(z + 16 * u) * ld + col];
    }
    for (; z < S; z += 16) a[0] += part[(int64_t)z * ld + col];
  }
  __shared__ float red[16][17];
  red[stripe][c] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  for (int h = 8; h > 0; h >>= 1) {
    if (stripe < h) red[stripe][c] += red[stripe + h][c];
    __syncthreads();
  }
  if (stripe == 0 && col < N) out[col] = (beta != 0.f ? beta * out[col] : 0.f) + alpha * red[0][c];
}

// |max| of a stored rows x cols fp32 matrix (row pitch ld) folded into *out as float bits:
// non-negative float bits order like the values, so an unsigned atomicMax per workgroup is
// order-independent (deterministic).  Four independent rows in flight per thread.
__global__ void __launch_bounds__(256) absmax_kernel(int64_t rows, int64_t cols,
                                                     const float* __restrict__ P, int64_t ld,
                                                     int vec, uint32_t* __restrict__ out) {
  float m[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t rs = gridDim.y;
  if (vec) {  // cols % 4 == 0, ld % 4 == 0, 16-B aligned base: c indexes float4 columns
    if (c < cols / 4) {
      int64_t r = blockIdx.y;
      for (; r + 3 * rs < rows; r += 4 * rs) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(P + (r + u * rs) * ld + 4 * c);
#pragma unroll
        for (int u = 0; u < 4; ++u)
          m[u] = fmaxf(m[u], fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
      }
      for (; r < rows; r += rs) {
        const float4 v = *reinterpret_cast<const float4*>(P + r * ld + 4 * c);
        m[0] = fmaxf(m[0], fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      }
    }
  } else if (c < cols) {
    for (int64_t r = blockIdx.y; r < rows; r += rs) m[0] = fmaxf(m[0], fabsf(P[r * ld + c]));
  }
  float v = wave_max(fmaxf(fmaxf(m[0], m[1]), fmaxf(m[2], m[3])));
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    v = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(out, __float_as_uint(v));
  }
}

// |max| of a contiguous run of n floats (a matrix with ld == cols, or one row): grid-stride over
// float4s (vec) or floats, 4 loads in flight per thread, one atomicMax per workgroup.  The
// column-parallel absmax_kernel leaves all but `cols` lanes of a workgroup idle, which for the
// GAT layers' max-of-row-maxima (N x 1) was 1 live lane in 256: ~0.4 ms per 1.75 M atoms.
__global__ void __launch_bounds__(256) absmax_flat_kernel(int64_t n, const float* __restrict__ P,
                                                          int vec, uint32_t* __restrict__ out) {
  float m[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (vec) {
    const int64_t n4 = n / 4;
    const float4* P4 = reinterpret_cast<const float4*>(P);
    for (; i + 3 * stride < n4; i += 4 * stride) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = P4[i + u * stride];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        m[u] = fmaxf(m[u], fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
    }
    for (; i < n4; i += stride) {
      const float4 v = P4[i];
      m[0] = fmaxf(m[0], fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
  } else {
    for (; i < n; i += stride) m[0] = fmaxf(m[0], fabsf(P[i]));
  }
  float v = wave_max(fmaxf(fmaxf(m[0], m[1]), fmaxf(m[2], m[3])));
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    v = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(out, __float_as_uint(v));
  }
}

// Per-row |max| bits: a group of 2^lg lanes per row (float4 columns when vec), butterfly max;
// one writer per row (accumulate: max with the stored bits), so no atomics.
__global__ void __launch_bounds__(256) absmax_rows_kernel(int64_t rows, int64_t cols,
                                                          const float* __restrict__ P, int64_t ld,
                                                          int vec, int lg, int accumulate,
                                                          uint32_t* __restrict__ out) {
  const int L = 1 << lg;
  const int64_t groups = (int64_t)gridDim.x * (256 >> lg);
  const int sub = threadIdx.x & (L - 1);
  for (int64_t row = (int64_t)blockIdx.x * (256 >> lg) + (threadIdx.x >> lg); row < rows; row += groups) {
    const float* p = P + row * ld;
    float m = 0.f;
    if (vec) {
      for (int64_t c = sub; c < cols / 4; c += L) {
        const float4 v = *reinterpret_cast<const float4*>(p + 4 * c);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      }
    } else {
      for (int64_t c = sub; c < cols; c += L) m = fmaxf(m, fabsf(p[c]));
    }
    for (int o = L / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (sub == 0) {
      uint32_t b = __float_as_uint(m);
      if (accumulate) b = max(b, out[row]);
      out[row] = b;
    }
  }
}

// Interleaved pre-split of a K-contiguous operand for the 128x128 kernel's BPS path: every
// 8-value k group becomes its 8 scaled high fp16 halves then its 8 low halves (split2h8's h, l),
// 32 B in place of the group's 32 B of fp32, so the LDS-DMA staging and the swizzle are unchanged
// and a fragment read yields the two MFMA operands ready-made.  K % 8 == 0 (host).
__global__ void __launch_bounds__(256) split_f16x2_il_kernel(int64_t rows, int64_t groups,
                                                             const float* __restrict__ P, int64_t ld,
                                                             const uint32_t* __restrict__ amax,
                                                             float* __restrict__ out) {
  const float sc = pow2f(amax_shift(*amax));
  const int64_t total = rows * groups;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t r = e / groups, c = 8 * (e - r * groups);
    const float* src = P + r * ld + c;
    bf16x8 h, l;
    split2h8(*reinterpret_cast<const float4*>(src), *reinterpret_cast<const float4*>(src + 4), sc, h, l);
    float* dst = out + r * ld + c;
    *reinterpret_cast<float4*>(dst) = __builtin_bit_cast(float4, h);
    *reinterpret_cast<float4*>(dst + 4) = __builtin_bit_cast(float4, l);
  }
}

// Interleaved-by-4 pre-split for the 256x256 kernels (BPS 2): every 4-value group of a row
// becomes [4 scaled high fp16 | 4 low fp16] = 16 B in place of its 16 B of fp32, so the image
// has the operand's own float indexing (any layout, K-contiguous or K-major) and a staged piece
// is one 16-B load, stored to the LDS planes as it is (split2h of the kernel's own staging).
__global__ void __launch_bounds__(256) split_f16x2_il4_kernel(int64_t rows, int64_t cols4,
                                                              const float* __restrict__ P, int64_t ld,
                                                              const uint32_t* __restrict__ amax,
                                                              float* __restrict__ out) {
  const float sc = pow2f(amax_shift(*amax));
  const int64_t total = rows * cols4;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t r = e / cols4, c = 4 * (e - r * cols4);
    uint2 h, l;
    split2h(*reinterpret_cast<const float4*>(P + r * ld + c), sc, h, l);
    *reinterpret_cast<float4*>(out + r * ld + c) =
        make_float4(__uint_as_float(h.x), __uint_as_float(h.y), __uint_as_float(l.x), __uint_as_float(l.y));
  }
}

int split_il_launch(int64_t rows, int64_t K, const float* P, const uint32_t* amax, float* out,
                    hipStream_t st) {
  const int64_t total = rows * (K / 8);
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(total, 256), 4096));
  split_f16x2_il_kernel<<<blocks, 256, 0, st>>>(rows, K / 8, P, K, amax, out);
  return check_launch("split_f16x2_il_kernel");
}

int absmax_launch(int64_t rows, int64_t cols, const float* P, int64_t ld, uint32_t* out,
                  bool accumulate, hipStream_t st) {
  if (!accumulate && hipMemsetAsync(out, 0, sizeof(uint32_t), st) != hipSuccess) {
    set_error("absmax: hipMemsetAsync failed");
    return MVML_ERR_LAUNCH;
  }
  if (rows <= 0 || cols <= 0) return MVML_OK;
  if (ld == cols || rows == 1) {  // contiguous: one flat pass (also bounds the atomics at ~1 K)
    const int64_t n = rows * cols;
    const int fvec = (n % 4 == 0) && ((uintptr_t)P % 16 == 0);
    const unsigned blocks =
        (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(fvec ? n / 4 : n, 256 * 4), 1024));
    absmax_flat_kernel<<<blocks, 256, 0, st>>>(n, P, fvec, out);
    return check_launch("absmax_flat_kernel");
  }
  const int vec = (cols % 4 == 0) && (ld % 4 == 0) && ((uintptr_t)P % 16 == 0);
  const int64_t cx = ceil_div(vec ? cols / 4 : cols, 256);
  // ~1 K workgroups (each ends with ONE atomicMax on the single output word: a word takes ~90
  // atomics per us, so the round-4 8 K workgroups spent ~90 us of a 150 us pass on them); each
  // thread walks its column down rows 4 at a time, enough loads in flight for HBM rate
  const int64_t ry = std::max<int64_t>(1, std::min<int64_t>(ceil_div(rows, 4), ceil_div(1024, cx)));
  absmax_kernel<<<dim3((unsigned)cx, (unsigned)ry), 256, 0, st>>>(rows, cols, P, ld, vec, out);
  return check_launch("absmax_kernel");
}

int absmax_rows_launch(int64_t rows, int64_t cols, const float* P, int64_t ld, uint32_t* out,
                       bool accumulate, hipStream_t st) {
  if (rows <= 0) return MVML_OK;
  if (cols <= 0) {
    if (accumulate) return MVML_OK;
    if (hipMemsetAsync(out, 0, rows * sizeof(uint32_t), st) != hipSuccess) {
      set_error("absmax_rows: hipMemsetAsync failed");
      return MVML_ERR_LAUNCH;
    }
    return MVML_OK;
  }
  const int vec = (cols % 4 == 0) && (ld % 4 == 0) && ((uintptr_t)P % 16 == 0);
  const int64_t units = vec ? cols / 4 : cols;
  int lg = 0;
  while ((1 << lg) < units && lg < 6) ++lg;  // lanes per row: enough for one unit each, <= 64
  const int64_t per_block = 256 >> lg;
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(rows, per_block), 16384));
  absmax_rows_kernel<<<blocks, 256, 0, st>>>(rows, cols, P, ld, vec, lg, accumulate ? 1 : 0, out);
  return check_launch("absmax_rows_kernel");
}

int colsum_splits(int64_t M, int64_t N) {
  const int64_t colblocks = ceil_div(N, 256);
  int64_t s = ceil_div(2048, colblocks);
  s = std::min<int64_t>(s, ceil_div(M, 64));
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, 4096));
}

// ---- small-K split-fp16 product: the layer-1 projection as the memory kernel it is ---------
// C[M][N] = A[M][K] B[N][K]^T for K <= 96 (the atom features: K = 76 against the 1544 rows of
// layer 1's Wcat) writes N / K ~ 20 output bytes per input byte: HBM-bound on the C stores, and
// the 256x256 tile (five 16-deep stages, then an LDS epilogue that cannot overlap the next
// tile's loads) reached 0.34 of HBM on it.  Here a WAVE owns 64 output columns: it loads the
// split-fp16 planes of its 64 B rows into registers ONCE (B's il4 image, or fp32 split in place
// -- bitwise the same planes), then walks chunk_blocks blocks of 16 A rows: A's fragments come
// straight from global memory (the next block's in flight behind the current block's MFMAs),
// are split with the row's own scale (split2h, as the tiles do) and multiplied as C^T = B A^T
// on v_mfma_f32_16x16x32_f16 (K <= 16: 16x16x16) — transposed so that each lane's four
// accumulators are FOUR CONSECUTIVE COLUMNS OF ONE ROW; a wave-private LDS slice turns the
// 16 x 64 block into 4-row x 256-B float4 stores (measured: float4 stores straight from the
// accumulators, 16 rows x 64 B per instruction, ran at the tile's 2.7 TB/s), no block barrier.  The
// three products per k-step keep the tiles' order (l_b h_a, h_b l_a, h_b h_a); the scales are
// undone as there (B's, then the row's).  Waves are numbered XCD-major (xcd_block), slab
// fastest: the ~25 waves sharing a block of A rows run together on one XCD and read the rows
// from its L2.  Same values as the tiles to fp32-GEMM accuracy (the MFMA shape changes the
// summation order, so not bitwise).
constexpr int kSkMaxK = 96;

// KS16 = ceil(K / 16): KS16 / 2 steps of 16x16x32 and, for odd KS16, a 16-deep tail on
// 16x16x16, each zero-padded past K.  The tail accumulates into its OWN registers, added once at
// the end: behind 16x16x32 steps on the same accumulators it came out wrong in the first two of
// each lane's four results (K = 76 / 80, a missing MFMA-to-MFMA wait between the two pass
// counts).  Skipping the 16 padding k of a 96-deep plan saves 1/6 of the MFMA time at K = 76.
// A rows with an all-zero low plane (fp16-exact values: layer 1's 0/1 atom features) skip the
// h_b l_a products — per 16-row block, wave-uniform (a ballot); adding exact zeros is all they
// would do.
// ABL (timing ablations, option smallk 5 / 6; wrong results): 1 = no MFMAs, 2 = no C stores
// WL (default): the workgroup's four waves share ONE 64-column slab (four consecutive row
// chunks) and its B planes live in LDS (filled once, one group per wave), read per block as
// fragments — no B registers (162 VGPRs instead of 230), so three waves fit per SIMD and the
// store stream overlaps more matrix work: 3.26 -> 2.75 ms at config 3 on one box.  WL = false
// (B fragments in registers, every wave its own slab) stays as option smallk 10.
template <int KS16, bool IL4, bool NT, int ABL = 0, int NG = 4, bool WL = false>
__global__ void __launch_bounds__(256, WL ? 3 : 2)  // two (three) waves per SIMD
gemm_smallk_kernel(int64_t M, int64_t N, int K, const float* __restrict__ A, int64_t lda,
                   const float* __restrict__ B, int64_t ldb, const uint32_t* __restrict__ a_rows,
                   const uint32_t* __restrict__ amax_b, const float* __restrict__ bias, int act,
                   float* __restrict__ C, int64_t ldc, int n_slabs, int chunk_blocks) {
  constexpr int N32 = KS16 / 2, T16 = KS16 % 2, NW = N32 > 0 ? N32 : 1;
  constexpr int NX = 2 * N32 + T16;  // A float4 per lane and row block
  constexpr int SW = 16 * NG, PITCH = SW + 4;  // slab width (columns per wave); LDS row pitch
  const int lane = threadIdx.x & 63, li = lane & 15, lq = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t lb = xcd_block(blockIdx.x, gridDim.x);
  const int64_t w = lb * 4 + wid;
  const int slab = (int)(WL ? lb % n_slabs : w % n_slabs);
  const int64_t nrb = (M + 15) >> 4;
  const int64_t rb0 = (WL ? (lb / n_slabs) * 4 + wid : w / n_slabs) * chunk_blocks;
  if (!WL && rb0 >= nrb) return;
  const int64_t rb1 = min(nrb, rb0 + (int64_t)chunk_blocks);
  const int kb = amax_shift(*amax_b);
  const float s_b = pow2f(kb), u_b = pow2f(-kb);
  // this lane's B rows (output columns c0 + 16 g + li) for the MFMA's A side: k = 32 s + 8 lq
  // + 0..7 (x32 steps), 32 N32 + 4 lq + 0..3 (x16 tail); k >= K reads as zero
  constexpr int RG = WL ? 1 : NG;  // register copies of the B fragments (WL: none)
  f16x8 bh[RG][NW], bl[RG][NW];
  f16x4 th[RG], tl[RG];
  __shared__ u32x4 s_wh[WL ? NG : 1][WL ? NW : 1][WL ? 64 : 1], s_wl[WL ? NG : 1][WL ? NW : 1][WL ? 64 : 1];
  __shared__ uint2 s_th[WL ? NG : 1][WL ? 64 : 1], s_tl[WL ? NG : 1][WL ? 64 : 1];
  auto piece = [&](const float* row, int k, uint2& h, uint2& l) {  // B[row][k .. k + 3] as planes
    const float4 v = *reinterpret_cast<const float4*>(row + min(k, K - 4));
    if constexpr (IL4) {
      h = make_uint2(__float_as_uint(v.x), __float_as_uint(v.y));
      l = make_uint2(__float_as_uint(v.z), __float_as_uint(v.w));
    } else {
      split2h(v, s_b, h, l);
    }
    if (k >= K) h = l = make_uint2(0u, 0u);
  };
  if constexpr (WL) {  // wave wid fills group wid's planes (NG == 4 waves), then one barrier
    static_assert(NG == 4, "one group per wave");
    const int g = wid;
    const int64_t col = (int64_t)slab * SW + 16 * g + li;
    const float* row = B + min(col, N - 1) * ldb;
#pragma unroll
    for (int s = 0; s < N32; ++s) {
      uint2 h0, l0, h1, l1;
      piece(row, 32 * s + 8 * lq, h0, l0);
      piece(row, 32 * s + 8 * lq + 4, h1, l1);
      s_wh[g][s][lane] = u32x4{h0.x, h0.y, h1.x, h1.y};
      s_wl[g][s][lane] = u32x4{l0.x, l0.y, l1.x, l1.y};
    }
    if constexpr (T16) {
      uint2 h, l;
      piece(row, 32 * N32 + 4 * lq, h, l);
      s_th[g][lane] = h;
      s_tl[g][lane] = l;
    }
    __syncthreads();
    if (rb0 >= nrb) return;
  } else {
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int64_t col = (int64_t)slab * SW + 16 * g + li;
    const float* row = B + min(col, N - 1) * ldb;
#pragma unroll
    for (int s = 0; s < N32; ++s) {
      uint2 h0, l0, h1, l1;
      piece(row, 32 * s + 8 * lq, h0, l0);
      piece(row, 32 * s + 8 * lq + 4, h1, l1);
      const u32x4 hv = {h0.x, h0.y, h1.x, h1.y}, lv = {l0.x, l0.y, l1.x, l1.y};
      bh[g][s] = __builtin_bit_cast(f16x8, hv);
      bl[g][s] = __builtin_bit_cast(f16x8, lv);
    }
    if constexpr (T16) {
      uint2 h, l;
      piece(row, 32 * N32 + 4 * lq, h, l);
      th[g] = __builtin_bit_cast(f16x4, h);
      tl[g] = __builtin_bit_cast(f16x4, l);
    }
  }
  }
  // the B fragments of group g (registers, or the LDS image)
  auto fbh = [&](int g, int s) -> f16x8 {
    if constexpr (WL) return __builtin_bit_cast(f16x8, s_wh[g][s][lane]); else return bh[g][s];
  };
  auto fbl = [&](int g, int s) -> f16x8 {
    if constexpr (WL) return __builtin_bit_cast(f16x8, s_wl[g][s][lane]); else return bl[g][s];
  };
  auto fth = [&](int g) -> f16x4 {
    if constexpr (WL) return __builtin_bit_cast(f16x4, s_th[g][lane]); else return th[g];
  };
  auto ftl = [&](int g) -> f16x4 {
    if constexpr (WL) return __builtin_bit_cast(f16x4, s_tl[g][lane]); else return tl[g];
  };
  float bv[NG][4];
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t col = (int64_t)slab * SW + 16 * g + 4 * lq + u;
      bv[g][u] = (bias && col < N) ? bias[col] : 0.f;
    }
  // A fragments of one 16-row block: row 16 rb + li, k as B's; KS16 float4 per lane
  auto load_a = [&](int64_t rb, float4 (&x)[NX], uint32_t& rbits) {
    const int64_t r = min(rb * 16 + li, M - 1);
    const float* p = A + r * lda;
#pragma unroll
    for (int s = 0; s < N32; ++s) {
      x[2 * s] = *reinterpret_cast<const float4*>(p + min(32 * s + 8 * lq, K - 4));
      x[2 * s + 1] = *reinterpret_cast<const float4*>(p + min(32 * s + 8 * lq + 4, K - 4));
    }
    if constexpr (T16) x[NX - 1] = *reinterpret_cast<const float4*>(p + min(32 * N32 + 4 * lq, K - 4));
    rbits = a_rows[r];
  };
  __shared__ __attribute__((aligned(16))) float s_c[4][16 * PITCH];
  float* wl = s_c[threadIdx.x >> 6];
  // two register sets, prefetch distance 2: a block's A rows are requested two blocks before
  // they are split (the first of the ~25 waves reading a row block pays the HBM miss)
  auto block = [&](int64_t rb, float4 (&xn)[NX], uint32_t& rn) {
    float4 x[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) x[i] = xn[i];
    const int ka = amax_shift(rn);
    if (rb + 2 < rb1) load_a(rb + 2, xn, rn);
    const float s_a = pow2f(ka);
    f16x8 ah[NW], al[NW];
    f16x4 ath, atl;
#pragma unroll
    for (int s = 0; s < N32; ++s) {
      uint2 h0, l0, h1, l1;
      split2h(x[2 * s], s_a, h0, l0);
      split2h(x[2 * s + 1], s_a, h1, l1);
      if (32 * s + 8 * lq >= K) h0 = l0 = make_uint2(0u, 0u);
      if (32 * s + 8 * lq + 4 >= K) h1 = l1 = make_uint2(0u, 0u);
      const u32x4 hv = {h0.x, h0.y, h1.x, h1.y}, lv = {l0.x, l0.y, l1.x, l1.y};
      ah[s] = __builtin_bit_cast(f16x8, hv);
      al[s] = __builtin_bit_cast(f16x8, lv);
    }
    if constexpr (T16) {
      uint2 h, l;
      split2h(x[NX - 1], s_a, h, l);
      if (32 * N32 + 4 * lq >= K) h = l = make_uint2(0u, 0u);
      ath = __builtin_bit_cast(f16x4, h);
      atl = __builtin_bit_cast(f16x4, l);
    }
    // any non-zero word in the block's A low plane (wave-uniform)
    uint32_t lo_bits = 0;
#pragma unroll
    for (int s = 0; s < N32; ++s) {
      const u32x4 q = __builtin_bit_cast(u32x4, al[s]);
      lo_bits |= q[0] | q[1] | q[2] | q[3];
    }
    if constexpr (T16) {
      const uint2 q = __builtin_bit_cast(uint2, atl);
      lo_bits |= q.x | q.y;
    }
    const bool a_lo = __ballot(lo_bits != 0) != 0;
    f32x4 acc[NG];
    auto products = [&](auto ALO) {
      constexpr bool kLo = decltype(ALO)::value;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (ABL == 1) {
#pragma unroll
          for (int s = 0; s < N32; ++s) {
            acc[g][0] += (float)ah[s][g] * (float)fbh(g, s)[0];
            acc[g][1] += (float)al[s][g] * (float)fbl(g, s)[1];
          }
          continue;
        }
#pragma unroll
        for (int s = 0; s < N32; ++s) {
          const f16x8 bhv = fbh(g, s), blv = fbl(g, s);
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(blv, ah[s], acc[g], 0, 0, 0);
          if constexpr (kLo) acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bhv, al[s], acc[g], 0, 0, 0);
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bhv, ah[s], acc[g], 0, 0, 0);
        }
      }
      if constexpr (T16 && ABL != 1) {
        f32x4 tac[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          tac[g] = f32x4{0.f, 0.f, 0.f, 0.f};
          const f16x4 thv = fth(g), tlv = ftl(g);
          tac[g] = __builtin_amdgcn_mfma_f32_16x16x16f16(tlv, ath, tac[g], 0, 0, 0);
          if constexpr (kLo) tac[g] = __builtin_amdgcn_mfma_f32_16x16x16f16(thv, atl, tac[g], 0, 0, 0);
          tac[g] = __builtin_amdgcn_mfma_f32_16x16x16f16(thv, ath, tac[g], 0, 0, 0);
        }
#pragma unroll
        for (int g = 0; g < NG; ++g) acc[g] = N32 > 0 ? acc[g] + tac[g] : tac[g];
      }
    };
    if (a_lo)
      products(std::true_type{});
    else
      products(std::false_type{});
    // the 16 x 64 block leaves through the wave's LDS slice: each lane's 4 x float4 (row li,
    // columns 16 g + 4 lq) in, then 4 rows x 256 contiguous bytes per store instruction out
    // (straight from the accumulators a store instruction would write 16 rows x 64 B)
    const float u_a = pow2f(-ka);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      float4 o;
      o.x = acc[g][0] * u_b * u_a + bv[g][0];
      o.y = acc[g][1] * u_b * u_a + bv[g][1];
      o.z = acc[g][2] * u_b * u_a + bv[g][2];
      o.w = acc[g][3] * u_b * u_a + bv[g][3];
      if (act == 1) {
        o.x = fmaxf(o.x, 0.f); o.y = fmaxf(o.y, 0.f); o.z = fmaxf(o.z, 0.f); o.w = fmaxf(o.w, 0.f);
      }
      *reinterpret_cast<float4*>(wl + li * PITCH + 16 * g + 4 * lq) = o;
    }
    wave_sync_lds();
#pragma unroll
    for (int t = 0; t < NG; ++t) {  // 64 / (4 NG) rows of SW floats per store instruction
      const int rr = (16 / NG) * t + lane / (4 * NG), c4 = 4 * (lane % (4 * NG));
      const float4 o = *reinterpret_cast<const float4*>(wl + rr * PITCH + c4);
      const int64_t row = rb * 16 + rr, col = (int64_t)slab * SW + c4;
      if (row < M && col < N && (ABL != 2 || __float_as_uint(o.x) == 0x7fc00123u)) {
        if constexpr (NT) {
          const f32x4 ov = {o.x, o.y, o.z, o.w};
          __builtin_nontemporal_store(ov, reinterpret_cast<f32x4*>(C + row * ldc + col));
        } else {
          *reinterpret_cast<float4*>(C + row * ldc + col) = o;
        }
      }
    }
    wave_sync_lds();  // the reads are done before the next block's writes
  };
  float4 xa[NX], xb[NX];
  uint32_t ra = 0, rbits = 0;
  load_a(rb0, xa, ra);
  if (rb0 + 1 < rb1) load_a(rb0 + 1, xb, rbits);
  // (measured: issuing block rb + 1's MFMAs before block rb's epilogue, two accumulator sets,
  // was ~5 % slower relative to the tile on the same box)
  for (int64_t rb = rb0; rb < rb1; rb += 2) {
    block(rb, xa, ra);
    if (rb + 1 < rb1) block(rb + 1, xb, rbits);
  }
}

// Host: the shapes the small-K kernel takes (per-row A scales, K-contiguous B, K <= 96, every
// row and pointer 16-B aligned, N % 4 == 0, no beta, act 0 / 1).
bool smallk_fits(int b_kmajor, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                 const float* Bp, int64_t ldb, float beta, int act, const float* C, int64_t ldc) {
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return option(MVML_OPT_SMALLK) != 0 && !b_kmajor && M > 0 && K >= 4 && K <= kSkMaxK && K % 4 == 0 &&
         N % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && ldc % 4 == 0 && al(A) && al(Bp) && al(C) &&
         beta == 0.f && (act == 0 || act == 1);
}

int smallk_launch(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const float* B,
                  int64_t ldb, bool il4, const uint32_t* a_rows, const uint32_t* amax_b,
                  const float* bias, int act, float* C, int64_t ldc, hipStream_t st) {
  // 64 columns per wave (NG = 4).  Measured: 32-column slabs (NG = 2, 152 VGPRs, three waves
  // per SIMD) 3.38 vs 2.87 ms at config 3 — twice the A reads cost more than the occupancy buys
  const int n_slabs = (int)ceil_div(N, 64);
  const int64_t nrb = ceil_div(M, 16);
  // ~32 row blocks (512 rows) per wave: the B slab's one load is 1/30 of what the wave stores;
  // fewer on small launches so that >= 4096 waves fill the chip
  const int sko = option(MVML_OPT_SMALLK);
  const int64_t cap = sko == 3 ? 8 : (sko == 4 ? 128 : 32);  // (3 / 4: chunk-size variants)
  const int64_t cb = std::max<int64_t>(1, std::min<int64_t>(cap, nrb * n_slabs / 4096));
  const int64_t waves = ceil_div(nrb, cb) * n_slabs;
  const int64_t blocks = ceil_div(waves, 4);
  if (blocks >= (int64_t(1) << 31)) {
    set_error("gemm small-K: too many blocks");
    return MVML_ERR_INVALID;
  }
  const bool nt = option(MVML_OPT_SMALLK) != 2;  // (3 .. 6: timing variants)
  const int ks = (int)ceil_div(K, 16);  // 1 .. 6: the k-step plans above
  // WL: a workgroup = four row chunks of one slab
  const int64_t wl_blocks = ceil_div(ceil_div(nrb, cb), 4) * n_slabs;
#define MVML_SK(KS, IL, NTV)                                                                      \
  gemm_smallk_kernel<KS, IL, NTV, 0, 4, true><<<(unsigned)wl_blocks, 256, 0, st>>>(              \
      M, N, (int)K, A, lda, B, ldb, a_rows, amax_b, bias, act, C, ldc, n_slabs, (int)cb)
#define MVML_SK_KS(IL, NTV)                 \
  switch (ks) {                             \
    case 1: MVML_SK(1, IL, NTV); break;     \
    case 2: MVML_SK(2, IL, NTV); break;     \
    case 3: MVML_SK(3, IL, NTV); break;     \
    case 4: MVML_SK(4, IL, NTV); break;     \
    case 5: MVML_SK(5, IL, NTV); break;     \
    default: MVML_SK(6, IL, NTV); break;    \
  }
  const int opt = option(MVML_OPT_SMALLK);
  if (opt == 10 && ks == 5 && il4) {  // (10: B fragments in registers — the round-5 first build)
    gemm_smallk_kernel<5, true, true, 0, 4, false><<<(unsigned)blocks, 256, 0, st>>>(
        M, N, (int)K, A, lda, B, ldb, a_rows, amax_b, bias, act, C, ldc, n_slabs, (int)cb);
    return check_launch("gemm_smallk_kernel(B in registers)");
  }
  if ((opt == 5 || opt == 6) && ks == 5 && il4) {
    if (opt == 5)
      gemm_smallk_kernel<5, true, true, 1, 4, true><<<(unsigned)wl_blocks, 256, 0, st>>>(
          M, N, (int)K, A, lda, B, ldb, a_rows, amax_b, bias, act, C, ldc, n_slabs, (int)cb);
    else
      gemm_smallk_kernel<5, true, true, 2, 4, true><<<(unsigned)wl_blocks, 256, 0, st>>>(
          M, N, (int)K, A, lda, B, ldb, a_rows, amax_b, bias, act, C, ldc, n_slabs, (int)cb);
    return check_launch("gemm_smallk_kernel(ablation)");
  }
  if (il4) {
    if (nt) { MVML_SK_KS(true, true) } else { MVML_SK_KS(true, false) }
  } else {
    if (nt) { MVML_SK_KS(false, true) } else { MVML_SK_KS(false, false) }
  }
#undef MVML_SK_KS
#undef MVML_SK
  return check_launch("gemm_smallk_kernel");
}

}  // namespace
}  // namespace mvml

using namespace mvml;

// Workspace: [256 B: the split-fp16 operand maxima | split-K slab (S M N floats)].
constexpr size_t kAmaxBytes = 256;
extern "C" size_t mvml_gemm_workspace_size(int64_t M, int64_t N, int64_t K) {
  const int S = choose_splits(M, N, K);
  return kAmaxBytes + (S > 1 ? carve_size((size_t)S * M * N * sizeof(float)) : 0);
}

namespace {
int gemm_launch(int prec, int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias,
                float beta, int act, float* C, int64_t ldc, void* workspace,
                size_t workspace_bytes, void* stream, int64_t batch = 1,
                BatchStrides bst = BatchStrides{}, AmaxPtrs amax = AmaxPtrs{},
                const uint16_t* bps = nullptr);
}

extern "C" int mvml_gemm_f32(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                             const float* A, int64_t lda, const float* B, int64_t ldb,
                             const float* bias, float beta, int act, float* C, int64_t ldc,
                             void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  return gemm_launch(kPrecF32, a_kmajor, b_kmajor, M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc,
                     workspace, workspace_bytes, stream);
}

extern "C" int mvml_gemm_f32x3(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                               const float* A, int64_t lda, const float* B, int64_t ldb,
                               const float* bias, float beta, int act, float* C, int64_t ldc,
                               void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  return gemm_launch(kPrecX3, a_kmajor, b_kmajor, M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc,
                     workspace, workspace_bytes, stream);
}

extern "C" int mvml_gemm_f16x2(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                               const float* A, int64_t lda, const float* B, int64_t ldb,
                               const float* bias, float beta, int act, float* C, int64_t ldc,
                               void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  return gemm_launch(kPrecF16x2, a_kmajor, b_kmajor, M, N, K, A, lda, B, ldb, bias, beta, act, C,
                     ldc, workspace, workspace_bytes, stream);
}

extern "C" int mvml_gemm_f16x2_amax(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                                    const float* A, int64_t lda, const float* B, int64_t ldb,
                                    const uint32_t* amax_a, const uint32_t* amax_b,
                                    const float* bias, float beta, int act,
                                    float* C, int64_t ldc, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  clear_error();
  MVML_REQUIRE(amax_a != nullptr && amax_b != nullptr, "gemm_f16x2_amax: amax_a / amax_b are required");
  return gemm_launch(kPrecF16x2, a_kmajor, b_kmajor, M, N, K, A, lda, B, ldb, bias, beta, act, C,
                     ldc, workspace, workspace_bytes, stream, 1, BatchStrides{},
                     AmaxPtrs{amax_a, amax_b});
}

extern "C" int mvml_gemm_f16x2_rows(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                                    const float* B, int64_t ldb, int b_kmajor, const float* b_il4,
                                    const uint32_t* amax_a_rows, const uint32_t* amax_b,
                                    const float* bias, float beta, int act, float* C, int64_t ldc,
                                    void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  MVML_REQUIRE(amax_a_rows != nullptr && amax_b != nullptr,
               "gemm_f16x2_rows: amax_a_rows / amax_b are required");
  MVML_REQUIRE(!b_il4 || ((uintptr_t)b_il4 % 16) == 0, "gemm_f16x2_rows: b_il4 must be 16-B aligned");
  MVML_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm_f16x2_rows: negative shape");
  if (M == 0 || N == 0) return MVML_OK;
  // small K (layer 1: the atom features): the wave-per-64-columns memory kernel
  if (smallk_fits(b_kmajor, M, N, K, A, lda, b_il4 ? b_il4 : B, ldb, beta, act, C, ldc) && ldc >= N &&
      lda >= K && ldb >= K)
    return smallk_launch(M, N, K, A, lda, b_il4 ? b_il4 : B, ldb, b_il4 != nullptr, amax_a_rows, amax_b,
                         bias, act, C, ldc, as_stream(stream));
  AmaxPtrs am;
  am.b = amax_b;
  am.a_rows = amax_a_rows;
  return gemm_launch(kPrecF16x2, 0, b_kmajor, M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc,
                     workspace, workspace_bytes, stream, 1, BatchStrides{}, am,
                     reinterpret_cast<const uint16_t*>(b_il4));
}

extern "C" int mvml_gemm_rows_smallk(int b_kmajor, int64_t M, int64_t N, int64_t K, const float* A,
                                     int64_t lda, const float* B, int64_t ldb, float beta, int act,
                                     const float* C, int64_t ldc) {
  return smallk_fits(b_kmajor, M, N, K, A, lda, B, ldb, beta, act, C, ldc) && ldc >= N && lda >= K &&
                 ldb >= K
             ? 1
             : 0;
}

extern "C" int mvml_gemm_f16x2_ex(int64_t M, int64_t N, int64_t K, int64_t batch, const float* A,
                                  int64_t lda, int64_t stride_a, const float* B, int64_t ldb,
                                  int b_kmajor, const float* b_il4, int64_t stride_b,
                                  const uint32_t* amax_a_rows, int64_t stride_rows,
                                  const uint32_t* amax_b, const float* bias, int64_t stride_bias,
                                  int act, float* C, int64_t ldc, int64_t stride_c, const float* aux,
                                  int64_t ld_aux, uint32_t* c_amax, uint32_t* c_rows,
                                  int64_t c_rows_stride, int c_rows_cols, int64_t stride_c_rows,
                                  void* stream) {
  clear_error();
  MVML_REQUIRE(M >= 0 && N >= 0 && K >= 0 && batch >= 1 && batch <= 65535, "gemm_f16x2_ex: bad shape");
  MVML_REQUIRE(amax_a_rows && amax_b, "gemm_f16x2_ex: amax_a_rows / amax_b are required");
  MVML_REQUIRE(act >= 0 && act <= 3 && (act != 3 || (aux && ld_aux >= N)), "gemm_f16x2_ex: bad act / aux");
  MVML_REQUIRE(c_rows_cols >= 0 && c_rows_cols % 64 == 0 && (!c_rows || c_rows_stride >= 0),
               "gemm_f16x2_ex: c_rows_cols must be a multiple of 64");
  MVML_REQUIRE(lda >= K && ldc >= N && (b_kmajor ? ldb >= N : ldb >= K), "gemm_f16x2_ex: bad leading dims");
  MVML_REQUIRE(stride_a >= 0 && stride_b >= 0 && stride_c >= 0 && stride_bias >= 0 && stride_rows >= 0 &&
                   stride_c_rows >= 0, "gemm_f16x2_ex: negative stride");
  if (M == 0 || N == 0) return MVML_OK;
  const float* Bp = b_il4 ? b_il4 : B;
  const int av = (lda % 4 == 0) && ((uintptr_t)A % 16 == 0) && stride_a % 4 == 0;
  const int bv = (ldb % 4 == 0) && ((uintptr_t)Bp % 16 == 0) && stride_b % 4 == 0;
  // the 256x256 tile at any size (K is a feature dimension here: no split-K)
  MVML_REQUIRE(x3w_fast(false, b_kmajor != 0, M, N, K, av, bv),
               "gemm_f16x2_ex: needs 16-B aligned rows and strides and K %% 4 == 0");
  const int64_t tiles = ceil_div(M, XBM) * ceil_div(N, XBN);
  MVML_REQUIRE(tiles < (int64_t(1) << 31), "gemm_f16x2_ex: too many tiles");
  const dim3 grid(x3w_grid_x(tiles, 1), 1, (unsigned)batch);
  const BatchStrides bst{stride_a, stride_b, stride_c};
  AmaxPtrs am;
  am.b = amax_b;
  am.a_rows = amax_a_rows;
  EpiX ex;
  ex.aux = aux; ex.ld_aux = ld_aux; ex.c_amax = c_amax; ex.c_rows = c_rows;
  ex.rows_stride = c_rows_stride; ex.rows_cols = c_rows_cols;
  ex.bias_z = stride_bias; ex.rows_z = stride_rows; ex.crows_z = stride_c_rows;
  hipStream_t st = as_stream(stream);
  const int64_t kc = K > 0 ? K : 1;
#define MVML_X3W_EX(BKV, BPSV)                                                                    \
  gemm_x3w_kernel<false, BKV, -1, true, 2, BPSV, true, true><<<grid, kXThreads, 0, st>>>(         \
      M, N, K, A, lda, Bp, ldb, bias, 0.f, act, C, ldc, kc, nullptr, av, bv, ProjEpi{}, bst,       \
      CellEpi{}, am, DualPtrs{}, ex)
  if (b_kmajor) {
    if (b_il4) MVML_X3W_EX(true, 2);
    else MVML_X3W_EX(true, 0);
  } else {
    if (b_il4) MVML_X3W_EX(false, 2);
    else MVML_X3W_EX(false, 0);
  }
#undef MVML_X3W_EX
  return check_launch("gemm_x3w_kernel(ex)");
}

extern "C" int mvml_gemm_f16x2_batched(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                                       int64_t batch, const float* A, int64_t lda, int64_t stride_a,
                                       const float* B, int64_t ldb, int64_t stride_b,
                                       const uint32_t* amax_a, const uint32_t* amax_b, float* C,
                                       int64_t ldc, int64_t stride_c, void* stream) {
  clear_error();
  MVML_REQUIRE(batch >= 2 && batch <= 65535 && stride_a >= 0 && stride_b >= 0 && stride_c >= 0,
               "gemm_f16x2_batched: bad batch / strides");
  MVML_REQUIRE(amax_a && amax_b, "gemm_f16x2_batched: amax_a / amax_b are required");
  return gemm_launch(kPrecF16x2, a_kmajor, b_kmajor, M, N, K, A, lda, B, ldb, nullptr, 0.f, 0, C, ldc,
                     nullptr, 0, stream, batch, BatchStrides{stride_a, stride_b, stride_c},
                     AmaxPtrs{amax_a, amax_b});
}

extern "C" int mvml_split_f16x2_il4(int64_t rows, int64_t cols, const float* P, int64_t ld,
                                    const uint32_t* amax, float* out, void* stream) {
  clear_error();
  MVML_REQUIRE(rows >= 0 && cols >= 0 && cols % 4 == 0 && ld % 4 == 0 && ld >= cols && amax &&
                   out && ((uintptr_t)P % 16) == 0 && ((uintptr_t)out % 16) == 0,
               "split_f16x2_il4: bad shape / alignment");
  if (rows == 0 || cols == 0) return MVML_OK;
  const int64_t total = rows * (cols / 4);
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(total, 256), 8192);
  split_f16x2_il4_kernel<<<blocks, 256, 0, as_stream(stream)>>>(rows, cols / 4, P, ld, amax, out);
  return check_launch("split_f16x2_il4_kernel");
}

extern "C" int mvml_absmax_rows_f32(int64_t rows, int64_t cols, const float* P, int64_t ld,
                                    uint32_t* out, int accumulate, void* stream) {
  clear_error();
  MVML_REQUIRE(rows >= 0 && cols >= 0 && (rows == 0 || ld >= cols) && out, "absmax_rows: bad shape");
  return absmax_rows_launch(rows, cols, P, ld, out, accumulate != 0, as_stream(stream));
}

extern "C" int mvml_gemm_f16x2_bsplit(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                                      const float* A, int64_t lda, const float* B, int64_t ldb,
                                      const uint16_t* b_planes, int64_t b_plane,
                                      const uint32_t* amax_a, const uint32_t* amax_b,
                                      const float* bias, float beta, int act, float* C,
                                      int64_t ldc, void* workspace, size_t workspace_bytes,
                                      void* stream) {
  clear_error();
  MVML_REQUIRE(amax_a && amax_b && b_planes && b_plane == 0 && ((uintptr_t)b_planes % 16) == 0,
               "gemm_f16x2_bsplit: maxima and B's planes are required");
  AmaxPtrs am{amax_a, amax_b, b_plane};
  return gemm_launch(kPrecF16x2, a_kmajor, b_kmajor, M, N, K, A, lda, B, ldb, bias, beta, act, C,
                     ldc, workspace, workspace_bytes, stream, 1, BatchStrides{}, am, b_planes);
}

extern "C" int mvml_absmax_f32(int64_t rows, int64_t cols, const float* P, int64_t ld,
                               uint32_t* out, int accumulate, void* stream) {
  clear_error();
  MVML_REQUIRE(rows >= 0 && cols >= 0 && (rows == 0 || ld >= cols) && out, "absmax: bad shape");
  return absmax_launch(rows, cols, P, ld, out, accumulate != 0, as_stream(stream));
}

extern "C" int mvml_gemm_f32x3_batched(int a_kmajor, int b_kmajor, int64_t M, int64_t N,
                                       int64_t K, int64_t batch, const float* A, int64_t lda,
                                       int64_t stride_a, const float* B, int64_t ldb,
                                       int64_t stride_b, const float* bias, float beta, int act,
                                       float* C, int64_t ldc, int64_t stride_c, void* stream) {
  clear_error();
  MVML_REQUIRE(batch >= 1 && batch <= 65535 && stride_a >= 0 && stride_b >= 0 && stride_c >= 0,
               "gemm_batched: bad batch / strides");
  return gemm_launch(kPrecX3, a_kmajor, b_kmajor, M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc,
                     nullptr, 0, stream, batch, BatchStrides{stride_a, stride_b, stride_c});
}

extern "C" int mvml_lstm_gates_cell_fwd(int64_t M, int D, int64_t K, const float* A, int64_t lda,
                                        const float* w_perm, int64_t ldw, const float* b_ih,
                                        const float* b_hh,
                                        const float* c_prev, float* c_out, float* h_out,
                                        int64_t ldh, float* act, float* h_out2, int64_t ldh2,
                                        const uint32_t* amax_a, const uint32_t* amax_b,
                                        const uint32_t* amax_a_rows,
                                        const uint16_t* w_planes, int64_t w_plane,
                                        void* stream) {
  clear_error();
  MVML_REQUIRE(M >= 0 && D > 0 && K > 0 && lda >= K && ldw >= K && ldh >= D &&
                   (!h_out2 || ldh2 >= D) && MVML_X3W_LDSEPI,
               "lstm_gates_cell_fwd: bad shape");
  MVML_REQUIRE(!amax_a_rows || amax_b, "lstm_gates_cell_fwd: per-row A maxima need max |w_perm|");
  if (amax_a_rows && !amax_a) amax_a = amax_a_rows;  // (unused: the rows' maxima replace it)
  if (M == 0) return MVML_OK;
  const int64_t N = 4 * (int64_t)D;
  const GemmPlan plan = plan_gemm(kPrecX3, M, N, K);
  const int av = (lda % 4 == 0) && ((uintptr_t)A % 16 == 0);
  const int bv = (ldw % 4 == 0) && ((uintptr_t)w_perm % 16 == 0);
  MVML_REQUIRE(plan.wide && plan.S == 1 && x3w_fast(false, false, M, N, K, av, bv),
               "lstm_gates_cell_fwd: needs the 256x256 plan without split-K and aligned rows "
               "(use mvml_gemm_f32x3 + mvml_lstm_cell_fwd)");
  const int64_t tiles = ceil_div(M, XBM) * ceil_div(N, XBN);
  CellEpi cep;
  cep.b_ih = b_ih; cep.b_hh = b_hh; cep.c_prev = c_prev; cep.c_out = c_out; cep.h_out = h_out;
  cep.h_out2 = h_out2; cep.act = act; cep.ldh = ldh; cep.ldh2 = ldh2; cep.D = D;
  const dim3 grid(x3w_grid_x(tiles, 1), 1, 1);
  MVML_REQUIRE(!amax_a == !amax_b, "lstm_gates_cell_fwd: give both maxima or neither");
  if (amax_a && option(MVML_OPT_LSTM_TILE) == 128 && K % BKT == 0) {
    // the 128x128 split-fp16 kernel with the same cell epilogue (the wide BiLSTM steps' plan)
    const int64_t t128 = ceil_div(M, BM) * ceil_div(N, BN);
    gemm_f32_kernel<false, false, -1, true, true><<<dim3((unsigned)t128, 1, 1), kThreads, 0, as_stream(stream)>>>(
        M, N, K, A, lda, w_perm, ldw, nullptr, 0.f, 0, nullptr, N, K, nullptr, av, bv, ProjEpi{},
        BatchStrides{}, AmaxPtrs{amax_a, amax_b, 0, amax_a_rows}, cep);
    return check_launch("gemm_f32_kernel(lstm cell)");
  }
  MVML_REQUIRE(!w_planes || w_plane == 0, "lstm_gates_cell_fwd: w_planes must be the il4 image (w_plane 0)");
  if (amax_a_rows && w_planes)  // per-row A, w_perm from its il4 image
    gemm_x3w_kernel<false, false, -1, true, 2, 2, true><<<grid, kXThreads, 0, as_stream(stream)>>>(
        M, N, K, A, lda, reinterpret_cast<const float*>(w_planes), ldw, nullptr, 0.f, 0, nullptr,
        N, K, nullptr, av, bv, ProjEpi{}, BatchStrides{}, cep, AmaxPtrs{amax_a, amax_b, 0, amax_a_rows});
  else if (amax_a_rows)  // a scale per A row (Set2Set: per molecule)
    gemm_x3w_kernel<false, false, -1, true, 2, 0, true><<<grid, kXThreads, 0, as_stream(stream)>>>(
        M, N, K, A, lda, w_perm, ldw, nullptr, 0.f, 0, nullptr, N, K, nullptr, av, bv, ProjEpi{},
        BatchStrides{}, cep, AmaxPtrs{amax_a, amax_b, 0, amax_a_rows});
  else if (amax_a)
    gemm_x3w_kernel<false, false, -1, true, 2><<<grid, kXThreads, 0, as_stream(stream)>>>(
        M, N, K, A, lda, w_perm, ldw, nullptr, 0.f, 0, nullptr, N, K, nullptr, av, bv, ProjEpi{},
        BatchStrides{}, cep, AmaxPtrs{amax_a, amax_b});
  else
    gemm_x3w_kernel<false, false, -1, true><<<grid, kXThreads, 0, as_stream(stream)>>>(
        M, N, K, A, lda, w_perm, ldw, nullptr, 0.f, 0, nullptr, N, K, nullptr, av, bv, ProjEpi{},
        BatchStrides{}, cep);
  return check_launch("gemm_x3w_kernel(lstm cell)");
}

extern "C" int mvml_lstm_gates_cell_plan_ok(int64_t M, int D, int64_t K) {
  const GemmPlan plan = plan_gemm(kPrecX3, M, 4 * (int64_t)D, K);
  return plan.wide && plan.S == 1 && K % 4 == 0;
}

extern "C" int mvml_gemm_bf16(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                              const float* A, int64_t lda, const float* B, int64_t ldb,
                              const float* bias, float beta, int act, float* C, int64_t ldc,
                              void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  return gemm_launch(kPrecBf16, a_kmajor, b_kmajor, M, N, K, A, lda, B, ldb, bias, beta, act, C,
                     ldc, workspace, workspace_bytes, stream);
}

namespace {
int gemm_launch(int prec, int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias,
                float beta, int act, float* C, int64_t ldc, void* workspace,
                size_t workspace_bytes, void* stream, int64_t batch, BatchStrides bst,
                AmaxPtrs amax, const uint16_t* bps) {
  MVML_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm: negative size");
  if (M == 0 || N == 0) return MVML_OK;
  MVML_REQUIRE(ldc >= N, "gemm: ldc < N");
  MVML_REQUIRE(a_kmajor ? lda >= M : lda >= K, "gemm: bad lda");
  MVML_REQUIRE(b_kmajor ? ldb >= N : ldb >= K, "gemm: bad ldb");
  MVML_REQUIRE(act == 0 || act == 1, "gemm: bad act");
  hipStream_t st = as_stream(stream);
  const bool hf = prec == kPrecF16x2;
  const bool x3 = prec == kPrecX3 || hf, bf = prec == kPrecBf16;
  GemmPlan plan = plan_gemm(prec, M, N, K);
  MVML_REQUIRE(!amax.a_rows || (hf && !a_kmajor && batch == 1 && amax.b),
               "gemm: per-row A maxima need split-fp16, a K-contiguous A, no batch and max |B|");
  if (hf && !amax.a && !amax.a_rows) {  // operand maxima into the workspace head, once per product
    if (!workspace || workspace_bytes < kAmaxBytes) {
      set_error("gemm: workspace too small (need %zu)", mvml_gemm_workspace_size(M, N, K));
      return MVML_ERR_WORKSPACE;
    }
    uint32_t* mx = static_cast<uint32_t*>(workspace);
    int rc = absmax_launch(a_kmajor ? K : M, a_kmajor ? M : K, A, lda, mx, false, st);
    if (!rc) rc = absmax_launch(b_kmajor ? K : N, b_kmajor ? N : K, B, ldb, mx + 1, false, st);
    if (rc) return rc;
    amax = AmaxPtrs{mx, mx + 1};
  }
  // N = 256 q + r with 0 < r <= 128 (384-column products: the fusion head's data / weight
  // gradients, the LSTM hh weight gradients): a last 256-wide tile column would be at least half
  // padding (so such products fell back to the 128x128 kernel entirely); instead the first
  // 256 q columns run on the 256x256 kernel and the last r on their own (narrow) plan — two
  // launches on the stream, one workspace reused in stream order.
  const bool nsplit_on = option(MVML_OPT_GEMM_NSPLIT) != 0;
  if (nsplit_on && x3 && batch == 1 && N > XBN && N % XBN != 0 && N % XBN <= XBN / 2 &&
      plan_gemm(prec, M, N / XBN * XBN, K).wide) {
    const int64_t N1 = N / XBN * XBN, N2 = N - N1;
    if (mvml_gemm_workspace_size(M, N1, K) <= workspace_bytes &&
        mvml_gemm_workspace_size(M, N2, K) <= workspace_bytes) {
      int rc = gemm_launch(prec, a_kmajor, b_kmajor, M, N1, K, A, lda, B, ldb, bias, beta, act, C,
                           ldc, workspace, workspace_bytes, stream, 1, BatchStrides{}, amax, bps);
      if (rc) return rc;
      const int64_t boff = b_kmajor ? N1 : N1 * ldb;
      return gemm_launch(prec, a_kmajor, b_kmajor, M, N2, K, A, lda, B + boff, ldb,
                         bias ? bias + N1 : nullptr, beta, act, C + N1, ldc, workspace,
                         workspace_bytes, stream, 1, BatchStrides{}, amax, bps ? bps + boff : nullptr);
    }
  }
  if (batch > 1) plan.S = 1;  // batched products are small: no split-K slab
  const int S = plan.S;
  float* slab = nullptr;
  if (S > 1) {
    if (workspace_bytes < mvml_gemm_workspace_size(M, N, K) || !workspace) {
      set_error("gemm: workspace too small (need %zu)", mvml_gemm_workspace_size(M, N, K));
      return MVML_ERR_WORKSPACE;
    }
    slab = reinterpret_cast<float*>(static_cast<uint8_t*>(workspace) + kAmaxBytes);
  }
  const int64_t kc = S > 1 ? k_chunk(K, S) : (K > 0 ? K : 1);
  const int64_t tiles = plan.wide ? ceil_div(M, XBM) * ceil_div(N, XBN) : ceil_div(M, BM) * ceil_div(N, BN);
  MVML_REQUIRE(tiles < (int64_t(1) << 31), "gemm: too many tiles");
  const int av = (lda % 4 == 0) && ((uintptr_t)A % 16 == 0) && bst.a % 4 == 0;
  const int bv = (ldb % 4 == 0) && ((uintptr_t)B % 16 == 0) && bst.b % 4 == 0;
  dim3 grid(plan.wide || bf ? x3w_grid_x(tiles, S) : (unsigned)tiles, (unsigned)S, (unsigned)batch);
  // B pre-split as an interleaved-by-4 image (bps with b_plane == 0, mvml_split_f16x2_il4) and /
  // or per-row A maxima, on the 256x256 tile (host: K-contiguous A)
  const bool il4 = bps && amax.b_plane == 0;
  const float* Bil = il4 ? reinterpret_cast<const float*>(bps) : B;
#define MVML_X3W_RB(BKV, BPSV, ROWSV)                                                            \
  gemm_x3w_kernel<false, BKV, -1, true, 2, BPSV, ROWSV><<<grid, kXThreads, 0, st>>>(             \
      M, N, K, A, lda, Bil, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst,       \
      CellEpi{}, amax)
  if ((amax.a_rows || il4) && plan.wide && !a_kmajor && batch == 1 &&
      x3w_fast(false, b_kmajor, M, N, K, av, bv)) {
    if (b_kmajor) {
      if (il4 && amax.a_rows) MVML_X3W_RB(true, 2, true);
      else if (il4) MVML_X3W_RB(true, 2, false);
      else MVML_X3W_RB(true, 0, true);
    } else {
      if (il4 && amax.a_rows) MVML_X3W_RB(false, 2, true);
      else if (il4) MVML_X3W_RB(false, 2, false);
      else MVML_X3W_RB(false, 0, true);
    }
  } else
#undef MVML_X3W_RB
  if (amax.a_rows && plan.wide) {  // per-row A maxima on the 256x256 tile (host: !a_kmajor)
    if (b_kmajor && x3w_fast(false, true, M, N, K, av, bv))
      gemm_x3w_kernel<false, true, -1, true, 2, 0, true><<<grid, kXThreads, 0, st>>>(
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst, CellEpi{}, amax);
    else if (b_kmajor)
      gemm_x3w_kernel<false, true, -1, false, 2, 0, true><<<grid, kXThreads, 0, st>>>(
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst, CellEpi{}, amax);
    else if (x3w_fast(false, false, M, N, K, av, bv))
      gemm_x3w_kernel<false, false, -1, true, 2, 0, true><<<grid, kXThreads, 0, st>>>(
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst, CellEpi{}, amax);
    else
      gemm_x3w_kernel<false, false, -1, false, 2, 0, true><<<grid, kXThreads, 0, st>>>(
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst, CellEpi{}, amax);
  } else
#define MVML_GEMM_LAUNCH(AKV, BKV)                                                              \
  do {                                                                                          \
    if (hf && plan.wide && x3w_fast(AKV, BKV, M, N, K, av, bv))                                 \
      gemm_x3w_kernel<AKV, BKV, -1, true, 2><<<grid, kXThreads, 0, st>>>(                       \
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst,   \
          CellEpi{}, amax);                                                                     \
    else if (hf && plan.wide)                                                                   \
      gemm_x3w_kernel<AKV, BKV, -1, false, 2><<<grid, kXThreads, 0, st>>>(                      \
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst,   \
          CellEpi{}, amax);                                                                     \
    else if (bf && x3w_fast(AKV, BKV, M, N, K, av, bv))                                         \
      gemm_x3w_kernel<AKV, BKV, -1, true, 1><<<grid, kXThreads, 0, st>>>(                       \
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst);  \
    else if (bf)                                                                                \
      gemm_x3w_kernel<AKV, BKV, -1, false, 1><<<grid, kXThreads, 0, st>>>(                      \
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst);  \
    else if (plan.wide && x3w_fast(AKV, BKV, M, N, K, av, bv))                                  \
      gemm_x3w_kernel<AKV, BKV, -1, true><<<grid, kXThreads, 0, st>>>(                          \
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst);  \
    else if (plan.wide)                                                                         \
      gemm_x3w_kernel<AKV, BKV, -1, false><<<grid, kXThreads, 0, st>>>(                         \
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst);  \
    else if (hf && AKV && BKV && amax.a_rowsum) /* + A's row sums (host: AKV) */               \
      gemm_f32_kernel<AKV, BKV, -1, true, true, false, AKV><<<grid, kThreads, 0, st>>>(         \
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst,   \
          amax);                                                                                \
    else if (hf && AKV && BKV) /* skinny, both k-major: split-fp16 fragment split */           \
      gemm_f32_kernel<AKV, BKV, -1, true, true><<<grid, kThreads, 0, st>>>(                     \
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst,   \
          amax);                                                                                \
    else if (x3 && AKV && BKV) /* both k-major: fragment split measured faster at 128x128 */    \
      gemm_f32_kernel<AKV, BKV, -1, true><<<grid, kThreads, 0, st>>>(                           \
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst);  \
    else if (hf) /* skinny: split-fp16 planes staged once per workgroup */                    \
      gemm_x3s_kernel<AKV, BKV, -1, true><<<grid, kThreads, 0, st>>>(                           \
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst,   \
          amax);                                                                                \
    else if (x3)                                                                                \
      gemm_x3s_kernel<AKV, BKV><<<grid, kThreads, 0, st>>>(                                     \
          M, N, K, A, lda, B, ldb, bias, beta, act, C, ldc, kc, slab, av, bv, ProjEpi{}, bst);  \
    else                                                                                        \
      gemm_f32_kernel<AKV, BKV><<<grid, kThreads, 0, st>>>(M, N, K, A, lda, B, ldb, bias, beta, \
                                                           act, C, ldc, kc, slab, av, bv,       \
                                                           ProjEpi{}, bst);                     \
  } while (0)
  if (!a_kmajor && !b_kmajor) MVML_GEMM_LAUNCH(false, false);
  else if (!a_kmajor && b_kmajor) MVML_GEMM_LAUNCH(false, true);
  else if (a_kmajor && !b_kmajor) MVML_GEMM_LAUNCH(true, false);
  else MVML_GEMM_LAUNCH(true, true);
#undef MVML_GEMM_LAUNCH
  int rc = check_launch("gemm_f32_kernel");
  if (rc) return rc;
  if (S > 1) {
    const int64_t total = M * N;
    const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(total, 256), 4096);
    splitk_reduce_kernel<<<blocks, 256, 0, st>>>(M, N, S, slab, bias, beta, act, C, ldc);
    rc = check_launch("splitk_reduce_kernel");
  }
  return rc;
}
}  // namespace

namespace mvml {
// Projection GEMM with the logits-partial epilogue: C[M,N] = A[M,K] B[N,K]^T (both
// K-contiguous, no split-K: K is the small feature dimension), part as in ProjEpi.
int gemm_proj_epi(int prec, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                  const float* B, int64_t ldb, float* C, int64_t ldc, const float* vec, int cols,
                  int logw, float* part, uint32_t* amax_ws, const uint32_t* amax_x,
                  const uint32_t* amax_w, const uint16_t* w_planes, int64_t w_plane,
                  hipStream_t st) {
  const bool hf = prec == kPrecF16x2;
  const bool x3 = prec == kPrecX3 || hf, bf = prec == kPrecBf16;
  const bool wide = bf || (x3 && plan_gemm(kPrecX3, M, N, K).wide);
  AmaxPtrs amx{amax_x, amax_w, w_plane};
  MVML_REQUIRE(!w_planes, "gat_proj_fwd: w_planes must be NULL (the two-plane weight image was removed)");
  if (hf && wide && !(amax_x && amax_w)) {  // maxima not supplied: one pass per operand
    MVML_REQUIRE(amax_ws != nullptr, "gat_proj_fwd: split-fp16 needs the maxima workspace");
    int rc = absmax_launch(M, K, A, lda, amax_ws, false, st);
    if (!rc) rc = absmax_launch(N, K, B, ldb, amax_ws + 1, false, st);
    if (rc) return rc;
    amx = AmaxPtrs{amax_ws, amax_ws + 1};
  }
  const int64_t tiles = wide ? ceil_div(M, XBM) * ceil_div(N, XBN) : ceil_div(M, BM) * ceil_div(N, BN);
  MVML_REQUIRE(tiles < (int64_t(1) << 31), "gat_proj_fwd: too many tiles");
  MVML_REQUIRE(cols <= N && (logw >= 2 && logw <= 5), "gat_proj_fwd: bad partial width");
  const int av = (lda % 4 == 0) && ((uintptr_t)A % 16 == 0);
  const int bv = (ldb % 4 == 0) && ((uintptr_t)B % 16 == 0);
  dim3 grid(wide ? x3w_grid_x(tiles, 1) : (unsigned)tiles, 1);
#define MVML_PROJ(LW)                                                                          \
  do {                                                                                         \
    if (hf && wide && x3w_fast(false, false, M, N, K, av, bv))                                 \
      gemm_x3w_kernel<false, false, LW, true, 2><<<grid, kXThreads, 0, st>>>(                  \
          M, N, K, A, lda, B, ldb, nullptr, 0.f, 0, C, ldc, K > 0 ? K : 1, nullptr, av, bv,    \
          ProjEpi{vec, cols, part}, BatchStrides{}, CellEpi{}, amx);                       \
    else if (hf && wide)                                                                       \
      gemm_x3w_kernel<false, false, LW, false, 2><<<grid, kXThreads, 0, st>>>(                 \
          M, N, K, A, lda, B, ldb, nullptr, 0.f, 0, C, ldc, K > 0 ? K : 1, nullptr, av, bv,    \
          ProjEpi{vec, cols, part}, BatchStrides{}, CellEpi{}, amx);                       \
    else if (bf && x3w_fast(false, false, M, N, K, av, bv))                                    \
      gemm_x3w_kernel<false, false, LW, true, 1><<<grid, kXThreads, 0, st>>>(                  \
          M, N, K, A, lda, B, ldb, nullptr, 0.f, 0, C, ldc, K > 0 ? K : 1, nullptr, av, bv,    \
          ProjEpi{vec, cols, part});                                                           \
    else if (bf)                                                                               \
      gemm_x3w_kernel<false, false, LW, false, 1><<<grid, kXThreads, 0, st>>>(                 \
          M, N, K, A, lda, B, ldb, nullptr, 0.f, 0, C, ldc, K > 0 ? K : 1, nullptr, av, bv,    \
          ProjEpi{vec, cols, part});                                                           \
    else if (wide && x3w_fast(false, false, M, N, K, av, bv))                                  \
      gemm_x3w_kernel<false, false, LW, true><<<grid, kXThreads, 0, st>>>(                     \
          M, N, K, A, lda, B, ldb, nullptr, 0.f, 0, C, ldc, K > 0 ? K : 1, nullptr, av, bv,    \
          ProjEpi{vec, cols, part});                                                           \
    else if (wide)                                                                             \
      gemm_x3w_kernel<false, false, LW, false><<<grid, kXThreads, 0, st>>>(                    \
          M, N, K, A, lda, B, ldb, nullptr, 0.f, 0, C, ldc, K > 0 ? K : 1, nullptr, av, bv,    \
          ProjEpi{vec, cols, part});                                                           \
    else if (x3)                                                                               \
      gemm_x3s_kernel<false, false, LW><<<grid, kThreads, 0, st>>>(                            \
          M, N, K, A, lda, B, ldb, nullptr, 0.f, 0, C, ldc, K > 0 ? K : 1, nullptr, av, bv,    \
          ProjEpi{vec, cols, part});                                                           \
    else                                                                                       \
      gemm_f32_kernel<false, false, LW><<<grid, kThreads, 0, st>>>(                            \
          M, N, K, A, lda, B, ldb, nullptr, 0.f, 0, C, ldc, K > 0 ? K : 1, nullptr, av, bv,    \
          ProjEpi{vec, cols, part});                                                           \
  } while (0)
  switch (logw) {
    case 5: MVML_PROJ(5); break;
    case 4: MVML_PROJ(4); break;
    case 3: MVML_PROJ(3); break;
    default: MVML_PROJ(2); break;
  }
#undef MVML_PROJ
  return check_launch("gemm_f32_kernel(proj)");
}
}  // namespace mvml

extern "C" size_t mvml_colsum_workspace_size(int64_t M, int64_t N) {
  return carve_size((size_t)colsum_splits(M, N) * N * sizeof(float));
}

extern "C" int mvml_colsum_f32(int64_t M, int64_t N, const float* X, int64_t ldx, float alpha,
                               float beta, float* out, void* workspace, size_t workspace_bytes,
                               void* stream) {
  clear_error();
  MVML_REQUIRE(M >= 0 && N >= 0 && ldx >= N, "colsum: bad shape");
  if (N == 0) return MVML_OK;
  if (workspace_bytes < mvml_colsum_workspace_size(M, N) || !workspace) {
    set_error("colsum: workspace too small");
    return MVML_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const int S = colsum_splits(M, N);
  const int64_t rows_per = ceil_div(M > 0 ? M : 1, S);
  float* part = static_cast<float*>(workspace);
  dim3 g1((unsigned)ceil_div(N, 256), (unsigned)S);
  colsum_partial_kernel<<<g1, 256, 0, st>>>(M, N, X, ldx, rows_per, part);
  colsum_final_kernel<<<(unsigned)ceil_div(N, 16), 256, 0, st>>>(N, S, part, N, alpha, beta, out);
  return check_launch("colsum");
}

// ---- weight gradient + bias gradient from one read of the gradient ------------------------
// C[M][N] = A^T B^T with both operands k-major (A = gY [K][lda]: a layer's weight gradient,
// K = atoms) and sum_out[c] = alpha sum_k A[k][sum_off + c] (its bias gradient, the column sums
// of gY).  Skinny products (the 128x128 split-fp16 plan: layer 1, N = 76) form the row sums
// from the fragments the product reads anyway (gemm_f32_kernel RS); other plans run the
// product and then mvml_colsum_f32 on the summed columns — the sequence this entry replaces.
namespace {
bool colsum_fused(int64_t M, int64_t N, int64_t K) {
  return M > 0 && N > 0 && K > 0 && N <= XBN && !plan_gemm(kPrecF16x2, M, N, K).wide;
}
}  // namespace

extern "C" int mvml_gemm_colsum_fused(int64_t M, int64_t N, int64_t K) { return colsum_fused(M, N, K) ? 1 : 0; }

extern "C" size_t mvml_gemm_colsum_workspace_size(int64_t M, int64_t N, int64_t K, int64_t sum_n) {
  const size_t parts = carve_size((size_t)2 * choose_splits(M, N, K) * std::max<int64_t>(M, 1) * sizeof(float));
  return carve_size(mvml_gemm_workspace_size(M, N, K)) +
         std::max(parts, mvml_colsum_workspace_size(K, std::max<int64_t>(sum_n, 1)));
}

extern "C" int mvml_gemm_f16x2_amax_colsum(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                                           const float* B, int64_t ldb, const uint32_t* amax_a,
                                           const uint32_t* amax_b, float* C, int64_t ldc, int64_t sum_off,
                                           int64_t sum_n, float alpha, float* sum_out, void* workspace,
                                           size_t workspace_bytes, void* stream) {
  clear_error();
  MVML_REQUIRE(amax_a != nullptr && amax_b != nullptr, "gemm_f16x2_amax_colsum: amax_a / amax_b are required");
  MVML_REQUIRE(M >= 0 && N >= 0 && K >= 0 && sum_off >= 0 && sum_n >= 0 && sum_off + sum_n <= M &&
                   (sum_n == 0 || sum_out),
               "gemm_f16x2_amax_colsum: bad shape");
  if (!workspace || workspace_bytes < mvml_gemm_colsum_workspace_size(M, N, K, sum_n)) {
    set_error("gemm_f16x2_amax_colsum: workspace too small (need %zu)",
              mvml_gemm_colsum_workspace_size(M, N, K, sum_n));
    return MVML_ERR_WORKSPACE;
  }
  const size_t gws = carve_size(mvml_gemm_workspace_size(M, N, K));
  float* extra = reinterpret_cast<float*>(static_cast<uint8_t*>(workspace) + gws);
  const size_t extra_bytes = workspace_bytes - gws;
  hipStream_t st = as_stream(stream);
  if (colsum_fused(M, N, K)) {
    AmaxPtrs am{amax_a, amax_b};
    am.a_rowsum = extra;
    int rc = gemm_launch(kPrecF16x2, 1, 1, M, N, K, A, lda, B, ldb, nullptr, 0.f, 0, C, ldc, workspace, gws,
                         stream, 1, BatchStrides{}, am);
    if (rc || sum_n == 0) return rc;
    const int parts = 2 * plan_gemm(kPrecF16x2, M, N, K).S;
    colsum_final_kernel<<<(unsigned)ceil_div(sum_n, 16), 256, 0, st>>>(sum_n, parts, extra + sum_off, M, alpha,
                                                                       0.f, sum_out);
    return check_launch("colsum_final_kernel(gemm row sums)");
  }
  int rc = gemm_launch(kPrecF16x2, 1, 1, M, N, K, A, lda, B, ldb, nullptr, 0.f, 0, C, ldc, workspace, gws, stream,
                       1, BatchStrides{}, AmaxPtrs{amax_a, amax_b});
  if (rc || sum_n == 0) return rc;
  return mvml_colsum_f32(K, sum_n, A + sum_off, lda, alpha, 0.f, sum_out, extra, extra_bytes, stream);
}

// ---- wide-batch BiLSTM steps (MVP's RNNModule at B > 512; BASELINE config 4) ---------------
// The recurrence of a bidirectional nn.LSTM layer (model.py:114-129) over a batch of thousands
// of sequences: one launch per time step for BOTH directions (direction 0 at t, direction 1 at
// T - 1 - t; a dual launch, blockIdx.z = direction) instead of a GEMM and a cell kernel per
// direction.
namespace {
struct LstmBwdArgs {
  int64_t M = 0, R = 0;             // rows of the step; rows fed a recurrent gradient (prefix)
  const float* gout = nullptr;      // dL/dh of the step's output rows (row stride ldgo)
  int64_t ldgo = 0;
  const float* slab = nullptr;      // [2][R][D] split-K halves of gg_next W_hh
  const float* act = nullptr;       // [M][4D] i, f, g, o (gate-major)
  const float* c = nullptr;         // [M][D]
  const float* c_prev = nullptr;    // [M][D] or null (the direction's first step)
  const float* carry_in = nullptr;  // [M][D] dL/dc from the step this one fed, or null
  float* carry_out = nullptr;       // [M][D]
  float* gg = nullptr;              // [M][4D] gate gradients (gate-major)
  uint32_t* gg_amax = nullptr;      // running max |gg| bits (split-fp16 scale of the next GEMMs)
};

// dh = (gg_next W_hh)[row] (the two split-K halves, in order) + dL/dh of the output, then
// lstm_cell_bwd_kernel's arithmetic in its order.
__global__ void __launch_bounds__(256) lstm_step_bwd_kernel(LstmBwdArgs a0, LstmBwdArgs a1, int D) {
  const LstmBwdArgs a = blockIdx.z ? a1 : a0;
  const int64_t total = a.M * D;
  float mx = 0.f;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / D;
    const int d = (int)(e - b * D);
    float gh = a.gout[b * a.ldgo + d];
    if (b < a.R) gh = (a.slab[e] + a.slab[a.R * D + e]) + gh;
    const float* ac = a.act + b * 4 * D;
    const float i = ac[d], f = ac[D + d], gt = ac[2 * D + d], o = ac[3 * D + d];
    const float tc = tanhf(a.c[e]);
    const float gc = (a.carry_in ? a.carry_in[e] : 0.f) + gh * o * (1.f - tc * tc);
    const float cp = a.c_prev ? a.c_prev[e] : 0.f;
    float* gg = a.gg + b * 4 * D;
    const float g0 = gc * gt * i * (1.f - i), g1 = gc * cp * f * (1.f - f);
    const float g2 = gc * i * (1.f - gt * gt), g3 = gh * tc * o * (1.f - o);
    gg[d] = g0;
    gg[D + d] = g1;
    gg[2 * D + d] = g2;
    gg[3 * D + d] = g3;
    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(g0), fabsf(g1)), fmaxf(fabsf(g2), fabsf(g3))));
    a.carry_out[e] = gc * f;
  }
  mx = wave_max(mx);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(a.gg_amax, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

// Tile of a step's products: the 256x256 tile's latency (~55 us for K = 384 however few its rows)
// sets the step time when there are too few row tiles to fill the chip; the 128x128 split-fp16
// kernel runs four times the workgroups at a quarter of the work each.  Measured per dual launch
// (tools/lstm_step_bench.py, H = 384; results bitwise equal): forward 128 <= 256 at every row
// count (24.9 / 54.0 us at 256 rows, 138.7 / 158.7 at 8192); backward 128 faster up to 4096 rows
// (90.6 / 101.9 us), level above (137.7 / 134.1 at 6144).  Option MVML_OPT_LSTM_TILE forces one.
constexpr int64_t kLstmBwdSmallRows = 4096;
bool lstm_small_tile(int64_t rows, bool bwd) {
  const int force = option(MVML_OPT_LSTM_TILE);
  if (force == 128 || force == 256) return force == 128;
  return !bwd || rows <= kLstmBwdSmallRows;
}
}  // namespace

// Wi_d: W_d's interleaved pre-split (split_il_launch, ld K) or null — the 128x128 plan then
// reads B ready-split (W is the same for every step of the layer).
static int wide_step_fwd(
    int64_t M0, int64_t M1, int D, int64_t K, const float* A0, const float* A1, int64_t lda,
    const float* W0, const float* W1, int64_t ldw, const float* gx0, const float* gx1,
    int64_t ldgx, const float* bih0, const float* bhh0, const float* bih1, const float* bhh1,
    const float* cprev0, const float* cprev1, float* c0, float* c1, float* h0, float* h1,
    int64_t ldh, float* act0, float* act1, const uint32_t* amax_a, const uint32_t* amax_w0,
    const uint32_t* amax_w1, void* stream, const float* Wi0, const float* Wi1) {
  const int64_t N = 4 * (int64_t)D;
  MVML_REQUIRE(M0 > 0 && M1 > 0 && D > 0 && K >= 0 && K % 4 == 0 && ldw >= K && ldw % 4 == 0 &&
                   ldgx >= N && ldh >= D && amax_a && amax_w0 && amax_w1 && MVML_X3W_LDSEPI,
               "bilstm_wide_step_fwd: bad shape");
  MVML_REQUIRE(K == 0 || (A0 && A1 && lda >= K && lda % 4 == 0 && (uintptr_t)A0 % 16 == 0 &&
                          (uintptr_t)A1 % 16 == 0),
               "bilstm_wide_step_fwd: A rows must be 16-B aligned");
  MVML_REQUIRE((uintptr_t)W0 % 16 == 0 && (uintptr_t)W1 % 16 == 0, "bilstm_wide_step_fwd: W alignment");
  CellEpi e0, e1;
  e0.b_ih = bih0; e0.b_hh = bhh0; e0.c_prev = cprev0; e0.c_out = c0; e0.h_out = h0; e0.act = act0;
  e0.ldh = ldh; e0.D = D; e0.gx = gx0; e0.ldgx = ldgx;
  e1 = e0;
  e1.b_ih = bih1; e1.b_hh = bhh1; e1.c_prev = cprev1; e1.c_out = c1; e1.h_out = h1; e1.act = act1;
  e1.gx = gx1;
  const float* a0 = K ? A0 : gx0;  // K = 0 (a direction's first step): no A rows are read
  const float* a1 = K ? A1 : gx1;
  if (lstm_small_tile(std::max(M0, M1), false)) {
    const int64_t tiles = ceil_div(std::max(M0, M1), BM) * ceil_div(N, BN);
    const dim3 grid((unsigned)tiles, 1, 2);
    if (Wi0 && Wi1 && K % BKT == 0)
      gemm_f32_kernel<false, false, -1, true, true, true><<<grid, kThreads, 0, as_stream(stream)>>>(
          M0, N, K, a0, K ? lda : 4, Wi0, K, nullptr, 0.f, 0, nullptr, N, K > 0 ? K : 1, nullptr, 1, 1,
          ProjEpi{}, BatchStrides{}, AmaxPtrs{amax_a, amax_w0}, e0, DualPtrs{a1, Wi1, nullptr, amax_w1, M1, e1});
    else
      gemm_f32_kernel<false, false, -1, true, true><<<grid, kThreads, 0, as_stream(stream)>>>(
          M0, N, K, a0, K ? lda : 4, W0, ldw, nullptr, 0.f, 0, nullptr, N, K > 0 ? K : 1, nullptr, 1, 1,
          ProjEpi{}, BatchStrides{}, AmaxPtrs{amax_a, amax_w0}, e0, DualPtrs{a1, W1, nullptr, amax_w1, M1, e1});
    return check_launch("gemm_f32_kernel(bilstm step)");
  }
  const int64_t tn = ceil_div(N, XBN);
  const int64_t tiles = std::max(ceil_div(M0, XBM), ceil_div(M1, XBM)) * tn;
  const dim3 grid((unsigned)tiles, 1, 2);
  gemm_x3w_kernel<false, false, -1, true, 2><<<grid, kXThreads, 0, as_stream(stream)>>>(
      M0, N, K, a0, K ? lda : 4, W0, ldw, nullptr, 0.f, 0, nullptr, N, K > 0 ? K : 1, nullptr, 1, 1,
      ProjEpi{}, BatchStrides{}, e0, AmaxPtrs{amax_a, amax_w0}, DualPtrs{a1, W1, nullptr, amax_w1, M1, e1});
  return check_launch("gemm_x3w_kernel(bilstm step)");
}

extern "C" int mvml_bilstm_wide_step_fwd(
    int64_t M0, int64_t M1, int D, int64_t K, const float* A0, const float* A1, int64_t lda,
    const float* W0, const float* W1, int64_t ldw, const float* gx0, const float* gx1,
    int64_t ldgx, const float* bih0, const float* bhh0, const float* bih1, const float* bhh1,
    const float* cprev0, const float* cprev1, float* c0, float* c1, float* h0, float* h1,
    int64_t ldh, float* act0, float* act1, const uint32_t* amax_a, const uint32_t* amax_w0,
    const uint32_t* amax_w1, void* stream) {
  clear_error();
  return wide_step_fwd(M0, M1, D, K, A0, A1, lda, W0, W1, ldw, gx0, gx1, ldgx, bih0, bhh0, bih1,
                       bhh1, cprev0, cprev1, c0, c1, h0, h1, ldh, act0, act1, amax_a, amax_w0, amax_w1,
                       stream, nullptr, nullptr);
}

extern "C" size_t mvml_bilstm_wide_step_bwd_workspace_size(int64_t M, int D) {
  return 2 * carve_size((size_t)2 * M * D * sizeof(float));
}

static int wide_step_bwd(
    int64_t M0, int64_t M1, int64_t R0, int64_t R1, int D, const float* gn0, const float* gn1,
    const float* wT0, const float* wT1, int64_t ldwT, const float* gout0, const float* gout1,
    int64_t ldgo, const float* act0, const float* act1, const float* c0, const float* c1,
    const float* cp0, const float* cp1, const float* carry_in0, const float* carry_in1,
    float* carry_out0, float* carry_out1, float* gg0, float* gg1, uint32_t* gg_amax0,
    uint32_t* gg_amax1, const uint32_t* amax_w0, const uint32_t* amax_w1, void* workspace,
    size_t workspace_bytes, void* stream, const float* Wi0, const float* Wi1) {
  const int64_t K = 4 * (int64_t)D, N = D;
  MVML_REQUIRE(M0 > 0 && M1 > 0 && R0 >= 0 && R0 <= M0 && R1 >= 0 && R1 <= M1 && (R0 > 0) == (R1 > 0) &&
                   D > 0 && D % 4 == 0 && ldwT >= K && ldwT % 4 == 0 && ldgo >= D && gg_amax0 &&
                   gg_amax1 && amax_w0 && amax_w1,
               "bilstm_wide_step_bwd: bad shape");
  const int64_t M = std::max(M0, M1);
  MVML_REQUIRE(workspace && workspace_bytes >= mvml_bilstm_wide_step_bwd_workspace_size(M, D),
               "bilstm_wide_step_bwd: workspace of mvml_bilstm_wide_step_bwd_workspace_size bytes required");
  hipStream_t st = as_stream(stream);
  float* slab0 = static_cast<float*>(workspace);
  float* slab1 = reinterpret_cast<float*>(static_cast<char*>(workspace) + carve_size((size_t)2 * M * D * sizeof(float)));
  if (R0 > 0) {  // dL/dh through the recurrence: gg_next W_hh, K split in two halves (slabs)
    MVML_REQUIRE(gn0 && gn1 && (uintptr_t)gn0 % 16 == 0 && (uintptr_t)gn1 % 16 == 0 &&
                     (uintptr_t)wT0 % 16 == 0 && (uintptr_t)wT1 % 16 == 0,
                 "bilstm_wide_step_bwd: alignment");
    const int S = 2;
    const int64_t kc = k_chunk(K, S);
    if (lstm_small_tile(std::max(R0, R1), true)) {
      const int64_t tiles = ceil_div(std::max(R0, R1), BM) * ceil_div(N, BN);
      const dim3 grid((unsigned)tiles, (unsigned)S, 2);
      if (Wi0 && Wi1 && kc % BKT == 0)
        gemm_f32_kernel<false, false, -1, true, true, true><<<grid, kThreads, 0, st>>>(
            R0, N, K, gn0, K, Wi0, K, nullptr, 0.f, 0, nullptr, N, kc, slab0, 1, 1, ProjEpi{},
            BatchStrides{}, AmaxPtrs{gg_amax0, amax_w0}, CellEpi{},
            DualPtrs{gn1, Wi1, slab1, amax_w1, R1, CellEpi{}, gg_amax1});
      else
        gemm_f32_kernel<false, false, -1, true, true><<<grid, kThreads, 0, st>>>(
            R0, N, K, gn0, K, wT0, ldwT, nullptr, 0.f, 0, nullptr, N, kc, slab0, 1, 1, ProjEpi{},
            BatchStrides{}, AmaxPtrs{gg_amax0, amax_w0}, CellEpi{},
            DualPtrs{gn1, wT1, slab1, amax_w1, R1, CellEpi{}, gg_amax1});
      int rc = check_launch("gemm_f32_kernel(bilstm step bwd)");
      if (rc) return rc;
    } else {
    const int64_t tiles = std::max(ceil_div(R0, XBM), ceil_div(R1, XBM)) * ceil_div(N, XBN);
    const dim3 grid((unsigned)tiles, (unsigned)S, 2);
    gemm_x3w_kernel<false, false, -1, true, 2><<<grid, kXThreads, 0, st>>>(
        R0, N, K, gn0, K, wT0, ldwT, nullptr, 0.f, 0, nullptr, N, kc, slab0, 1, 1, ProjEpi{},
        BatchStrides{}, CellEpi{}, AmaxPtrs{gg_amax0, amax_w0},
        DualPtrs{gn1, wT1, slab1, amax_w1, R1, CellEpi{}, gg_amax1});
    int rc = check_launch("gemm_x3w_kernel(bilstm step bwd)");
    if (rc) return rc;
    }
  }
  LstmBwdArgs a0, a1;
  a0.M = M0; a0.R = R0; a0.gout = gout0; a0.ldgo = ldgo; a0.slab = slab0; a0.act = act0; a0.c = c0;
  a0.c_prev = cp0; a0.carry_in = R0 > 0 ? carry_in0 : nullptr; a0.carry_out = carry_out0; a0.gg = gg0;
  a0.gg_amax = gg_amax0;
  a1 = a0;
  a1.M = M1; a1.R = R1; a1.gout = gout1; a1.slab = slab1; a1.act = act1; a1.c = c1; a1.c_prev = cp1;
  a1.carry_in = R1 > 0 ? carry_in1 : nullptr; a1.carry_out = carry_out1; a1.gg = gg1;
  a1.gg_amax = gg_amax1;
  const int64_t work = M * D;
  const unsigned blocks = (unsigned)std::min<int64_t>(std::max<int64_t>(256, ceil_div(work, 4096)),
                                                      ceil_div(work, 256));
  lstm_step_bwd_kernel<<<dim3(blocks, 1, 2), 256, 0, st>>>(a0, a1, D);
  return check_launch("lstm_step_bwd_kernel");
}

extern "C" int mvml_bilstm_wide_step_bwd(
    int64_t M0, int64_t M1, int64_t R0, int64_t R1, int D, const float* gn0, const float* gn1,
    const float* wT0, const float* wT1, int64_t ldwT, const float* gout0, const float* gout1,
    int64_t ldgo, const float* act0, const float* act1, const float* c0, const float* c1,
    const float* cp0, const float* cp1, const float* carry_in0, const float* carry_in1,
    float* carry_out0, float* carry_out1, float* gg0, float* gg1, uint32_t* gg_amax0,
    uint32_t* gg_amax1, const uint32_t* amax_w0, const uint32_t* amax_w1, void* workspace,
    size_t workspace_bytes, void* stream) {
  clear_error();
  return wide_step_bwd(M0, M1, R0, R1, D, gn0, gn1, wT0, wT1, ldwT, gout0, gout1, ldgo, act0, act1,
                       c0, c1, cp0, cp1, carry_in0, carry_in1, carry_out0, carry_out1, gg0, gg1,
                       gg_amax0, gg_amax1, amax_w0, amax_w1, workspace, workspace_bytes, stream,
                       nullptr, nullptr);
}

// The whole recurrence of a wide bidirectional layer: every step's dual launch enqueued from this
// loop (the host side of the recurrence is native, so enqueueing a step costs a few microseconds,
// not a Python frame building some thirty arguments and tensor views per step).
// Both layer loops pre-split W_hh (resp. its transpose) once into the workspace: every step's
// 128x128 launch then reads B ready-split (split_f16x2_il_kernel) instead of splitting it again in
// every workgroup of every step.
extern "C" size_t mvml_bilstm_wide_fwd_workspace_size(int D) {
  return 2 * carve_size((size_t)4 * D * D * sizeof(float));
}

extern "C" int mvml_bilstm_wide_fwd(int64_t T, int64_t B, int D, const int32_t* batch_sizes,
                                    const float* W0, const float* W1, const float* gx0,
                                    const float* gx1, const float* bih0, const float* bhh0,
                                    const float* bih1, const float* bhh1, float* c0, float* c1,
                                    float* out, float* act0, float* act1, const uint32_t* amax,
                                    int gx_packed, void* workspace, size_t workspace_bytes,
                                    void* stream) {
  clear_error();
  MVML_REQUIRE(T > 0 && B > 0 && D > 0 && D % 8 == 0 && batch_sizes && amax,
               "bilstm_wide_fwd: bad arguments");
  MVML_REQUIRE(workspace && workspace_bytes >= mvml_bilstm_wide_fwd_workspace_size(D),
               "bilstm_wide_fwd: workspace of mvml_bilstm_wide_fwd_workspace_size bytes required");
  for (int64_t t = 0; t < T; ++t)
    MVML_REQUIRE(batch_sizes[t] > 0 && batch_sizes[t] <= B && (t == 0 || batch_sizes[t] <= batch_sizes[t - 1]),
                 "bilstm_wide_fwd: batch_sizes must be positive, <= B and non-increasing");
  const int64_t G = 4 * (int64_t)D, H2 = 2 * (int64_t)D;
  // first gx row of step t: time-major t B, or packed (step blocks of batch_sizes[t] rows)
  std::vector<int64_t> row(T);
  for (int64_t t = 0, acc = 0; t < T; acc += batch_sizes[t], ++t) row[t] = gx_packed ? acc : t * B;
  float* Wi0 = static_cast<float*>(workspace);
  float* Wi1 = reinterpret_cast<float*>(static_cast<char*>(workspace) + carve_size((size_t)G * D * sizeof(float)));
  hipStream_t st = as_stream(stream);
  int rc0 = split_il_launch(G, D, W0, amax + 1, Wi0, st);
  if (!rc0) rc0 = split_il_launch(G, D, W1, amax + 2, Wi1, st);
  if (rc0) return rc0;
  for (int64_t s = 0; s < T; ++s) {
    const int64_t t0 = s, t1 = T - 1 - s, p0 = t0 - 1, p1 = t1 + 1;
    const bool first = s == 0;
    const int rc = wide_step_fwd(
        batch_sizes[t0], batch_sizes[t1], D, first ? 0 : D, first ? nullptr : out + p0 * B * H2,
        first ? nullptr : out + p1 * B * H2 + D, H2, W0, W1, D, gx0 + row[t0] * G, gx1 + row[t1] * G, G,
        bih0, bhh0, bih1, bhh1, first ? nullptr : c0 + p0 * B * D, first ? nullptr : c1 + p1 * B * D,
        c0 + t0 * B * D, c1 + t1 * B * D, out + t0 * B * H2, out + t1 * B * H2 + D, H2,
        act0 + t0 * B * G, act1 + t1 * B * G, amax, amax + 1, amax + 2, stream, Wi0, Wi1);
    if (rc) return rc;
  }
  return MVML_OK;
}

extern "C" size_t mvml_bilstm_wide_bwd_workspace_size(int64_t B, int D) {
  return mvml_bilstm_wide_step_bwd_workspace_size(B, D) + 2 * carve_size((size_t)4 * D * D * sizeof(float));
}

extern "C" int mvml_bilstm_wide_bwd(int64_t T, int64_t B, int D, const int32_t* batch_sizes,
                                    const float* wT0, const float* wT1, const float* gout,
                                    const float* act0, const float* act1, const float* c0,
                                    const float* c1, float* carry, float* gg0, float* gg1,
                                    uint32_t* gg_amax, const uint32_t* amax, int gg_packed,
                                    void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  MVML_REQUIRE(T > 0 && B > 0 && D > 0 && D % 8 == 0 && batch_sizes && carry && gg_amax && amax,
               "bilstm_wide_bwd: bad arguments");
  MVML_REQUIRE(workspace && workspace_bytes >= mvml_bilstm_wide_bwd_workspace_size(B, D),
               "bilstm_wide_bwd: workspace of mvml_bilstm_wide_bwd_workspace_size bytes required");
  for (int64_t t = 0; t < T; ++t)
    MVML_REQUIRE(batch_sizes[t] > 0 && batch_sizes[t] <= B && (t == 0 || batch_sizes[t] <= batch_sizes[t - 1]),
                 "bilstm_wide_bwd: batch_sizes must be positive, <= B and non-increasing");
  const int64_t G = 4 * (int64_t)D, H2 = 2 * (int64_t)D, BD = B * (int64_t)D;
  // carry: [direction][ping-pong][B][D]
  float* cr[2][2] = {{carry, carry + BD}, {carry + 2 * BD, carry + 3 * BD}};
  std::vector<int64_t> row(T);  // first gg row of step t (time-major or packed, as the forward's gx)
  for (int64_t t = 0, acc = 0; t < T; acc += batch_sizes[t], ++t) row[t] = gg_packed ? acc : t * B;
  const size_t slabs = mvml_bilstm_wide_step_bwd_workspace_size(B, D);
  float* Wi0 = reinterpret_cast<float*>(static_cast<char*>(workspace) + slabs);
  float* Wi1 = reinterpret_cast<float*>(static_cast<char*>(workspace) + slabs + carve_size((size_t)G * D * sizeof(float)));
  hipStream_t st = as_stream(stream);
  int rc0 = split_il_launch(D, G, wT0, amax + 1, Wi0, st);  // W_hh^T: D rows of K = 4 D
  if (!rc0) rc0 = split_il_launch(D, G, wT1, amax + 2, Wi1, st);
  if (rc0) return rc0;
  for (int64_t s = 0; s < T; ++s) {
    const int64_t t0 = T - 1 - s, t1 = s, n0 = t0 + 1, n1 = t1 - 1;  // n: the steps these fed
    const int64_t R0 = s == 0 ? 0 : std::min(batch_sizes[t0], batch_sizes[n0]);
    const int64_t R1 = s == 0 ? 0 : std::min(batch_sizes[t1], batch_sizes[n1]);
    const int ci = (int)(s % 2), co = (int)((s + 1) % 2);
    const int rc = wide_step_bwd(
        batch_sizes[t0], batch_sizes[t1], R0, R1, D, gg0 + row[s ? n0 : t0] * G,
        gg1 + row[s ? n1 : t1] * G, wT0, wT1, G, gout + t0 * B * H2, gout + t1 * B * H2 + D, H2,
        act0 + t0 * B * G, act1 + t1 * B * G, c0 + t0 * BD, c1 + t1 * BD,
        t0 >= 1 ? c0 + (t0 - 1) * BD : nullptr, t1 + 1 < T ? c1 + (t1 + 1) * BD : nullptr,
        cr[0][ci], cr[1][ci], cr[0][co], cr[1][co], gg0 + row[t0] * G, gg1 + row[t1] * G, gg_amax,
        gg_amax + 1, amax + 1, amax + 2, workspace, slabs, stream, Wi0, Wi1);
    if (rc) return rc;
  }
  return MVML_OK;
}
