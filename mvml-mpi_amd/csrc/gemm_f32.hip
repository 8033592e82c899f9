// Dense fp32 GEMM on CDNA4 matrix cores (v_mfma_f32_32x32x2_f32) + column sums.
//
// Used for every dense product of the view: GATConv fc/res_fc (+ the folded el/er columns),
// their backward (dX = dY * W, dW = dY^T * X), the Set2Set LSTM gate GEMMs and
// GNNModule.fc (model.py:86-87).  f32-input MFMA is exact f32 (a k-ordered fmaf chain), so
// results match a CPU fp32 GEMM to rounding.
//
// Tiling: 128x128 output tile per 256-thread workgroup (4 waves as 2x2, 64x64 per wave =
// 2x2 MFMA 32x32 tiles), K staged through LDS 32 deep with register prefetch of the next
// stage.  LDS images are k-major ([k][m], [k][n]) so that an MFMA operand fragment
// (lane l -> row l&31, k = l>>5) is one conflict-free ds_read_b32.  Operands may be stored
// k-major or not (a_kmajor / b_kmajor); rows that allow it are loaded 16 B per lane.
// Small-output / long-K products (the weight gradients, K = atoms in the batch) split K over
// workgroups into fp32 slabs that a second kernel sums in fixed order — deterministic, no
// float atomics.
#include "common.h"

namespace mvml {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BKT = 32, kThreads = 256;

template <bool KMAJ>
struct TileLoader {
  // Loads a (rows=128) x (k=32) operand tile. KMAJ: element(r,k) = P[k*ld + r], else P[r*ld + k].
  static constexpr int PAD = KMAJ ? 4 : 1;
  static constexpr int LDS_LD = 128 + PAD;
  float4 reg[4];

  __device__ __forceinline__ void load(const float* __restrict__ P, int64_t ld, int64_t r0,
                                       int64_t rows, int64_t k0, int64_t kend, bool vec) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = threadIdx.x + it * kThreads;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (!KMAJ) {
        const int r = idx >> 3, k4 = idx & 7;
        const int64_t gr = r0 + r, gk = k0 + 4 * k4;
        if (gr < rows) {
          const float* p = P + gr * ld + gk;
          if (vec && gk + 3 < kend) {
            float4 t = *reinterpret_cast<const float4*>(p);
            v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (gk + j < kend) v[j] = p[j];
          }
        }
      } else {
        const int k = idx >> 5, r4 = idx & 31;
        const int64_t gk = k0 + k, gr = r0 + 4 * r4;
        if (gk < kend) {
          const float* p = P + gk * ld + gr;
          if (vec && gr + 3 < rows) {
            float4 t = *reinterpret_cast<const float4*>(p);
            v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (gr + j < rows) v[j] = p[j];
          }
        }
      }
      reg[it] = make_float4(v[0], v[1], v[2], v[3]);
    }
  }

  __device__ __forceinline__ void store(float* lds) const {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = threadIdx.x + it * kThreads;
      if (!KMAJ) {
        const int r = idx >> 3, k4 = idx & 7;
        lds[(4 * k4 + 0) * LDS_LD + r] = reg[it].x;
        lds[(4 * k4 + 1) * LDS_LD + r] = reg[it].y;
        lds[(4 * k4 + 2) * LDS_LD + r] = reg[it].z;
        lds[(4 * k4 + 3) * LDS_LD + r] = reg[it].w;
      } else {
        const int k = idx >> 5, r4 = idx & 31;
        *reinterpret_cast<float4*>(&lds[k * LDS_LD + 4 * r4]) = reg[it];
      }
    }
  }
};

template <bool AK, bool BKM>
__global__ void __launch_bounds__(kThreads)
gemm_f32_kernel(int64_t M, int64_t N, int64_t K, const float* __restrict__ A, int64_t lda,
                const float* __restrict__ B, int64_t ldb, const float* __restrict__ bias,
                float beta, int act, float* __restrict__ C, int64_t ldc, int64_t k_split,
                float* __restrict__ slab, int a_vec, int b_vec) {
  using LA = TileLoader<AK>;
  using LB = TileLoader<BKM>;
  __shared__ __attribute__((aligned(16))) float lds[BKT * LA::LDS_LD + BKT * LB::LDS_LD];
  float* As = lds;
  float* Bs = lds + BKT * LA::LDS_LD;

  // Tile order: consecutive workgroups walk N first so an A row-panel is reused from L2.
  const int64_t tiles_n = ceil_div(N, BN);
  const int64_t tile = blockIdx.x;
  const int64_t m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int64_t kbeg = (int64_t)blockIdx.y * k_split;
  const int64_t kend = min(K, kbeg + k_split);

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int li = lane & 31, lk = lane >> 5;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  LA la;
  LB lb;
  if (kbeg < kend) {
    la.load(A, lda, m0, M, kbeg, kend, a_vec);
    lb.load(B, ldb, n0, N, kbeg, kend, b_vec);
  }
  for (int64_t kt = kbeg; kt < kend; kt += BKT) {
    la.store(As);
    lb.store(Bs);
    __syncthreads();
    if (kt + BKT < kend) {
      la.load(A, lda, m0, M, kt + BKT, kend, a_vec);
      lb.load(B, ldb, n0, N, kt + BKT, kend, b_vec);
    }
#pragma unroll
    for (int kk = 0; kk < BKT; kk += 2) {
      const float a0 = As[(kk + lk) * LA::LDS_LD + wm * 64 + li];
      const float a1 = As[(kk + lk) * LA::LDS_LD + wm * 64 + 32 + li];
      const float b0 = Bs[(kk + lk) * LB::LDS_LD + wn * 64 + li];
      const float b1 = Bs[(kk + lk) * LB::LDS_LD + wn * 64 + 32 + li];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }

  // Epilogue. C/D map of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wn * 64 + j * 32 + li;
      if (col >= N) continue;
      const float bcol = (bias && !slab) ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row >= M) continue;
        float v = acc[i][j][r];
        if (slab) {
          slab[((int64_t)blockIdx.y * M + row) * N + col] = v;
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

// Split policy: enough workgroups to cover the chip (~2 per CU) for small-output, long-K
// products; K chunks are multiples of the 32-deep stage.
int choose_splits(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ceil_div(M, BM) * ceil_div(N, BN);
  if (tiles >= 512 || K < 1024) return 1;
  int64_t s = ceil_div(512, tiles);
  s = std::min<int64_t>(s, ceil_div(K, 512));  // keep >= 512 K per split
  s = std::min<int64_t>(s, 64);
  return (int)std::max<int64_t>(s, 1);
}

int64_t k_chunk(int64_t K, int S) { return ceil_div(ceil_div(K, S), BKT) * BKT; }

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

__global__ void colsum_final_kernel(int64_t N, int S, const float* __restrict__ part, float alpha,
                                    float beta, float* __restrict__ out) {
  const int64_t col = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= N) return;
  float s = 0.f;
  for (int z = 0; z < S; ++z) s += part[(int64_t)z * N + col];
  out[col] = (beta != 0.f ? beta * out[col] : 0.f) + alpha * s;
}

int colsum_splits(int64_t M, int64_t N) {
  const int64_t colblocks = ceil_div(N, 256);
  int64_t s = ceil_div(2048, colblocks);
  s = std::min<int64_t>(s, ceil_div(M, 64));
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, 4096));
}

}  // namespace
}  // namespace mvml

using namespace mvml;

extern "C" size_t mvml_gemm_workspace_size(int64_t M, int64_t N, int64_t K) {
  const int S = choose_splits(M, N, K);
  return S > 1 ? carve_size((size_t)S * M * N * sizeof(float)) : 0;
}

extern "C" int mvml_gemm_f32(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                             const float* A, int64_t lda, const float* B, int64_t ldb,
                             const float* bias, float beta, int act, float* C, int64_t ldc,
                             void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  MVML_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm: negative size");
  if (M == 0 || N == 0) return MVML_OK;
  MVML_REQUIRE(ldc >= N, "gemm: ldc < N");
  MVML_REQUIRE(a_kmajor ? lda >= M : lda >= K, "gemm: bad lda");
  MVML_REQUIRE(b_kmajor ? ldb >= N : ldb >= K, "gemm: bad ldb");
  MVML_REQUIRE(act == 0 || act == 1, "gemm: bad act");
  hipStream_t st = as_stream(stream);
  const int S = choose_splits(M, N, K);
  float* slab = nullptr;
  if (S > 1) {
    if (workspace_bytes < mvml_gemm_workspace_size(M, N, K) || !workspace) {
      set_error("gemm: workspace too small (need %zu)", mvml_gemm_workspace_size(M, N, K));
      return MVML_ERR_WORKSPACE;
    }
    slab = static_cast<float*>(workspace);
  }
  const int64_t kc = S > 1 ? k_chunk(K, S) : (K > 0 ? K : 1);
  const int64_t tiles = ceil_div(M, BM) * ceil_div(N, BN);
  MVML_REQUIRE(tiles < (int64_t(1) << 31), "gemm: too many tiles");
  const int av = (lda % 4 == 0) && ((uintptr_t)A % 16 == 0);
  const int bv = (ldb % 4 == 0) && ((uintptr_t)B % 16 == 0);
  dim3 grid((unsigned)tiles, (unsigned)S);
#define MVML_GEMM_LAUNCH(AKV, BKV)                                                         \
  gemm_f32_kernel<AKV, BKV><<<grid, kThreads, 0, st>>>(M, N, K, A, lda, B, ldb, bias, beta, \
                                                       act, C, ldc, kc, slab, av, bv)
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
  colsum_final_kernel<<<(unsigned)ceil_div(N, 256), 256, 0, st>>>(N, S, part, alpha, beta, out);
  return check_launch("colsum");
}
