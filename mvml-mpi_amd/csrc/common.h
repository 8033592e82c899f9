// Shared helpers for the mvml_gat HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include <algorithm>

#include "../../include/mvml_gat.h"

namespace mvml {

// Thread-local last-error string (mvml_last_error).
void set_error(const char* fmt, ...);
void clear_error();

constexpr int kWave = 64;
// Target size of a node group (mvml_build_node_groups): whole molecules, ~this many atoms.
constexpr int kNodeGroupAtoms = 64;
// Node-group plan caps (mvml_build_node_groups): the LDS aggregation kernels' limits.
constexpr int kPlanWinAtoms = 128;  // atoms per group
constexpr int kPlanEdgeCap = 512;   // in-edges per group
constexpr int kPlanDegCap = 5;      // forward: in-degree of every atom
// Big LDS window (kind bit 2): node groups of up to kPlanBigAtoms atoms / kPlanBigEdgeCap
// in-edges (a 150-400-atom molecule with hubs, BASELINE config 5) staged 16 columns at a time.
constexpr int kPlanBigAtoms = 512;
constexpr int kPlanBigEdgeCap = 2432;
// Plan layout (int32, G = mvml_node_group_count(N)): [0, G] group starts | [G+1, 2G+1) kinds |
// 2G+1, 2G+2: forward / backward fallback counts | [2G+3, 3G+3) forward fallback groups |
// [3G+3, 4G+3) backward fallback groups.
struct GroupPlan {
  const int32_t* start;
  const int32_t* kind;
  const int32_t* count;
  const int32_t* fwd_list;
  const int32_t* bwd_list;
  __host__ __device__ GroupPlan(const int32_t* p, int64_t G)
      : start(p), kind(p + G + 1), count(p + 2 * G + 1), fwd_list(p + 2 * G + 3),
        bwd_list(p + 3 * G + 3) {}
};

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Check the launch we just enqueued; never synchronises.
int check_launch(const char* what);
// Current value of a kernel-path option (MVML_OPT_*, capi.cpp).
int option(int which);

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Workspace carving: 256-byte aligned sub-buffers.
struct Carver {
  char* base;
  size_t cap;
  size_t used = 0;
  Carver(void* b, size_t c) : base(static_cast<char*>(b)), cap(c) {}
  template <typename T>
  T* take(size_t count) {
    size_t off = (used + 255) & ~size_t(255);
    used = off + count * sizeof(T);
    return reinterpret_cast<T*>(base + off);
  }
  bool ok() const { return used <= cap; }
};
inline size_t carve_size(size_t bytes) { return (bytes + 255) & ~size_t(255); }

// ---- device helpers -------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Raw buffer addressing: a wave-uniform base in a 128-bit SGPR resource + a 32-bit per-lane
// byte offset (one VGPR per address instead of a 64-bit pointer pair).  Out-of-range offsets
// (>= bytes) read 0 and drop stores.  Resource word 3 = 0x00020000 for gfx9 (32-bit data).
typedef unsigned int mvml_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float4 buf_ld4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}
__device__ __forceinline__ void buf_st4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(mvml_u32x4, v), r, byte_off, 0, 0);
}

// XCD-aware workgroup remap (bijective for any grid size).  The dispatcher deals workgroups
// round-robin over the 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch); this returns a logical
// block index such that each XCD walks ONE contiguous range, so neighbouring atoms / molecules
// share an XCD's L2.  Speed only: correctness never depends on the placement.
__device__ __forceinline__ int64_t xcd_block(unsigned b, unsigned nb) {
  const unsigned q = nb / 8, r = nb % 8, x = b % 8, i = b / 8;
  return (int64_t)((x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// gemm_f32.hip: projection GEMM with the GAT logits-partial epilogue (see ProjEpi there).
int gemm_proj_epi(int prec, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                  const float* B, int64_t ldb, float* C, int64_t ldc, const float* vec, int cols,
                  int logw, float* part, uint32_t* amax_ws, const uint32_t* amax_x,
                  const uint32_t* amax_w, const uint16_t* w_planes, int64_t w_plane,
                  hipStream_t st);
// Partial-logit group width of mvml_gat_proj_fwd: the largest power of two <= 32 dividing F.
inline int proj_logw(int F) {
  int lw = 0;
  while (lw < 5 && F % (2 << lw) == 0) ++lw;
  return lw;
}

}  // namespace mvml

#define MVML_REQUIRE(cond, ...)          \
  do {                                   \
    if (!(cond)) {                       \
      ::mvml::set_error(__VA_ARGS__);    \
      return MVML_ERR_INVALID;           \
    }                                    \
  } while (0)
