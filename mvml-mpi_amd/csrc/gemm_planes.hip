// Split-fp16 GEMM with LDS-DMA staging of pre-split operand images (round 6).
//
// C[M][N] = A[M][K] B[N][K]^T at fp32 accuracy on fp16 MFMA (the scaled split-fp16 of
// gemm_common.h: x s = h + l, three MFMAs per fragment pair: l_a h_b, h_a l_b, h_a h_b).
// The products it serves are the row-scaled ones of a training step (GATConv projection and
// data gradient, the Set2Set LSTM gate products, /root/reference/model.py:81-95): K is a
// feature dimension (76 .. 1928) and M is atoms or molecules.
//
// What differs from gemm_x3w_kernel (gemm_f32.hip), whose counters on these products show the
// matrix pipe busy 0.43-0.49 of the time, a third of the wave time parked on the one-stage
// register pipeline and 3-4 VALU per MFMA (profiles/r05_pmc_gemm_config3.txt):
//  * B arrives as its "il8" image (mvml_split_f16x2_il8: every 8-value k group of a row is its
//    8 scaled high fp16 halves, then its 8 low halves — 32 B in place of the group's 32 B of
//    fp32, rows zero-padded to a multiple of 16 k), so B is never split in the loop;
//  * A arrives as fp32 (split by the wave that reads it, with its row's own scale) or as its
//    il8 image (APS: no split at all);
//  * both operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4: no staging registers,
//    no ds_write), into a 4-slot ring of 16-deep stages with up to three stages in flight
//    behind the one being read (counted vmcnt, raw s_barrier: a barrier never drains the ring);
//  * 8 waves as 4 (M) x 2 (N), 64 x 128 outputs per wave, so an A fragment is split by the two
//    waves that share its rows (not four).
// Stage image per operand: [256 rows][64 B] = the row's 16 k as four 16-B chunks (fp32: k
// 0-3, 4-7, 8-11, 12-15; il8: h(0-7), l(0-7), h(8-15), l(8-15)), chunk index XOR-swizzled by
// (row >> 2) & 3 through the DMA's SOURCE address (the LDS side of a DMA is lane-linear), so a
// 32x32x16 fragment read (ds_read_b128, lane = row, k group = lane >> 5) is conflict-free.
// The epilogue is gemm_x3w_kernel's (epilogue_lds: bias, beta, ReLU / ELU / ELU', the LSTM
// cell, folded per-row output maxima), run on the two 64-column halves of a wave's tile.
#include <cstdlib>

#include "common.h"
#include "gemm_common.h"

namespace mvml {
namespace {

constexpr int kPBM = 256, kPBN = 256, kPThreads = 512;
// Stage geometry of the BK-deep ring (BK = 16: four 32-KB slots, three stages in flight; BK = 32:
// two 64-KB slots, one in flight, but every DMA moves whole 128-B row segments)
template <int BK>
struct PGeo {
  static constexpr int RB = BK * 4;           // bytes of a row per stage (fp32 or il8 alike)
  static constexpr int CH = BK / 4;           // 16-B chunks per row
  static constexpr int OP = 256 * RB;         // one operand's stage image
  static constexpr int STAGE = 2 * OP;        // [A | B]
  static constexpr int RING = BK == 16 ? 4 : 2;
  static constexpr int RING_BYTES = RING * STAGE;  // 128 KB
  static constexpr int RPI = 1024 / RB;       // rows per DMA wave-instruction
  static constexpr int IPW = 256 / RPI / 8;   // DMA instructions per wave and operand
  static constexpr int DPS = 2 * IPW;         // ... per wave and stage
  static constexpr int SUB = BK / 16;         // 16-deep MFMA steps per stage
  static_assert(RING_BYTES >= 8 * 32 * kEpiLd * 4, "the epilogue reuses the ring");
  // the 16-B chunk index XOR that makes a 32x32x16 fragment read (ds_read_b128, 16-lane groups
  // of 16 rows at one chunk) conflict-free: 64-B rows (r >> 2) & 3, 128-B rows (r >> 1) & 7
  __device__ static __forceinline__ int swz(int row) { return BK == 16 ? ((row >> 2) & 3) : ((row >> 1) & 7); }
};

// One operand's stage by LDS-DMA: wave wid's IPW 1-KB pieces (RPI rows each; lane -> row
// RPI inst + lane / CH, chunk (lane % CH) ^ swz(row)).  Rows past `rows` re-read the last row
// (their outputs are never stored); k is clamped to kmax4 (the last in-row float4 of an fp32 A:
// the K tail reads in-row values that the split zeroes; images are zero-padded past K).
template <int BK>
__device__ __forceinline__ void p_issue(const float* __restrict__ P, int64_t ld, int64_t r0,
                                        int64_t rows, int64_t k0, int64_t kmax4, uint8_t* dst,
                                        int wid, int lane) {
  using G = PGeo<BK>;
#pragma unroll
  for (int it = 0; it < G::IPW; ++it) {
    const int inst = G::IPW * wid + it;
    const int row = G::RPI * inst + lane / G::CH;
    const int64_t k = min(k0 + 4 * ((lane % G::CH) ^ G::swz(row)), kmax4);
    const float* src = P + min(r0 + row, rows - 1) * ld + k;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(dst + inst * 1024),
                                     16, 0, 0);
  }
}

// Fragment read the compiler does not see (it would otherwise wait vmcnt(0) — draining the
// ring — before every ds_read of LDS that a DMA writes); the caller waits lgkmcnt.
template <int OFF>
__device__ __forceinline__ void p_rd(u32x4& r, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF) : "memory");
}
template <int N>
__device__ __forceinline__ void p_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// A row-maximum load outside the compiler's wait bookkeeping (read after a counted vmcnt that
// covers it: it is issued before the stage DMAs)
__device__ __forceinline__ uint32_t p_ld_u32(const uint32_t* p) {
  uint32_t v;
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// ABL (timing ablations, MVML_PLANES_ABL; wrong results): 1 = no epilogue (the accumulators
// are consumed, nothing is stored), 2 = no MFMAs
template <bool APS, bool ROWS, bool EX, bool CELL, int BK, int ABL = 0>
__global__ void __launch_bounds__(kPThreads, 2)  // one workgroup per CU, two waves per SIMD
gemm_planes_kernel(int64_t M, int64_t N, int64_t K, const float* __restrict__ A, int64_t lda,
                   const float* __restrict__ B, int64_t ldb, const float* __restrict__ bias,
                   float beta, int act, float* __restrict__ C, int64_t ldc, AmaxPtrs amax,
                   CellEpi cep_arg, EpiX ex_arg) {
  using G = PGeo<BK>;
  const CellEpi cep = CELL ? cep_arg : CellEpi{};
  const EpiX ex = EX ? ex_arg : EpiX{};
  // ring | per-row scale shifts of the tile | folded per-row output maxima (one __shared__
  // object: a second one can make hipcc drain the DMA ring before LDS reads)
  __shared__ __attribute__((aligned(16))) uint8_t lds[G::RING_BYTES + 2 * kPBM * 4];
  int* rsh = reinterpret_cast<int*>(lds + G::RING_BYTES);
  uint32_t* s_rmax = reinterpret_cast<uint32_t*>(lds + G::RING_BYTES + kPBM * 4);
  const uint32_t lds_b = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int li = lane & 31, lk = lane >> 5;
  const int kb = amax_shift(*amax.b);
  const int ka = ROWS ? 0 : amax_shift(*amax.a);
  // this lane's fragment offsets in a stage image: row li of a 32-row block (blocks 32 RB apart),
  // 16-deep step u: chunks 4 u + 2 lk and 4 u + 2 lk + 1
  const int sw = G::swz(li);
  uint32_t o0[G::SUB], o1[G::SUB];
#pragma unroll
  for (int u = 0; u < G::SUB; ++u) {
    o0[u] = li * G::RB + 16 * ((4 * u + 2 * lk) ^ sw);
    o1[u] = li * G::RB + 16 * ((4 * u + 2 * lk + 1) ^ sw);
  }
  const uint32_t oa = wm * 64 * G::RB, ob = G::OP + wn * 128 * G::RB;
  const int64_t nst = ceil_div(K, BK);
  const int64_t kmax_a = APS ? nst * BK - 4 : K - 4, kmax_b = nst * BK - 4;
  const bool tail = !APS && (K % BK) != 0;
  const bool lds_rows = EX && ex.c_rows && cep.D == 0 && (ex.rows_cols == 0 || ex.rows_cols % kPBN == 0);
  // XCD x (the workgroups b % 8 == x) walks one contiguous tile range, N fastest: the tiles in
  // flight on an XCD share A row panels in its L2
  const int64_t tiles_n = ceil_div(N, kPBN);
  const int64_t n_tiles = ceil_div(M, kPBM) * tiles_n;
  const unsigned xq = n_tiles / 8, xr = n_tiles % 8, bx = blockIdx.x % 8;
  const int64_t t_beg = (bx < xr) ? bx * (xq + 1) : xr * (xq + 1) + (bx - xr) * xq;
  const int64_t t_end = t_beg + xq + (bx < xr ? 1 : 0);
  const unsigned bq = gridDim.x / 8, br = gridDim.x % 8;
  const int64_t t_step = bq + (bx < br ? 1 : 0);
  for (int64_t tile = t_beg + blockIdx.x / 8; tile < t_end; tile += t_step) {
    // the previous tile's epilogue is done with the LDS (its global stores may still drain)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int64_t m0 = (tile / tiles_n) * kPBM, n0 = (tile % tiles_n) * kPBN;
    // per-row maxima first (older than the DMAs, so the prologue's counted wait covers them)
    uint32_t rb_t = 0, rb_0 = 0, rb_1 = 0;
    if constexpr (ROWS) {
      if (tid < kPBM) rb_t = p_ld_u32(amax.a_rows + min(m0 + tid, M - 1));
      if constexpr (!APS) {
        rb_0 = p_ld_u32(amax.a_rows + min(m0 + wm * 64 + li, M - 1));
        rb_1 = p_ld_u32(amax.a_rows + min(m0 + wm * 64 + 32 + li, M - 1));
      }
    }
    auto issue = [&](int64_t t) {
      uint8_t* st = lds + (t % G::RING) * G::STAGE;
      p_issue<BK>(A, lda, m0, M, t * BK, kmax_a, st, wid, lane);
      p_issue<BK>(B, ldb, n0, N, t * BK, kmax_b, st + G::OP, wid, lane);
    };
    const int pro = (int)min<int64_t>(nst, G::RING - 1);
    for (int d = 0; d < pro; ++d) issue(d);
    // the row maxima have landed; the prologue's DMAs stay in flight
    if (pro == 3) p_vmcnt<3 * G::DPS>();
    else if (pro == 2) p_vmcnt<2 * G::DPS>();
    else if (pro == 1) p_vmcnt<G::DPS>();
    else p_vmcnt<0>();
    asm volatile("" : "+v"(rb_t), "+v"(rb_0), "+v"(rb_1));
    float s_a0 = pow2f(ka), s_a1 = s_a0;
    if constexpr (ROWS) {
      if (tid < kPBM) rsh[tid] = amax_shift(rb_t);  // read by the epilogue, after the loop's barriers
      if constexpr (!APS) {
        s_a0 = pow2f(amax_shift(rb_0));
        s_a1 = pow2f(amax_shift(rb_1));
      }
    }
    if constexpr (EX) {
      if (lds_rows && tid < kPBM) s_rmax[tid] = 0u;
    }

    f32x16 acc[2][2][2];  // [column half][32-row block i][32-column block]
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[h][i][j][r] = 0.f;

    // A fragment (two chunks) -> the two MFMA operands: the il8 image's planes as they are, or
    // the fp32 values split with the row's scale (the K tail's chunks past K zeroed first)
    auto a_ops = [&](const u32x4 (&c)[2], float s, bool tl, int64_t k0, f16x8& ah, f16x8& al) {
      if constexpr (APS) {
        ah = __builtin_bit_cast(f16x8, c[0]);
        al = __builtin_bit_cast(f16x8, c[1]);
      } else {
        float4 lo = __builtin_bit_cast(float4, c[0]), hi = __builtin_bit_cast(float4, c[1]);
        if (tl) {
          if (k0 + 8 * lk >= K) lo = make_float4(0.f, 0.f, 0.f, 0.f);
          if (k0 + 8 * lk + 4 >= K) hi = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        bf16x8 h, l;
        split2h8(lo, hi, s, h, l);
        ah = __builtin_bit_cast(f16x8, h);
        al = __builtin_bit_cast(f16x8, l);
      }
    };
    auto mfma3 = [](f32x16 c, const f16x8& ah, const f16x8& al, const u32x4& bh,
                    const u32x4& bl) -> f32x16 {
      if constexpr (ABL == 2) {
        asm volatile("" ::"v"(ah), "v"(al), "v"(bh), "v"(bl));
        return c;
      }
      const f16x8 bhv = __builtin_bit_cast(f16x8, bh), blv = __builtin_bit_cast(f16x8, bl);
      c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bhv, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, blv, c, 0, 0, 0);
      return __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bhv, c, 0, 0, 0);
    };
    // one 16-deep step u of the stage in slot base sb
    auto step16 = [&](uint32_t sb, int u, bool tl, int64_t k0) {
      const uint32_t vb0 = sb + ob + o0[u], vb1 = sb + ob + o1[u];
      const uint32_t va0 = sb + oa + o0[u], va1 = sb + oa + o1[u];
      constexpr int R = 32 * G::RB;  // one 32-row block
      u32x4 bh[4], bl[4], a[2];
      // B's four column blocks and A's first row block; A's second is read under the first's
      // MFMAs into the registers the first's split has freed
      p_rd<0>(bh[0], vb0);
      p_rd<0>(bl[0], vb1);
      p_rd<R>(bh[1], vb0);
      p_rd<R>(bl[1], vb1);
      p_rd<2 * R>(bh[2], vb0);
      p_rd<2 * R>(bl[2], vb1);
      p_rd<3 * R>(bh[3], vb0);
      p_rd<3 * R>(bl[3], vb1);
      p_rd<0>(a[0], va0);
      p_rd<0>(a[1], va1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      f16x8 ah, al;
      a_ops(a, s_a0, tl, k0, ah, al);
      __builtin_amdgcn_sched_barrier(0);
      p_rd<R>(a[0], va0);
      p_rd<R>(a[1], va1);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        acc[jj >> 1][0][jj & 1] = mfma3(acc[jj >> 1][0][jj & 1], ah, al, bh[jj], bl[jj]);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      a_ops(a, s_a1, tl, k0, ah, al);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        acc[jj >> 1][1][jj & 1] = mfma3(acc[jj >> 1][1][jj & 1], ah, al, bh[jj], bl[jj]);
      __builtin_amdgcn_sched_barrier(0);
    };
    auto stage = [&](int64_t t, bool tl) {
      const uint32_t sb = lds_b + (uint32_t)(t % G::RING) * G::STAGE;
#pragma unroll
      for (int u = 0; u < G::SUB; ++u) step16(sb, u, tl, t * BK + 16 * u);
    };
    // this wave's DMAs of stage t have landed (those of the stages after it may still fly);
    // after the barrier every wave's have, and every wave is done reading stage t - 1's slot
    auto wait_stage = [&](int64_t t) {
      const int64_t ahead = min<int64_t>(nst - 1 - t, G::RING - 2);
      if constexpr (G::RING > 2) {
        if (ahead >= 2) p_vmcnt<2 * G::DPS>();
        else if (ahead == 1) p_vmcnt<G::DPS>();
        else p_vmcnt<0>();
      } else {
        p_vmcnt<0>();
      }
      asm volatile("s_barrier" ::: "memory");
      if (t + G::RING - 1 < nst) issue(t + G::RING - 1);
    };
    for (int64_t t = 0; t + 1 < nst; ++t) {
      wait_stage(t);
      stage(t, false);
    }
    if (nst > 0) {  // the last stage (the K tail of an fp32 A: its chunks past K zeroed)
      wait_stage(nst - 1);
      stage(nst - 1, tail);
    }
    // every wave is past its last ring read before the ring becomes the epilogue's staging
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    {  // undo the scales (exact: powers of two); per-row A scales leave through rsh
      const float u = ROWS ? pow2f(-kb) : pow2f(-kb) * pow2f(-ka);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[h][i][j][r] = acc[h][i][j][r] * u;
    }
    if constexpr (ABL == 1) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(acc[h][i][j]));
      continue;
    }
    float* wl = reinterpret_cast<float*>(lds) + wid * 32 * kEpiLd;
    const int* rs = ROWS ? rsh + wm * 64 : nullptr;
    uint32_t* srm = lds_rows ? s_rmax + wm * 64 : nullptr;
    epilogue_lds<2, EX>(acc[0], wl, M, N, m0 + wm * 64, n0 + wn * 128, lane, bias, beta, act, C, ldc,
                        nullptr, cep, rs, ex, srm);
    wave_sync_lds();
    epilogue_lds<2, EX>(acc[1], wl, M, N, m0 + wm * 64, n0 + wn * 128 + 64, lane, bias, beta, act, C,
                        ldc, nullptr, cep, rs, ex, srm);
    if constexpr (EX) {
      if (lds_rows) {  // (uniform) one global atomicMax per row of the tile
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const int64_t slot = ex.rows_cols > 0 ? n0 / ex.rows_cols : 0;
        if (tid < kPBM && m0 + tid < M && s_rmax[tid] != 0u)
          atomicMax(ex.c_rows + slot * ex.rows_stride + m0 + tid, s_rmax[tid]);
      }
    }
  }
}

// Ping-pong form (PP, BK = 16, 4-slot ring): the 8 waves are two groups of four — waves 0-3
// (rows 0-127 of the tile) and 4-7 (rows 128-255), one wave of each on every SIMD — that run the
// same stage loop one phase apart, separated by workgroup barriers:
//   phase 2t:     group 0 reads stage t's fragments (and splits A) | group 1 runs stage t-1's MFMAs
//   phase 2t + 1: group 0 runs stage t's MFMAs                   | group 1 reads stage t
// so each SIMD's matrix core is fed by one group while the other group's LDS reads, A split and
// DMA issue run beside it (the one-group loop above alternates the whole CU between an LDS phase
// and an MFMA phase: its ablations add the two up).  Stage s is DMA'd at phase 2(s - 3) by every
// wave (its slot was last read by group 1 in phase 2s - 7), and every wave waits for its own
// pieces of stage t + 1 at the end of phase 2t + 1, before the barrier that opens group 0's read.
template <bool APS, bool ROWS, int ABL = 0>
__global__ void __launch_bounds__(kPThreads, 2)
gemm_planes_pp_kernel(int64_t M, int64_t N, int64_t K, const float* __restrict__ A, int64_t lda,
                      const float* __restrict__ B, int64_t ldb, const float* __restrict__ bias,
                      float beta, int act, float* __restrict__ C, int64_t ldc, AmaxPtrs amax) {
  constexpr int BK = 16;
  using G = PGeo<BK>;
  static_assert(G::RING == 4 && G::SUB == 1, "ping-pong: four 16-deep slots");
  __shared__ __attribute__((aligned(16))) uint8_t lds[G::RING_BYTES + kPBM * 4];
  int* rsh = reinterpret_cast<int*>(lds + G::RING_BYTES);
  const uint32_t lds_b = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2;
  const int wm = wid >> 1, wn = wid & 1;
  const int li = lane & 31, lk = lane >> 5;
  const int kb = amax_shift(*amax.b);
  const int ka = ROWS ? 0 : amax_shift(*amax.a);
  const int sw = G::swz(li);
  const uint32_t o0 = li * G::RB + 16 * ((2 * lk) ^ sw), o1 = li * G::RB + 16 * ((2 * lk + 1) ^ sw);
  const uint32_t oa = wm * 64 * G::RB, ob = G::OP + wn * 128 * G::RB;
  const int64_t nst = ceil_div(K, BK);
  const int64_t kmax_a = APS ? nst * BK - 4 : K - 4, kmax_b = nst * BK - 4;
  const int64_t tiles_n = ceil_div(N, kPBN);
  const int64_t n_tiles = ceil_div(M, kPBM) * tiles_n;
  const unsigned xq = n_tiles / 8, xr = n_tiles % 8, bx = blockIdx.x % 8;
  const int64_t t_beg = (bx < xr) ? bx * (xq + 1) : xr * (xq + 1) + (bx - xr) * xq;
  const int64_t t_end = t_beg + xq + (bx < xr ? 1 : 0);
  const unsigned bq = gridDim.x / 8, br = gridDim.x % 8;
  const int64_t t_step = bq + (bx < br ? 1 : 0);
  constexpr int R = 32 * G::RB;  // one 32-row block of a stage image
  for (int64_t tile = t_beg + blockIdx.x / 8; tile < t_end; tile += t_step) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int64_t m0 = (tile / tiles_n) * kPBM, n0 = (tile % tiles_n) * kPBN;
    uint32_t rb_t = 0, rb_0 = 0, rb_1 = 0;
    if constexpr (ROWS) {
      if (tid < kPBM) rb_t = p_ld_u32(amax.a_rows + min(m0 + tid, M - 1));
      if constexpr (!APS) {
        rb_0 = p_ld_u32(amax.a_rows + min(m0 + wm * 64 + li, M - 1));
        rb_1 = p_ld_u32(amax.a_rows + min(m0 + wm * 64 + 32 + li, M - 1));
      }
    }
    auto issue = [&](int64_t t) {
      if (t >= nst) return;
      uint8_t* st = lds + (t % G::RING) * G::STAGE;
      p_issue<BK>(A, lda, m0, M, t * BK, kmax_a, st, wid, lane);
      p_issue<BK>(B, ldb, n0, N, t * BK, kmax_b, st + G::OP, wid, lane);
    };
    // this wave's pieces of stage t have landed (stages after it, up to two, may still fly)
    auto wait_own = [&](int64_t t) {
      const int64_t ahead = min<int64_t>(nst - 1 - t, 2);
      if (ahead >= 2) p_vmcnt<2 * G::DPS>();
      else if (ahead == 1) p_vmcnt<G::DPS>();
      else p_vmcnt<0>();
    };
    issue(0);
    issue(1);
    issue(2);
    wait_own(0);  // (and the row maxima, issued before)
    asm volatile("" : "+v"(rb_t), "+v"(rb_0), "+v"(rb_1));
    float s_a0 = pow2f(ka), s_a1 = s_a0;
    if constexpr (ROWS) {
      if (tid < kPBM) rsh[tid] = amax_shift(rb_t);
      if constexpr (!APS) {
        s_a0 = pow2f(amax_shift(rb_0));
        s_a1 = pow2f(amax_shift(rb_1));
      }
    }
    f32x16 acc[2][2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[h][i][j][r] = 0.f;
    u32x4 bh[4], bl[4];
    f16x8 ah[2], al[2];
    auto a_ops = [&](const u32x4& c0, const u32x4& c1, float s, bool tl, int64_t k0, f16x8& h8, f16x8& l8) {
      if constexpr (APS) {
        h8 = __builtin_bit_cast(f16x8, c0);
        l8 = __builtin_bit_cast(f16x8, c1);
      } else {
        float4 lo = __builtin_bit_cast(float4, c0), hi = __builtin_bit_cast(float4, c1);
        if (tl) {
          if (k0 + 8 * lk >= K) lo = make_float4(0.f, 0.f, 0.f, 0.f);
          if (k0 + 8 * lk + 4 >= K) hi = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        bf16x8 h, l;
        split2h8(lo, hi, s, h, l);
        h8 = __builtin_bit_cast(f16x8, h);
        l8 = __builtin_bit_cast(f16x8, l);
      }
    };
    // READ phase: every fragment of stage t into registers, A split
    auto read = [&](int64_t t) {
      const uint32_t sb = lds_b + (uint32_t)(t % G::RING) * G::STAGE;
      const uint32_t vb0 = sb + ob + o0, vb1 = sb + ob + o1, va0 = sb + oa + o0, va1 = sb + oa + o1;
      u32x4 a[4];
      p_rd<0>(bh[0], vb0);
      p_rd<0>(bl[0], vb1);
      p_rd<R>(bh[1], vb0);
      p_rd<R>(bl[1], vb1);
      p_rd<2 * R>(bh[2], vb0);
      p_rd<2 * R>(bl[2], vb1);
      p_rd<3 * R>(bh[3], vb0);
      p_rd<3 * R>(bl[3], vb1);
      p_rd<0>(a[0], va0);
      p_rd<0>(a[1], va1);
      p_rd<R>(a[2], va0);
      p_rd<R>(a[3], va1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      const bool tl = !APS && t == nst - 1 && (K % BK) != 0;
      a_ops(a[0], a[1], s_a0, tl, t * BK, ah[0], al[0]);
      a_ops(a[2], a[3], s_a1, tl, t * BK, ah[1], al[1]);
      __builtin_amdgcn_sched_barrier(0);
    };
    // MFMA phase: the 24 products of the fragments read
    auto mfma = [&]() {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          f32x16 c = acc[jj >> 1][i][jj & 1];
          if constexpr (ABL == 2) {
            asm volatile("" ::"v"(ah[i]), "v"(al[i]), "v"(bh[jj]), "v"(bl[jj]));
          } else {
            const f16x8 bhv = __builtin_bit_cast(f16x8, bh[jj]), blv = __builtin_bit_cast(f16x8, bl[jj]);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bhv, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], blv, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bhv, c, 0, 0, 0);
          }
          acc[jj >> 1][i][jj & 1] = c;
        }
      __builtin_amdgcn_sched_barrier(0);
    };
    auto bar = [] { asm volatile("s_barrier" ::: "memory"); };
    bar();  // every wave's stage 0 has landed
    if (grp == 0) {
      for (int64_t t = 0; t < nst; ++t) {
        issue(t + 3);  // phase 2t: stage t + 3 into the slot group 1 left at the last barrier
        read(t);
        bar();
        mfma();  // phase 2t + 1
        if (t + 1 < nst) wait_own(t + 1);
        bar();
      }
      bar();  // group 1's last MFMA phase
    } else {
      issue(3);  // phase 0
      bar();
      for (int64_t t = 0; t < nst; ++t) {
        read(t);  // phase 2t + 1
        if (t + 1 < nst) wait_own(t + 1);
        bar();
        issue(t + 4);  // phase 2t + 2
        mfma();
        bar();
      }
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    {
      const float u = ROWS ? pow2f(-kb) : pow2f(-kb) * pow2f(-ka);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[h][i][j][r] = acc[h][i][j][r] * u;
    }
    if constexpr (ABL == 1) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(acc[h][i][j]));
      continue;
    }
    float* wl = reinterpret_cast<float*>(lds) + wid * 32 * kEpiLd;
    const int* rs = ROWS ? rsh + wm * 64 : nullptr;
    epilogue_lds<2, false>(acc[0], wl, M, N, m0 + wm * 64, n0 + wn * 128, lane, bias, beta, act, C, ldc,
                           nullptr, CellEpi{}, rs);
    wave_sync_lds();
    epilogue_lds<2, false>(acc[1], wl, M, N, m0 + wm * 64, n0 + wn * 128 + 64, lane, bias, beta, act, C,
                           ldc, nullptr, CellEpi{}, rs);
  }
}

// 16x16x32 form (M16, BK = 32, experiment): the same staging and stage images as BK = 32, the
// products on v_mfma_f32_16x16x32_f16 (lane l: A row l & 15, k 8 (l >> 4) .. + 7; C rows
// 4 (l >> 4) + r, column l & 15), 4 x 8 blocks of 16 x 16 per wave.  The point of the shape:
// under load the chip holds a higher clock on 16x16x32 than on 32x32x16 MFMA streams of equal
// cycles (MI355X_MICROARCH.md, DVFS (7): 1.12-1.15 x the FLOP/s).  Direct epilogue (per-row and
// operand scales, bias, beta, ReLU; 64-B row pieces).  The k order inside an MFMA differs from
// the 32x32x16 tile's, so results agree to rounding, not bitwise.
template <bool APS, bool ROWS>
__global__ void __launch_bounds__(kPThreads, 2)
gemm_planes16_kernel(int64_t M, int64_t N, int64_t K, const float* __restrict__ A, int64_t lda,
                     const float* __restrict__ B, int64_t ldb, const float* __restrict__ bias,
                     float beta, int act, float* __restrict__ C, int64_t ldc, AmaxPtrs amax) {
  constexpr int BK = 32;
  using G = PGeo<BK>;
  __shared__ __attribute__((aligned(16))) uint8_t lds[G::RING_BYTES];
  const uint32_t lds_b = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int lr = lane & 15, lg = lane >> 4;
  const int kb = amax_shift(*amax.b);
  const int ka = ROWS ? 0 : amax_shift(*amax.a);
  // lane's two 16-B chunks (k group lg: chunks 2 lg, 2 lg + 1) of row lr of a 16-row block; the
  // stage images are swizzled per row as for BK = 32 (chunk ^ ((row >> 1) & 7)); blocks of 16
  // rows keep (row >> 1) & 7 of rows 16 b + lr equal to that of lr
  const int sw = G::swz(lr);
  const uint32_t o0 = lr * G::RB + 16 * ((2 * lg) ^ sw), o1 = lr * G::RB + 16 * ((2 * lg + 1) ^ sw);
  const uint32_t oa = wm * 64 * G::RB, ob = G::OP + wn * 128 * G::RB;
  const int64_t nst = ceil_div(K, BK);
  const int64_t kmax_a = APS ? nst * BK - 4 : K - 4, kmax_b = nst * BK - 4;
  const bool tail = !APS && (K % BK) != 0;
  const int64_t tiles_n = ceil_div(N, kPBN);
  const int64_t n_tiles = ceil_div(M, kPBM) * tiles_n;
  const unsigned xq = n_tiles / 8, xr = n_tiles % 8, bx = blockIdx.x % 8;
  const int64_t t_beg = (bx < xr) ? bx * (xq + 1) : xr * (xq + 1) + (bx - xr) * xq;
  const int64_t t_end = t_beg + xq + (bx < xr ? 1 : 0);
  const unsigned bq = gridDim.x / 8, br = gridDim.x % 8;
  const int64_t t_step = bq + (bx < br ? 1 : 0);
  constexpr int R16 = 16 * G::RB;  // one 16-row block of a stage image
  for (int64_t tile = t_beg + blockIdx.x / 8; tile < t_end; tile += t_step) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int64_t m0 = (tile / tiles_n) * kPBM, n0 = (tile % tiles_n) * kPBN;
    uint32_t rbv[4] = {0u, 0u, 0u, 0u};  // this lane's A rows 16 i + lr (split scales)
    if constexpr (ROWS) {
#pragma unroll
      for (int i = 0; i < 4; ++i) rbv[i] = p_ld_u32(amax.a_rows + min(m0 + wm * 64 + 16 * i + lr, M - 1));
    }
    auto issue = [&](int64_t t) {
      uint8_t* st = lds + (t % G::RING) * G::STAGE;
      p_issue<BK>(A, lda, m0, M, t * BK, kmax_a, st, wid, lane);
      p_issue<BK>(B, ldb, n0, N, t * BK, kmax_b, st + G::OP, wid, lane);
    };
    issue(0);
    p_vmcnt<0>();  // stage 0 and the row maxima
    asm volatile("" : "+v"(rbv[0]), "+v"(rbv[1]), "+v"(rbv[2]), "+v"(rbv[3]));
    float sa[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) sa[i] = ROWS ? pow2f(amax_shift(rbv[i])) : pow2f(ka);
    f32x4 acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto stage = [&](int64_t t, bool tl) {
      const uint32_t sb = lds_b + (uint32_t)(t % G::RING) * G::STAGE;
      // A's four 16-row blocks first (split once), then B in two halves of four 16-column
      // blocks (32 VGPRs of B fragments live instead of 64)
      f16x8 ah[4], al[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        u32x4 c0, c1;
        asm volatile("ds_read_b128 %0, %1" : "=v"(c0) : "v"(sb + oa + o0 + i * R16) : "memory");
        asm volatile("ds_read_b128 %0, %1" : "=v"(c1) : "v"(sb + oa + o1 + i * R16) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (APS) {
          ah[i] = __builtin_bit_cast(f16x8, c0);
          al[i] = __builtin_bit_cast(f16x8, c1);
        } else {
          float4 lo = __builtin_bit_cast(float4, c0), hi = __builtin_bit_cast(float4, c1);
          if (tl) {
            if (t * BK + 8 * lg >= K) lo = make_float4(0.f, 0.f, 0.f, 0.f);
            if (t * BK + 8 * lg + 4 >= K) hi = make_float4(0.f, 0.f, 0.f, 0.f);
          }
          bf16x8 h, l;
          split2h8(lo, hi, sa[i], h, l);
          ah[i] = __builtin_bit_cast(f16x8, h);
          al[i] = __builtin_bit_cast(f16x8, l);
        }
      }
#pragma unroll
      for (int jh = 0; jh < 2; ++jh) {
        u32x4 bh[4], bl[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t vb0 = sb + ob + o0 + (4 * jh + j) * R16, vb1 = sb + ob + o1 + (4 * jh + j) * R16;
          asm volatile("ds_read_b128 %0, %1" : "=v"(bh[j]) : "v"(vb0) : "memory");
          asm volatile("ds_read_b128 %0, %1" : "=v"(bl[j]) : "v"(vb1) : "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f16x8 bhv = __builtin_bit_cast(f16x8, bh[j]), blv = __builtin_bit_cast(f16x8, bl[j]);
            f32x4 c = acc[i][4 * jh + j];
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bhv, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], blv, c, 0, 0, 0);
            acc[i][4 * jh + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bhv, c, 0, 0, 0);
          }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    for (int64_t t = 0; t < nst; ++t) {
      // stage t landed for this wave; after the barrier, for every wave, and stage t - 1's slot
      // is free: stage t + 1 goes into it
      p_vmcnt<0>();
      asm volatile("s_barrier" ::: "memory");
      if (t + 1 < nst) issue(t + 1);
      stage(t, tail && t == nst - 1);
    }
    // direct epilogue: lane's rows 16 i + 4 lg + r, column 16 j + lr of the wave's 64 x 128
    const float ub = pow2f(-kb) * (ROWS ? 1.f : pow2f(-ka));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 64 + 16 * i + 4 * lg + r;
        if (row >= M) continue;
        float us = ub;
        if constexpr (ROWS) us *= pow2f(-amax_shift(amax.a_rows[row]));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int64_t col = n0 + wn * 128 + 16 * j + lr;
          if (col >= N) continue;
          float v = acc[i][j][r] * us;
          if (bias) v += bias[col];
          float* cp = C + row * ldc + col;
          if (beta != 0.f) v += beta * (*cp);
          if (act == 1) v = fmaxf(v, 0.f);
          *cp = v;
        }
      }
    }
  }
}

// il8 image of a K-contiguous ([rows][ld]) or K-major ([K][ld], kmajor) fp32 operand: out[r]
// holds, per 8-value k group g < ld_out / 8, the 8 scaled high halves of x[r][8g .. 8g+7] then
// the 8 low halves (split2h8 with the operand's scale, or the row's own with amax_rows); k >= K
// reads as zero, so the image is zero-padded to ld_out.
__global__ void __launch_bounds__(256) split_il8_kernel(int64_t rows, int64_t K, const float* __restrict__ P,
                                                        int64_t ld, int kmajor, int vec,
                                                        const uint32_t* __restrict__ amax,
                                                        const uint32_t* __restrict__ amax_rows,
                                                        float* __restrict__ out, int64_t ld_out) {
  const int64_t G = ld_out / 8, total = rows * G;
  const float s_all = amax ? pow2f(amax_shift(*amax)) : 1.f;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    int64_t r, g;
    if (kmajor) {  // consecutive threads take consecutive rows (coalesced k-row reads)
      g = e / rows;
      r = e - g * rows;
    } else {
      r = e / G;
      g = e - r * G;
    }
    const int64_t k = 8 * g;
    float v[8];
    if (!kmajor && vec && k + 8 <= K) {
      const float4 x0 = *reinterpret_cast<const float4*>(P + r * ld + k);
      const float4 x1 = *reinterpret_cast<const float4*>(P + r * ld + k + 4);
      v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
      v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        v[i] = k + i < K ? (kmajor ? P[(k + i) * ld + r] : P[r * ld + k + i]) : 0.f;
    }
    const float s = amax_rows ? pow2f(amax_shift(amax_rows[r])) : s_all;
    bf16x8 h, l;
    split2h8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), s, h, l);
    float* dst = out + r * ld_out + k;
    *reinterpret_cast<float4*>(dst) = __builtin_bit_cast(float4, h);
    *reinterpret_cast<float4*>(dst + 4) = __builtin_bit_cast(float4, l);
  }
}

}  // namespace
}  // namespace mvml

using namespace mvml;

extern "C" int mvml_split_f16x2_il8(int64_t rows, int64_t K, const float* P, int64_t ld, int kmajor,
                                    const uint32_t* amax, const uint32_t* amax_rows, float* out,
                                    int64_t ld_out, void* stream) {
  clear_error();
  MVML_REQUIRE(rows >= 0 && K >= 0 && ld_out >= ((K + 31) / 32) * 32 && ld_out % 8 == 0 && out &&
                   ((uintptr_t)out % 16) == 0 && (amax != nullptr) != (amax_rows != nullptr) &&
                   (kmajor ? ld >= rows : ld >= K),
               "split_f16x2_il8: bad shape / alignment, or not exactly one of amax / amax_rows");
  if (rows == 0 || ld_out == 0) return MVML_OK;
  const int vec = !kmajor && ld % 4 == 0 && ((uintptr_t)P % 16) == 0;
  const int64_t total = rows * (ld_out / 8);
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(total, 256), 16384);
  split_il8_kernel<<<blocks, 256, 0, as_stream(stream)>>>(rows, K, P, ld, kmajor, vec, amax, amax_rows,
                                                           out, ld_out);
  return check_launch("split_il8_kernel");
}

extern "C" int mvml_gemm_f16x2_planes(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                                      int a_image, const uint32_t* amax_a, const uint32_t* amax_a_rows,
                                      const float* b_image, int64_t ldb, const uint32_t* amax_b,
                                      const float* bias, float beta, int act, float* C, int64_t ldc,
                                      void* stream) {
  clear_error();
  MVML_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm_f16x2_planes: negative shape");
  MVML_REQUIRE(amax_b && ((amax_a != nullptr) != (amax_a_rows != nullptr)),
               "gemm_f16x2_planes: amax_b and exactly one of amax_a / amax_a_rows are required");
  MVML_REQUIRE(act == 0 || act == 1, "gemm_f16x2_planes: act must be 0 or 1");
  const int64_t kp = ((K + 31) / 32) * 32;
  MVML_REQUIRE(ldc >= N && ldb >= kp && ldb % 4 == 0 && (a_image ? lda >= kp : (lda >= K && K % 4 == 0)) &&
                   lda % 4 == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)b_image % 16) == 0,
               "gemm_f16x2_planes: needs 16-B aligned rows, K %% 4 == 0 and images padded to K rounded "
               "up to 16");
  if (M == 0 || N == 0) return MVML_OK;
  const int64_t tiles = ceil_div(M, kPBM) * ceil_div(N, kPBN);
  MVML_REQUIRE(tiles < (int64_t(1) << 31), "gemm_f16x2_planes: too many tiles");
  int persist = option(MVML_OPT_GEMM_PERSIST);
  persist = persist <= 0 ? 256 : (persist + 7) / 8 * 8;
  const unsigned grid = (unsigned)std::min<int64_t>(tiles, persist);
  AmaxPtrs am;
  am.a = amax_a;
  am.b = amax_b;
  am.a_rows = amax_a_rows;
  hipStream_t st = as_stream(stream);
  // experiment switches, read per call (tools/planes_bench.py, tests/test_gpu_planes.py):
  // MVML_PLANES_ABL timing ablations (1 no epilogue, 2 no MFMAs: wrong results),
  // MVML_PLANES_BK stage depth 16 / 32, MVML_PLANES_PP ping-pong wave groups (BK 16)
  auto env_int = [](const char* k, int d) {
    const char* e = getenv(k);
    return e ? atoi(e) : d;
  };
  const int abl = env_int("MVML_PLANES_ABL", 0);
  const int bk = env_int("MVML_PLANES_BK", 32);
  const int pp = env_int("MVML_PLANES_PP", 0);
  if (env_int("MVML_PLANES_M16", 0)) {
    if (a_image) {
      if (amax_a_rows) gemm_planes16_kernel<true, true><<<grid, kPThreads, 0, st>>>(M, N, K, A, lda, b_image, ldb, bias, beta, act, C, ldc, am);
      else gemm_planes16_kernel<true, false><<<grid, kPThreads, 0, st>>>(M, N, K, A, lda, b_image, ldb, bias, beta, act, C, ldc, am);
    } else {
      if (amax_a_rows) gemm_planes16_kernel<false, true><<<grid, kPThreads, 0, st>>>(M, N, K, A, lda, b_image, ldb, bias, beta, act, C, ldc, am);
      else gemm_planes16_kernel<false, false><<<grid, kPThreads, 0, st>>>(M, N, K, A, lda, b_image, ldb, bias, beta, act, C, ldc, am);
    }
    return check_launch("gemm_planes16_kernel");
  }
  if (pp) {
#define MVML_PP(APSV, ROWSV)                                                                           \
  do {                                                                                                 \
    if (abl == 1) gemm_planes_pp_kernel<APSV, ROWSV, 1><<<grid, kPThreads, 0, st>>>(                   \
        M, N, K, A, lda, b_image, ldb, bias, beta, act, C, ldc, am);                                   \
    else if (abl == 2) gemm_planes_pp_kernel<APSV, ROWSV, 2><<<grid, kPThreads, 0, st>>>(              \
        M, N, K, A, lda, b_image, ldb, bias, beta, act, C, ldc, am);                                   \
    else gemm_planes_pp_kernel<APSV, ROWSV, 0><<<grid, kPThreads, 0, st>>>(                            \
        M, N, K, A, lda, b_image, ldb, bias, beta, act, C, ldc, am);                                   \
  } while (0)
    if (a_image) {
      if (amax_a_rows) MVML_PP(true, true);
      else MVML_PP(true, false);
    } else {
      if (amax_a_rows) MVML_PP(false, true);
      else MVML_PP(false, false);
    }
#undef MVML_PP
    return check_launch("gemm_planes_pp_kernel");
  }
#define MVML_PL4(APSV, ROWSV, BKV, ABLV)                                                             \
  gemm_planes_kernel<APSV, ROWSV, false, false, BKV, ABLV><<<grid, kPThreads, 0, st>>>(               \
      M, N, K, A, lda, b_image, ldb, bias, beta, act, C, ldc, am, CellEpi{}, EpiX{})
#define MVML_PL3(APSV, ROWSV, BKV)                                 \
  do {                                                             \
    if (abl == 1 && ROWSV) MVML_PL4(APSV, ROWSV, BKV, 1);          \
    else if (abl == 2 && ROWSV) MVML_PL4(APSV, ROWSV, BKV, 2);     \
    else MVML_PL4(APSV, ROWSV, BKV, 0);                            \
  } while (0)
#define MVML_PL(APSV, ROWSV)                  \
  do {                                        \
    if (bk == 16) MVML_PL3(APSV, ROWSV, 16);  \
    else MVML_PL3(APSV, ROWSV, 32);           \
  } while (0)
  if (a_image) {
    if (amax_a_rows) MVML_PL(true, true);
    else MVML_PL(true, false);
  } else {
    if (amax_a_rows) MVML_PL(false, true);
    else MVML_PL(false, false);
  }
#undef MVML_PL
#undef MVML_PL3
#undef MVML_PL4
  return check_launch("gemm_planes_kernel");
}
