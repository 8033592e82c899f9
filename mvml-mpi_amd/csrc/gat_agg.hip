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
// el / er come from the projection GEMM (2H extra columns, elr); the edge_softmax runs inside
// the aggregation kernels (softmax_pair: one thread per destination and head, before the column
// sweep), so mvml_gat_agg_fwd is one launch per kernel kind and attn is written, never re-read.
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
// explicit roundings: with the device default -ffp-contract=fast the compiler would pick the
// contraction per call site, so kernels that promise the same dots bitwise could differ
__device__ __forceinline__ float dot4(float4 a, float4 b) {
  return __fmaf_rn(a.w, b.w, __fmaf_rn(a.z, b.z, __fmaf_rn(a.y, b.y, __fmul_rn(a.x, b.x))));
}
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
// streaming (non-temporal) 16-B load / store: rows read or written exactly once pass through
// without displacing the rows an XCD's waves share in L2
typedef float mvml_f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld4nt(const float* p) {
  const mvml_f4v v = __builtin_nontemporal_load(reinterpret_cast<const mvml_f4v*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st4nt(float* p, float4 v) {
  mvml_f4v w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<mvml_f4v*>(p));
}

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

// |max| bookkeeping of the backward's gY stores (the split-fp16 scale of the GEMMs that read gY)
__device__ __forceinline__ float amax4(float m, float4 v) {
  return fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
}
// Block |max| -> one unsigned atomicMax of the (non-negative) float bits: order-independent.
// Every thread of the block calls it (a barrier inside).
template <int NT>
__device__ __forceinline__ void block_amax_commit(float m, uint32_t* out) {
  __shared__ float red[NT / 64];
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = red[0];
#pragma unroll
    for (int i = 1; i < NT / 64; ++i) r = fmaxf(r, red[i]);
    atomicMax(out, __float_as_uint(r));
  }
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
// Logits: el[n,h] = <Z[n,h,:], attn_l[h,:]>, er likewise.  The projection GEMM's epilogue leaves
// per-W-column partial dots part[g][side][n]; this sums a head's F/32 blocks in order and
// writes the compact elr[n] = [el | er] (the softmax's gathers and the backward read it).
template <int H>
__global__ void __launch_bounds__(256)
gat_logits_finalize_kernel(int64_t N, int F, int W, const float* __restrict__ part,
                           float* __restrict__ elr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over N * 2H
  if (i >= N * 2 * H) return;
  const int64_t v = i % N;           // node-fastest: coalesced partial reads
  const int sh = (int)(i / N);        // side * H + h
  const int side = sh / H, h = sh % H;
  const int nbh = F / W;
  const float* p = part + ((int64_t)(h * nbh) * 2 + side) * N + v;  // [group][side][node]
  float acc = p[0];
  for (int b = 1; b < nbh; ++b) acc += p[(int64_t)b * 2 * N];
  elr[v * 2 * H + sh] = acc;
}

// edge_softmax of one (destination v, head h) pair inside the aggregation kernels (the same
// arithmetic and order as the round-3 standalone softmax kernel: max over the in-edges, sum of
// exp(s - max) in edge order, a_e = exp(s_e - max) / sum): writes attn[e, h] (the backward's
// input) and, when s_att is given, the group-relative copy s_att[(e - e0) H + h] the aggregation
// reads.  Logits past the register cache are recomputed in each pass (one more read of the
// L2-resident el rows; no limit on the degree).
template <int H>
__device__ __forceinline__ void softmax_pair(int64_t v, int h, const int32_t* __restrict__ rowptr,
                                             const int32_t* __restrict__ in_src,
                                             const float* __restrict__ elr, float slope,
                                             float* __restrict__ attn, float* s_att, int e0) {
  const float er = elr[v * 2 * H + H + h];
  const int eb = rowptr[v], ee = rowptr[v + 1];
  constexpr int DC = 6;
  float sc[DC];
  float m = -INFINITY, sum = 0.f;
#pragma unroll
  for (int t = 0; t < DC; ++t) {
    sc[t] = (eb + t < ee) ? leaky(elr[(int64_t)in_src[eb + t] * 2 * H + h] + er, slope) : -INFINITY;
    m = fmaxf(m, sc[t]);
  }
  for (int e = eb + DC; e < ee; ++e) m = fmaxf(m, leaky(elr[(int64_t)in_src[e] * 2 * H + h] + er, slope));
#pragma unroll
  for (int t = 0; t < DC; ++t)
    if (eb + t < ee) sum += expf(sc[t] - m);
  for (int e = eb + DC; e < ee; ++e) sum += expf(leaky(elr[(int64_t)in_src[e] * 2 * H + h] + er, slope) - m);
#pragma unroll
  for (int t = 0; t < DC; ++t)
    if (eb + t < ee) {
      const float a = expf(sc[t] - m) / sum;
      attn[(int64_t)(eb + t) * H + h] = a;
      if (s_att) s_att[(eb + t - e0) * H + h] = a;
    }
  for (int e = eb + DC; e < ee; ++e) {
    const float a = expf(leaky(elr[(int64_t)in_src[e] * 2 * H + h] + er, slope) - m) / sum;
    attn[(int64_t)e * H + h] = a;
    if (s_att) s_att[(e - e0) * H + h] = a;
  }
}

// Aggregation over NODE GROUPS.  A node group is a contiguous range of whole molecules of about
// kNodeGroupAtoms atoms (mvml_build_node_groups); edges never leave a molecule, so every in-edge
// of a group's atoms has its source inside the group, and one workgroup per group can read each
// projection row from HBM once.  The attention comes from softmax_pair.  The projection
// columns are swept CW at a time; CW/4 lanes own one destination atom (16-B column slices).
// Flatten modes walk the chunks head-major; the mean mode walks them f-chunk-major, head-minor,
// summing the heads in registers (+ bias per head, / H, + head-mean residual).
//
// Two kernels share the groups (each block decides with the same block-wide predicate):
//  * gat_agg_fwd_lds_kernel — the molecule case: a group of <= kWinL atoms, <= kECap in-edges,
//    in-degree <= kEC everywhere (organic atoms: 4 bonds + self-loop).  The group's rows are
//    streamed ONCE into an LDS double buffer through a register ring two chunks deep (chunks
//    k+1, k+2 and the next residual in flight while chunk k is aggregated, one barrier per
//    chunk); the kEC source-row LDS offsets of every destination are cached in registers, so a
//    chunk's gathers are kEC x NP independent ds_read_b128 (branch-free: a missing edge reads
//    the destination's own row and is discarded by a select) — one LDS round trip per chunk.
//  * gat_agg_fwd_gather_kernel — everything else (large molecules, hubs): no staging; the
//    gathers go straight to global memory, where the chunk-synchronous sweep keeps the group's
//    chunk rows in the XCD's L2.  Correct for any graph.
// Which kernel takes a group is decided once per batch by mvml_build_node_groups (the group
// plan: kind bits + fallback lists), so no launch scans the CSR to find its groups.
constexpr int kWinL = kPlanWinAtoms;  // LDS kernel: atoms per group
constexpr int kECap = kPlanEdgeCap;   // LDS kernel: in-edges per group (attention staged in LDS)
constexpr int kWin = 64;              // gather kernel: destination atoms per pass set
constexpr int kEC = kPlanDegCap;      // in-edges per destination with cached offsets
constexpr int kAggThreads = 512;
constexpr int kHubDeg = 16;           // gather kernel: in-degree above which the hub pass runs
constexpr int kHubCols = 1024;        // gather kernel: float4 columns of the hub pass (H*F <= 4096)
// Fallback-list entry of block b in a grid of nb >= count blocks: XCD x (the blocks b % 8 == x)
// walks ONE contiguous range of the list (the lists are in group order), so the molecules in
// flight on an XCD are neighbours and their rows share its L2; -1 for idle blocks.
__device__ __forceinline__ int list_block(unsigned b, unsigned nb, int count) {
  const unsigned x = b % 8, i = b / 8;
  const unsigned q = count / 8, r = count % 8;
  const unsigned beg = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  const unsigned len = q + (x < r ? 1 : 0);
  return i < len ? (int)(beg + i) : -1;
}
constexpr int kBigThreads = 512;      // big-window kernels: 128 rows per pass (16-column chunks),
                                      // up to 4 passes; 2 waves per SIMD leave 256 registers
constexpr int kBigBlocks = 256;       // ... one workgroup per CU walking the fallback list
// Hub segments of a big window: the edges of a row past its kEC cached ones are cut into
// segments of kSegI in-edges (kSegO out-edges), each one a task for any lane group of the chunk
// sweep (a partial sum / edge dots), so a hub's 32-128 edges cost one LDS round trip per chunk
// instead of a serial walk on its own lanes.  Rows whose segments would pass the table keep the
// serial walk (correct for any graph; the tables cover config 5's 1-4 hubs per molecule).  The
// backward's out-edge partials are short of LDS: there rows of out-degree <= kSegMinO (a hub's
// partners: one or two edges past kEC, staged in s_oxe) walk theirs too.
constexpr int kSegI = 8, kSegO = 16, kSegMinO = 12;
constexpr int kSegCapI = 256, kSegCapO = 48;
constexpr int kOXCap = 640;  // backward: out-edges past kEC staged in LDS (dst row << 16 | slot)

// Block-wide exclusive prefix sum of one int per thread (NT / 64 waves); *total = the sum.
template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int* s_wsum, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_wsum[w] = x;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    const int t = s_wsum[i];
    base += i < w ? t : 0;
    tot += t;
  }
  *total = tot;
  return base + x - v;
}

// The segment table of rows d = threadIdx.x < nr (edge range [eb, eb + deg) of the window's
// CSR; rows of degree <= MIN get none): seg[t] = row << 16 | first edge << 4 | (count - 1);
// *rs = first segment | count << 12 for this thread's row (0: no segments, or segments past
// CAP: the owner walks them).  Returns the table length.  Ends with a barrier (the table is
// visible to the block).
template <int NT, int SEG, int CAP, int MIN = kEC>
__device__ __forceinline__ int hub_segments(int nr, int eb, int deg, uint32_t* s_seg, int* rs,
                                            int* s_wsum) {
  static_assert(CAP < 4096 && SEG <= 16, "segment packing");
  const int d = threadIdx.x;
  int n = (d < nr && deg > MIN) ? (deg - kEC + SEG - 1) / SEG : 0;
  int total;
  const int sb = block_excl_scan<NT>(n, s_wsum, &total);
  if (sb + n > CAP) n = 0;  // rows are in order: every later row is past the table too
  for (int j = 0; j < n; ++j) {
    const int e = eb + kEC + SEG * j;
    s_seg[sb + j] = (uint32_t)d << 16 | (uint32_t)e << 4 | (uint32_t)(min(SEG, eb + deg - e) - 1);
  }
  *rs = n ? (sb | n << 12) : 0;
  // the table length: the end of the last row that fits (a block max over the rows)
  const int end = n ? sb + n : 0;
  int m = end;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
  __syncthreads();  // s_wsum reads of the scan are done
  if ((threadIdx.x & 63) == 0) s_wsum[threadIdx.x >> 6] = m;
  __syncthreads();
  int len = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) len = max(len, s_wsum[i]);
  __syncthreads();  // s_wsum reusable
  return len;
}

// The big-window kernels stage 16-column chunks (F % 16 == 0) and their LDS holds the per-edge
// attention of up to kPlanBigEdgeCap edges for H <= 4 heads.  On config 5 (8192 molecules) they
// take fwd / bwd L1 6.4 / 13.5 ms and L2 7.0 / 21.7 ms against the per-atom fallbacks' 7.0 /
// 15.9 and 10.2 / 29.7 ms.  Option MVML_OPT_BIG_WINDOW = 0 routes those groups to the
// fallbacks (tests).
inline bool use_big_window(int H, int F) {
  return option(MVML_OPT_BIG_WINDOW) != 0 && H <= 4 && F % 16 == 0;
}

#ifndef MVML_LDS_WAVES
#define MVML_LDS_WAVES 4
#endif
#ifndef MVML_FWD_RING
#define MVML_FWD_RING 2
#endif
// Chunk loop of the forward LDS kernel for a group of at most NPA * DPP atoms (NPA passes of
// DPP destinations).  Chunks k+1 .. k+RING are in flight in a register ring while chunk k is
// aggregated from LDS.  Loads are unconditional (rows past the group read 0 through the buffer
// resource's range check; chunks past the end use an out-of-range offset), so the loop is
// straight-line and the compiler's vmcnt waits are exact; stores of rows past the group are
// skipped (an out-of-range store is not free).
template <int H, int CW, int MODE, int NT, int NPA, int WIN = kWinL, int ECAP = kECap, bool BIG = false>
__device__ __forceinline__ float fwd_lds_chunks(float4 (*zbuf)[WIN * (CW / 4)], const float* s_att,
                                               const int32_t* __restrict__ rowptr,
                                               const int32_t* __restrict__ in_src,
                                               __amdgpu_buffer_rsrc_t rY, uint32_t rowb,
                                               __amdgpu_buffer_rsrc_t rO, int a0, int nr, int e0,
                                               int F, const float* __restrict__ bias,
                                               const uint16_t* s_srcs = nullptr,
                                               const uint32_t* s_seg = nullptr,
                                               const int* s_rs = nullptr, float4* s_part = nullptr,
                                               int nseg = 0, uint32_t* __restrict__ out_rows = nullptr) {
  constexpr int LPD = CW / 4;                        // lanes per destination atom
  constexpr int DPP = NT / LPD;                      // destinations per pass
  constexpr int RING = NPA >= 3 ? 1 : MVML_FWD_RING;  // 3-4 pass groups: registers
  const int tid = threadIdx.x;
  const int ds = tid / LPD, q = tid % LPD;
  const int HF = H * F;
  const int nfc = F / CW;     // column chunks per head
  const int nch = H * nfc;
  const int ocols = MODE == 1 ? F : HF;
  // this thread's destinations: the LDS slots of their first kEC source rows and attention
  // values; a missing edge (i >= in-degree) points at the destination's own row and at a zero
  // attention, so the edge loop is branch- and mask-free (fma(0, z, acc) == acc)
  int so[NPA][kEC], ab[NPA], ad[NPA];
  uint32_t rb[NPA], ob[NPA];  // byte offsets of this thread's rows in Y and in out
  // "no access" offsets: just past the resource's range (reads 0, drops stores) yet next to
  // the group's own rows, so the address still translates through a warm TLB entry (a wild
  // out-of-range offset costs a page walk per access)
  const uint32_t noY = (uint32_t)nr * rowb;
  float omx = 0.f;  // |max| of this thread's output stores (live rows)
  float rmx[NPA];   // ... per destination (out_rows: each row's |max|, the next GEMM's row scale)
  bool live[NPA];
#pragma unroll
  for (int p = 0; p < NPA; ++p) {
    const int d = ds + DPP * p;
    live[p] = d < nr;
    int eb = 0, deg = 0;
    if (live[p]) {
      eb = rowptr[a0 + d] - e0;
      deg = rowptr[a0 + d + 1] - e0 - eb;
    }
    ab[p] = eb * H;
    ad[p] = deg;
    rmx[p] = 0.f;
#pragma unroll
    for (int i = 0; i < kEC; ++i) {
      so[p][i] = ((i < deg) ? in_src[e0 + eb + i] - a0 : (live[p] ? d : 0)) * LPD + q;
    }
    rb[p] = (uint32_t)d * rowb;            // d >= nr: past the resource, reads 0
    ob[p] = 4u * (uint32_t)(d * ocols);
  }
  // BIG: this thread's rows' hub segments (first | count << 12); the edges of a row with none
  // past kEC are walked by the row's own lanes (hend)
  int sbn[NPA], hend[NPA];
#pragma unroll
  for (int p = 0; p < NPA; ++p) {
    sbn[p] = 0;
    if constexpr (BIG) sbn[p] = live[p] ? s_rs[ds + DPP * p] : 0;
    hend[p] = sbn[p] ? kEC : ad[p];
  }
  // chunk k -> global column of this lane
  auto col_of = [&](int k) {
    return (MODE == 1 ? (k % H) * F + (k / H) * CW : (k / nfc) * F + (k % nfc) * CW) + 4 * q;
  };
  auto load_rows = [&](int k, float4 (&dst)[NPA]) {
    const bool ok = k < nch;
    const uint32_t cb = 4u * (uint32_t)col_of(k);
#pragma unroll
    for (int j = 0; j < NPA; ++j) dst[j] = buf_ld4(rY, ok ? rb[j] + cb : noY);
  };
  // residual of chunk k (mean mode: of its f-chunk, re-read per head from L2 so that the loop
  // stays branch-free; loading it for the last head only measured slower, L2 mean 3.86 -> 4.20 ms)
  auto load_res = [&](int k, float4 (&dst)[NPA]) {
    const bool ok = k < nch;
    const uint32_t cb = 4u * (uint32_t)(HF + (MODE == 1 ? (k / H) * CW + 4 * q : col_of(k)));
#pragma unroll
    for (int j = 0; j < NPA; ++j) dst[j] = buf_ld4(rY, ok ? rb[j] + cb : noY);
  };
  auto store_rows = [&](int buf, const float4 (&src)[NPA]) {
#pragma unroll
    for (int j = 0; j < NPA; ++j) zbuf[buf][(ds + DPP * j) * LPD + q] = src[j];
  };
  // BIG emits after the barrier: chunk k's residual is loaded at the top of iteration k (no
  // second residual set in registers)
  float4 ring[RING][NPA], rres[NPA], rnx[BIG ? 1 : NPA], tot[NPA];
  {
    float4 z0[NPA];
    load_rows(0, z0);
#pragma unroll
    for (int i = 0; i < RING; ++i) load_rows(1 + i, ring[i]);
    if constexpr (!BIG) load_res(0, rres);
    store_rows(0, z0);
  }
  __syncthreads();  // chunk 0 and s_att staged
  for (int k = 0; k < nch; ++k) {
    const int h = MODE == 1 ? k % H : k / nfc;
    const int col = col_of(k);
    if constexpr (BIG) load_res(k, rres);
    else load_res(k + 1, rnx);
    const float4 b4 = ld4(bias + col);
    const float4* zl = zbuf[k & 1];
    float4 acc[NPA];
#pragma unroll
    for (int p = 0; p < NPA; ++p) acc[p] = f4(0.f);
#pragma unroll
    for (int p = 0; p < NPA; ++p)
#pragma unroll
      for (int i = 0; i < kEC; ++i)
        acc[p] = fma4(s_att[(i < ad[p] ? ab[p] + i * H : ECAP * H) + h], zl[so[p][i]], acc[p]);
    if constexpr (BIG) {
      // rows past the segment table: their in-edges past kEC on their own lanes (edge order)
#pragma unroll
      for (int p = 0; p < NPA; ++p)
        for (int i = kEC; i < hend[p]; i += 4) {
          float av[4];
          float4 zv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bool ok = i + j < ad[p];
            const int e = ab[p] / H + (ok ? i + j : i);
            av[j] = ok ? s_att[e * H + h] : 0.f;
            zv[j] = zl[(int)s_srcs[e] * LPD + q];
          }
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (i + j < ad[p]) acc[p] = fma4(av[j], zv[j], acc[p]);
        }
      // hub segments: any lane group, kSegI independent LDS reads each; partials to s_part[k & 1]
      float4* sp = s_part + (k & 1) * (kSegCapI * LPD);
      for (int t = ds; t < nseg; t += DPP) {
        const uint32_t sg = s_seg[t];
        const int eb = (int)((sg >> 4) & 0xFFFu), c = (int)(sg & 15u) + 1;
        float4 part = f4(0.f);
#pragma unroll
        for (int j0 = 0; j0 < kSegI; j0 += 4) {  // two batches of 4 reads (registers)
          float av[4];
          float4 zv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bool ok = j0 + j < c;
            const int e = eb + (ok ? j0 + j : 0);
            av[j] = ok ? s_att[e * H + h] : 0.f;
            zv[j] = zl[(int)s_srcs[e] * LPD + q];
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) part = fma4(av[j], zv[j], part);
        }
        sp[t * LPD + q] = part;
      }
    }
    auto emit = [&](int p) {
      if (MODE == 1) {
        const float4 t = add4(acc[p], b4);
        tot[p] = (h == 0) ? t : add4(tot[p], t);
        // a store whose lanes are ALL out of range still costs a real one: branch (uniform)
        if (h == H - 1) {
          const float invh = (float)H;
          const float4 o = make_float4(tot[p].x / invh + rres[p].x, tot[p].y / invh + rres[p].y,
                                       tot[p].z / invh + rres[p].z, tot[p].w / invh + rres[p].w);
          buf_st4(rO, ob[p] + 4u * (uint32_t)((k / H) * CW + 4 * q), o);
          rmx[p] = amax4(rmx[p], o);
        }
      } else {
        float4 o = add4(add4(acc[p], rres[p]), b4);
        if (MODE == 0) o = make_float4(elu(o.x), elu(o.y), elu(o.z), elu(o.w));
        buf_st4(rO, ob[p] + 4u * (uint32_t)col, o);  // rows past the group: dropped
        rmx[p] = amax4(rmx[p], o);
      }
    };
    if constexpr (!BIG) {
#pragma unroll
      for (int p = 0; p < NPA; ++p) emit(p);
    }
    // stage chunk k+1 into the other buffer (read by nobody until the barrier) and rotate
    store_rows((k + 1) & 1, ring[0]);
#pragma unroll
    for (int i = 0; i + 1 < RING; ++i)
#pragma unroll
      for (int j = 0; j < NPA; ++j) ring[i][j] = ring[i + 1][j];
    load_rows(k + 1 + RING, ring[RING - 1]);
    __syncthreads();
    if constexpr (BIG) {  // the segment partials of chunk k are complete: add them in order, emit
      const float4* sp = s_part + (k & 1) * (kSegCapI * LPD);
#pragma unroll
      for (int p = 0; p < NPA; ++p) {
        const int n = sbn[p] >> 12;
        for (int j = 0; j < n; ++j) acc[p] = add4(acc[p], sp[((sbn[p] & 0xFFF) + j) * LPD + q]);
        emit(p);
      }
    }
#pragma unroll
    for (int j = 0; j < NPA; ++j)
      if constexpr (!BIG) rres[j] = rnx[j];
  }
  // a row's |max| over its LPD lanes (consecutive lanes of one wave); one writer per row
#pragma unroll
  for (int p = 0; p < NPA; ++p) {
    float m = live[p] ? rmx[p] : 0.f;
    omx = fmaxf(omx, m);
#pragma unroll
    for (int o = LPD / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (out_rows && live[p] && q == 0) out_rows[a0 + ds + DPP * p] = __float_as_uint(m);
  }
  return omx;
}

// NT = 16 * CW threads: 64 destinations per pass; groups of <= 64 atoms (most of them: the
// target is kNodeGroupAtoms) run one pass, larger ones two (kWinL = 128 atoms).  16 waves per
// CU either way (2 x 512 threads for CW = 32, 1 x 1024 for CW = 64).
// BIG (kind bit 2): the big-window variant for the groups on the forward fallback list (config
// 5's 150-400-atom molecules with hubs): 16-column chunks so that 512 rows fit LDS, in-degree
// unbounded (the hub loop above), one workgroup per CU walking the list.
template <int H, int CW, int MODE, int NT, int WIN = kWinL, int ECAP = kECap, bool BIG = false>
__global__ void __launch_bounds__(NT, MVML_LDS_WAVES)
gat_agg_fwd_lds_kernel(const int32_t* __restrict__ plan, int64_t G, const int32_t* __restrict__ rowptr,
                       const int32_t* __restrict__ in_src, const float* __restrict__ Y, int64_t ldy,
                       int F, const float* __restrict__ bias, const float* __restrict__ elr,
                       float slope, float* __restrict__ attn, float* __restrict__ out,
                       uint32_t* __restrict__ out_amax, uint32_t* __restrict__ out_rows) {
  constexpr int LPD = CW / 4;
  constexpr int DPP = NT / LPD;
  constexpr int NPM = WIN / DPP;  // passes over a full window
  static_assert(NPM * DPP == WIN && (NPM == 2 || NPM == 4), "the passes must tile the LDS rows exactly");
  __shared__ float4 zbuf[2][WIN * LPD];
  __shared__ float s_att[(ECAP + 1) * H];  // + H zeros: the attention of a missing edge
  // BIG: in-edge sources (window rows), the hub segment table, per-row segments, the
  // double-buffered segment partials and the scan's wave sums
  __shared__ uint16_t s_srcs[BIG ? ECAP : 1];
  __shared__ uint32_t s_seg[BIG ? kSegCapI : 1];
  __shared__ int s_rs[BIG ? WIN : 1];
  __shared__ float4 s_part[BIG ? 2 * kSegCapI * LPD : 1];
  __shared__ int s_wsum[BIG ? NT / 64 : 1];
  const int tid = threadIdx.x;
  const GroupPlan gp(plan, G);
  const int nlist = BIG ? gp.count[0] : (int)blockIdx.x + 1;
  float omx = 0.f;  // |max| of this thread's output stores, committed after the group loop
  for (int li = blockIdx.x; li < nlist; li += BIG ? gridDim.x : 1) {
  const int g = BIG ? gp.fwd_list[li] : li;
  if (BIG) __syncthreads();  // the previous group's LDS reads are done
  if (!(gp.kind[g] & (BIG ? 4 : 1))) continue;
  const int a0 = gp.start[g], a1 = gp.start[g + 1];
  const int nr = a1 - a0;
  const int ocols = MODE == 1 ? F : H * F;
  const int e0 = rowptr[a0];
  const int ne = rowptr[a1] - e0;
  // the group's edge_softmax, fused: one thread per (destination, head) pair into s_att (and
  // attn for the backward); fwd_lds_chunks' first barrier publishes it
  for (int pr = tid; pr < nr * H; pr += NT)
    softmax_pair<H>(a0 + pr / H, pr % H, rowptr, in_src, elr, slope, attn, s_att, e0);
  if (tid < H) s_att[ECAP * H + tid] = 0.f;
  int nseg = 0;
  if constexpr (BIG) {
    static_assert(NT >= WIN, "one row per thread for the segment scan");
    for (int i = tid; i < ne; i += NT) s_srcs[i] = (uint16_t)(in_src[e0 + i] - a0);
    const int eb = tid < nr ? rowptr[a0 + tid] - e0 : 0;
    const int deg = tid < nr ? rowptr[a0 + tid + 1] - e0 - eb : 0;
    int rs;
    nseg = hub_segments<NT, kSegI, kSegCapI>(nr, eb, deg, s_seg, &rs, s_wsum);
    if (tid < nr) s_rs[tid] = rs;
    __syncthreads();
  }
  const uint32_t rowb = (uint32_t)ldy * 4u;
  const __amdgpu_buffer_rsrc_t rY = make_rsrc(Y + (int64_t)a0 * ldy, (uint32_t)nr * rowb);
  const __amdgpu_buffer_rsrc_t rO = make_rsrc(out + (int64_t)a0 * ocols, (uint32_t)(nr * ocols) * 4u);
  if (nr <= DPP)
    omx = fmaxf(omx, fwd_lds_chunks<H, CW, MODE, NT, 1, WIN, ECAP, BIG>(zbuf, s_att, rowptr, in_src, rY, rowb, rO, a0, nr, e0, F, bias, s_srcs, s_seg, s_rs, s_part, nseg, out_rows));
  else if (NPM == 2 || nr <= 2 * DPP)
    omx = fmaxf(omx, fwd_lds_chunks<H, CW, MODE, NT, 2, WIN, ECAP, BIG>(zbuf, s_att, rowptr, in_src, rY, rowb, rO, a0, nr, e0, F, bias, s_srcs, s_seg, s_rs, s_part, nseg, out_rows));
  else if (nr <= 3 * DPP)
    omx = fmaxf(omx, fwd_lds_chunks<H, CW, MODE, NT, (NPM > 2 ? 3 : 2), WIN, ECAP, BIG>(zbuf, s_att, rowptr, in_src, rY, rowb, rO, a0, nr, e0, F, bias, s_srcs, s_seg, s_rs, s_part, nseg, out_rows));
  else
    omx = fmaxf(omx, fwd_lds_chunks<H, CW, MODE, NT, NPM, WIN, ECAP, BIG>(zbuf, s_att, rowptr, in_src, rY, rowb, rO, a0, nr, e0, F, bias, s_srcs, s_seg, s_rs, s_part, nseg, out_rows));
  }
  if (out_amax) block_amax_commit<NT>(omx, out_amax);
}

template <int H, int CW, int MODE>
__global__ void __launch_bounds__(kAggThreads, 4)  // 2 workgroups (16 waves) per CU
gat_agg_fwd_gather_kernel(const int32_t* __restrict__ plan, int64_t G, const int32_t* __restrict__ rowptr,
                   const int32_t* __restrict__ in_src, const float* __restrict__ Y, int64_t ldy,
                   int F, const float* __restrict__ bias, const float* __restrict__ elr, float slope,
                   float* __restrict__ attn, float* __restrict__ out, int skip_big,
                   uint32_t* __restrict__ out_amax, uint32_t* __restrict__ out_rows) {
  constexpr int LPD = CW / 4;                        // lanes per destination atom
  constexpr int DPP = kAggThreads / LPD;             // destinations per pass
  constexpr int NP = (kWin + DPP - 1) / DPP;         // passes over a full window
  const int tid = threadIdx.x;
  const int ds = tid / LPD, q = tid % LPD;
  const int HF = H * F;
  const GroupPlan gp(plan, G);
  const int li = list_block(blockIdx.x, gridDim.x, gp.count[0]);
  if (li < 0) return;
  const int g = gp.fwd_list[li];
  if (skip_big && (gp.kind[g] & 4)) return;  // the big-window kernel takes it
  float omx = 0.f;  // |max| of this thread's output stores (block-uniform early returns only)
  const int a0 = gp.start[g], a1 = gp.start[g + 1];
  const int nfc = F / CW;     // column chunks per head
  const int nch = H * nfc;
  const int ocols = MODE == 1 ? F : HF;
  // group-relative 32-bit byte offsets from a wave-uniform base (< 2^31: a group spans at most
  // kNodeGroupAtoms + one molecule's atoms, rows of <= 2^20 floats are checked by the host)
  const float* Yg = Y + (int64_t)a0 * ldy;
  const uint32_t rowb = (uint32_t)ldy * 4u;
  const __amdgpu_buffer_rsrc_t rY = make_rsrc(Yg, (uint32_t)(a1 - a0) * rowb);
  constexpr uint32_t kNone = 0xFFFFFFF0u;  // out of range: the load returns 0, moves no data
  // Hub destinations (in-degree > kHubDeg) leave the chunk sweep: after it, the whole block
  // aggregates one hub at a time over ALL its columns at once, so a hub costs deg / 8 memory
  // round trips instead of (column chunks) x deg / 8 on 16 lanes.  Same summation order.
  __shared__ float4 s_hub[kHubCols];
  __shared__ float s_red[kAggThreads / 64];
  const bool hubpass = HF / 4 <= kHubCols;
  // the group's edge_softmax, fused (global attn: the sweep below gathers it per edge; the
  // barrier makes this workgroup's stores visible to it)
  for (int pr = tid; pr < (a1 - a0) * H; pr += kAggThreads)
    softmax_pair<H>(a0 + pr / H, pr % H, rowptr, in_src, elr, slope, attn, nullptr, 0);
  __syncthreads();

  for (int w0 = a0; w0 < a1; w0 += kWin) {
    const int nr = min(kWin, a1 - w0);
    const int e0 = rowptr[w0];

    const float* __restrict__ attw = attn + (int64_t)e0 * H;
    const __amdgpu_buffer_rsrc_t rO = make_rsrc(out + (int64_t)w0 * ocols, (uint32_t)(nr * ocols) * 4u);
    // this thread's destinations: in-CSR ranges and the cached source-row offsets
    int eb[NP], deg[NP];
    bool hub[NP];
    uint32_t so[NP][kEC];
    int dmax = 0;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int d = ds + DPP * p;
      eb[p] = 0;
      deg[p] = 0;
      if (d < nr) {
        eb[p] = rowptr[w0 + d] - e0;
        deg[p] = rowptr[w0 + d + 1] - e0 - eb[p];
      }
      hub[p] = hubpass && deg[p] > kHubDeg;
      if (hub[p]) deg[p] = 0;  // aggregated by the hub pass below
#pragma unroll
      for (int i = 0; i < kEC; ++i)
        so[p][i] = (i < deg[p]) ? (uint32_t)(in_src[e0 + eb[p] + i] - a0) * rowb : kNone;
      dmax = max(dmax, deg[p]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) dmax = max(dmax, __shfl_xor(dmax, o, 64));  // wave-uniform
    auto att = [&](int e, int h) -> float { return attw[e * H + h]; };

    float4 tot[NP], rm[NP];
    float rmx[NP];  // per destination |max| (out_rows)
#pragma unroll
    for (int p = 0; p < NP; ++p) rmx[p] = 0.f;
    for (int k = 0; k < nch; ++k) {
      const int h = MODE == 1 ? k % H : k / nfc;
      const int fc = MODE == 1 ? k / H : k % nfc;
      const int col = h * F + fc * CW + 4 * q;
      const uint32_t colb = 4u * (uint32_t)col;
      float4 acc[NP], res[NP];
      // residual (flatten: this chunk's columns; mean: the f-chunk's head-mean columns)
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int d = ds + DPP * p;
        const uint32_t rb = (d < nr) ? (uint32_t)(w0 + d - a0) * rowb : kNone;
        if (MODE != 1) res[p] = buf_ld4(rY, rb == kNone ? kNone : rb + 4u * (uint32_t)(HF + col));
        else if (h == 0) rm[p] = buf_ld4(rY, rb == kNone ? kNone : rb + 4u * (uint32_t)(HF + fc * CW + 4 * q));
      }
      // cached edges: one batch of independent loads (one memory round trip per chunk)
#pragma unroll
      for (int p = 0; p < NP; ++p) acc[p] = f4(0.f);
      {
        float4 z[NP][kEC];
        float a[NP][kEC];
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
          for (int i = 0; i < kEC; ++i) {
            z[p][i] = buf_ld4(rY, so[p][i] == kNone ? kNone : so[p][i] + colb);
            a[p][i] = (i < deg[p]) ? att(eb[p] + i, h) : 0.f;
          }
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
          for (int i = 0; i < kEC; ++i)
            if (i < deg[p]) acc[p] = fma4(a[p][i], z[p][i], acc[p]);
      }
      if (dmax > kEC) {  // hubs: batches of 8 independent gathers (same summation order)
#pragma unroll
        for (int p = 0; p < NP; ++p)
          for (int i = kEC; i < deg[p]; i += 8) {
            uint32_t ob[8];
            float av[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const bool ok = i + j < deg[p];
              const int e = eb[p] + (ok ? i + j : i);
              ob[j] = ok ? (uint32_t)(in_src[e0 + e] - a0) * rowb + colb : kNone;
              av[j] = ok ? att(e, h) : 0.f;
            }
            float4 zv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) zv[j] = buf_ld4(rY, ob[j]);
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if (i + j < deg[p]) acc[p] = fma4(av[j], zv[j], acc[p]);
          }
      }
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int d = ds + DPP * p;
        if (d < nr && !hub[p]) {
          if (MODE == 1) {
            const float4 t = add4(acc[p], ld4(bias + col));
            tot[p] = (h == 0) ? t : add4(tot[p], t);
            if (h == H - 1) {
              const float invh = (float)H;
              const float4 o = make_float4(tot[p].x / invh + rm[p].x, tot[p].y / invh + rm[p].y,
                                           tot[p].z / invh + rm[p].z, tot[p].w / invh + rm[p].w);
              buf_st4(rO, 4u * (uint32_t)(d * F + fc * CW + 4 * q), o);
              rmx[p] = amax4(rmx[p], o);
            }
          } else {
            float4 o = add4(add4(acc[p], res[p]), ld4(bias + col));
            if (MODE == 0) o = make_float4(elu(o.x), elu(o.y), elu(o.z), elu(o.w));
            buf_st4(rO, 4u * (uint32_t)(d * HF + col), o);
            rmx[p] = amax4(rmx[p], o);
          }
        }
      }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {  // rows of the sweep: |max| over their LPD lanes, one writer
      const int d = ds + DPP * p;
      float m = rmx[p];
      omx = fmaxf(omx, m);
#pragma unroll
      for (int o = LPD / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      if (out_rows && d < nr && !hub[p] && q == 0) out_rows[w0 + d] = __float_as_uint(m);
    }
    if (!hubpass) continue;
    for (int d = 0; d < nr; ++d) {  // block-uniform walk over the window's hubs
      const int hb = rowptr[w0 + d] - e0, hdeg = rowptr[w0 + d + 1] - e0 - hb;
      if (hdeg <= kHubDeg) continue;
      const uint32_t vb = (uint32_t)(w0 + d - a0) * rowb;
      float hmx = 0.f;  // this thread's part of the hub row's |max|
      for (int c4 = tid; c4 < HF / 4; c4 += kAggThreads) {
        const int col = 4 * c4, h = col / F;
        const uint32_t colb = 4u * (uint32_t)col;
        float4 acc = f4(0.f);
        for (int i = 0; i < hdeg; i += 8) {
          uint32_t ob[8];
          float av[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const bool ok = i + j < hdeg;
            const int e = hb + (ok ? i + j : i);
            ob[j] = ok ? (uint32_t)(in_src[e0 + e] - a0) * rowb + colb : kNone;
            av[j] = ok ? attw[e * H + h] : 0.f;
          }
          float4 zv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) zv[j] = buf_ld4(rY, ob[j]);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (i + j < hdeg) acc = fma4(av[j], zv[j], acc);
        }
        if (MODE == 1) {
          s_hub[c4] = add4(acc, ld4(bias + col));
        } else {
          const float4 res = buf_ld4(rY, vb + 4u * (uint32_t)(HF + col));
          float4 o = add4(add4(acc, res), ld4(bias + col));
          if (MODE == 0) o = make_float4(elu(o.x), elu(o.y), elu(o.z), elu(o.w));
          buf_st4(rO, 4u * (uint32_t)(d * HF + col), o);
          hmx = amax4(hmx, o);
        }
      }
      if (MODE == 1) {  // head mean, heads summed in order as in the chunk sweep
        __syncthreads();
        for (int f4 = tid; f4 < F / 4; f4 += kAggThreads) {
          float4 tot = s_hub[f4];
          for (int hh = 1; hh < H; ++hh) tot = add4(tot, s_hub[hh * (F / 4) + f4]);
          const float4 rmv = buf_ld4(rY, vb + 4u * (uint32_t)(HF + 4 * f4));
          const float invh = (float)H;
          const float4 o = make_float4(tot.x / invh + rmv.x, tot.y / invh + rmv.y,
                                       tot.z / invh + rmv.z, tot.w / invh + rmv.w);
          buf_st4(rO, 4u * (uint32_t)(d * F + 4 * f4), o);
          hmx = amax4(hmx, o);
        }
        __syncthreads();
      }
      omx = fmaxf(omx, hmx);
      if (out_rows) {  // the hub row's |max| over the block (block-uniform branch)
        hmx = wave_max(hmx);
        if ((tid & 63) == 0) s_red[tid >> 6] = hmx;
        __syncthreads();
        if (tid == 0) {
          float m = s_red[0];
#pragma unroll
          for (int w = 1; w < kAggThreads / 64; ++w) m = fmaxf(m, s_red[w]);
          out_rows[w0 + d] = __float_as_uint(m);
        }
        __syncthreads();
      }
    }
  }
  if (out_amax) block_amax_commit<kAggThreads>(omx, out_amax);
}

// ---- Forward by destination wave (MVML_OPT_DST_FWD) -------------------------------------------
// One wave per destination atom v.  xcd_block hands each XCD one contiguous atom range, so the
// projection rows a destination gathers were just read by its neighbours' waves and come from
// the XCD's L2 (tree / ring edges), or from the Infinity Cache (a hub's partners); each row
// crosses HBM about once.  SM (fused softmax): the wave forms v's edge softmax with its lanes on
// the in-edges (softmax_pair's arithmetic and order: max, then the sum of exp in edge order,
// a = exp / sum) and writes attn; !SM: gat_softmax_dst_kernel wrote attn before, and the wave
// reads it (one dependent load less per atom).  Then it gathers the WHOLE Z[src] row of each
// in-edge into registers, U rows in flight, sums them in edge order starting from 0 (bitwise the
// LDS / gather kernels' sums), adds residual and bias, applies ELU or the head mean and writes
// out[v] once.  No LDS, no barriers, no size classes: one code path for every molecule size.
// Column slots: flatten modes: lane l owns float4 columns c = l + 64 j (j < NJ, 4c < H F);
// mean mode (H >= 2): the two half-waves own heads [0, H/2) and [H/2, H), lane l the f-float4
// columns q = (l & 31) + 32 k (k < NJ, 4q < F) of its half's heads (6 slots per lane at
// H = 4, F = 384, no idle lane), and the halves meet by a cross-half shuffle for the head sum,
// added in head order (bitwise the LDS kernel's head mean).  H = 1 mean: q = l + 64 k.
// LR (late residual): the residual row is loaded after the gather instead of before the softmax
// (12 fewer VGPRs live across the gather loop in mean mode: five waves per SIMD instead of four)
// (measured: the head-mean form held to six waves per SIMD spills 17 VGPRs with the fused softmax
// and ran 6.1 -> 7.6-8.1 ms on config 5; even without it)
template <int H, int MODE, int NJ, int U, bool SM, bool LR = false>
__global__ void __launch_bounds__(256, LR ? (MODE == 1 ? 5 : 8) : 1)
gat_agg_fwd_dst_kernel(int64_t N, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ in_src,
                       const float* __restrict__ Y, int64_t ldy, int F, const float* __restrict__ bias,
                       const float* __restrict__ elr, float slope, float* __restrict__ attn,
                       float* __restrict__ out, uint32_t* __restrict__ out_amax,
                       uint32_t* __restrict__ out_rows) {
  constexpr bool PAIR = MODE == 1 && H >= 2;
  constexpr int NH = PAIR ? H / 2 : 1;  // heads per lane (mean mode); 1 register set (flatten)
  const int lane = threadIdx.x & 63;
  const int64_t v = xcd_block(blockIdx.x, gridDim.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float omx = 0.f;
  // (a non-persistent grid: the dispatcher hands out blocks in atom order, which keeps an XCD's
  // waves on one compact window of neighbouring atoms; a persistent walk let them drift apart
  // and ran 1.3-1.7x slower on config 5)
  if (v < N) {  // (no early return: block_amax_commit below has a barrier)
    const int HF = H * F;
    const int hp = PAIR ? lane >> 5 : 0;       // mean: this lane's half (heads hp H/2 ..)
    const int ql = PAIR ? (lane & 31) : lane;  // mean: f-float4 base of this lane
    const float* yv = Y + v * ldy;
    bool ok[NJ];
    int hc[NJ];   // flatten: the head of each column slot
    int cz[NJ];   // float offset of slot j in a projection row (mean: of head hp * NH)
    float4 res[NJ], acc[NH][NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if constexpr (MODE == 1) {
        const int q = ql + (PAIR ? 32 : 64) * j;
        ok[j] = 4 * q < F;
        hc[j] = 0;
        cz[j] = hp * NH * F + 4 * q;
        // the residual first (its HBM latency overlaps the softmax); the lower half stores out
        if constexpr (!LR) res[j] = (ok[j] && hp == 0) ? ld4nt(yv + HF + 4 * q) : f4(0.f);
      } else {
        const int c = lane + 64 * j;
        ok[j] = 4 * c < HF;
        hc[j] = ok[j] ? 4 * c / F : 0;
        cz[j] = 4 * c;
        if constexpr (!LR) res[j] = ok[j] ? ld4nt(yv + HF + 4 * c) : f4(0.f);
      }
#pragma unroll
      for (int h = 0; h < NH; ++h) acc[h][j] = f4(0.f);
    }
    const int eb = rowptr[v], deg = rowptr[v + 1] - eb;
    float er[H], m[H], sum[H], s0[H];
    int src0 = 0;
    // logits of the in-edges [eb + base, ...) on the lanes (edge order); -inf past the row
    auto logits = [&](int base, int& src, float (&s)[H]) {
      const bool in = base + lane < deg;
      src = in ? in_src[eb + base + lane] : 0;
#pragma unroll
      for (int h = 0; h < H; ++h)
        s[h] = in ? leaky(elr[(int64_t)src * 2 * H + h] + er[h], slope) : -INFINITY;
    };
    if constexpr (SM) {
#pragma unroll
      for (int h = 0; h < H; ++h) er[h] = elr[v * 2 * H + H + h];
      logits(0, src0, s0);
#pragma unroll
      for (int h = 0; h < H; ++h) m[h] = s0[h];
      for (int base = 64; base < deg; base += 64) {  // in-degree > 64 (hubs): more chunks
        int s_;
        float s[H];
        logits(base, s_, s);
#pragma unroll
        for (int h = 0; h < H; ++h) m[h] = fmaxf(m[h], s[h]);
      }
      HeadReduce<H>::template all<true>(m, lane);
      // sum of exp in edge order (softmax_pair's order), lane by lane
#pragma unroll
      for (int h = 0; h < H; ++h) sum[h] = 0.f;
      for (int base = 0; base < deg; base += 64) {
        int s_ = src0;
        float s[H];
        if (base == 0) {
#pragma unroll
          for (int h = 0; h < H; ++h) s[h] = s0[h];
        } else {
          logits(base, s_, s);
        }
        float p[H];
#pragma unroll
        for (int h = 0; h < H; ++h) p[h] = base + lane < deg ? expf(s[h] - m[h]) : 0.f;
        const int cnt = min(64, deg - base);
        for (int i = 0; i < cnt; ++i)
#pragma unroll
          for (int h = 0; h < H; ++h) sum[h] += rl(p[h], i);
      }
    } else {
      src0 = lane < deg ? in_src[eb + lane] : 0;
    }
    // (the attention of) the in-edges and the gather, 64 edges per chunk
    for (int base = 0; base < deg; base += 64) {
      const int cnt = min(64, deg - base);
      int src_l = src0;
      float a_l[H];
      if constexpr (SM) {
        float s[H];
        if (base == 0) {
#pragma unroll
          for (int h = 0; h < H; ++h) s[h] = s0[h];
        } else {
          logits(base, src_l, s);
        }
#pragma unroll
        for (int h = 0; h < H; ++h) a_l[h] = lane < cnt ? expf(s[h] - m[h]) / sum[h] : 0.f;
        if (lane < cnt) {
          float* ap = attn + (int64_t)(eb + base + lane) * H;
          if constexpr (H == 4) {
            st4(ap, make_float4(a_l[0], a_l[1], a_l[2], a_l[3]));
          } else {
#pragma unroll
            for (int h = 0; h < H; ++h) ap[h] = a_l[h];
          }
        }
      } else {
        if (base > 0) src_l = lane < cnt ? in_src[eb + base + lane] : 0;
        const float* ap = attn + (int64_t)(eb + base + lane) * H;
        if constexpr (H == 4) {
          const float4 a4 = lane < cnt ? ld4(ap) : f4(0.f);
          a_l[0] = a4.x; a_l[1] = a4.y; a_l[2] = a4.z; a_l[3] = a4.w;
        } else {
#pragma unroll
          for (int h = 0; h < H; ++h) a_l[h] = lane < cnt ? ap[h] : 0.f;
        }
      }
      for (int j0 = 0; j0 < cnt; j0 += U) {
        float4 z[U][NH][NJ];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e = min(j0 + u, cnt - 1);  // past the chunk: a duplicate row, not summed
          const float* zr = Y + (int64_t)rl(src_l, e) * ldy;
#pragma unroll
          for (int h = 0; h < NH; ++h)
#pragma unroll
            for (int j = 0; j < NJ; ++j) z[u][h][j] = ok[j] ? ld4(zr + cz[j] + h * F) : f4(0.f);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (j0 + u < cnt) {  // (uniform)
            float a[H];
#pragma unroll
            for (int h = 0; h < H; ++h) a[h] = rl(a_l[h], j0 + u);
#pragma unroll
            for (int h = 0; h < NH; ++h) {
              // mean: this half's head hp NH + h (a select between the halves' heads)
              float ah = a[h];
              if constexpr (PAIR) ah = hp ? a[NH + h] : a[h];
#pragma unroll
              for (int j = 0; j < NJ; ++j)
                acc[h][j] = fma4(MODE == 1 ? ah : pick<H>(a, hc[j]), z[u][h][j], acc[h][j]);
            }
          }
        }
      }
    }
    float rmx = 0.f;
    if constexpr (LR) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if constexpr (MODE == 1) {
          const int q = ql + (PAIR ? 32 : 64) * j;
          res[j] = (ok[j] && hp == 0) ? ld4nt(yv + HF + 4 * q) : f4(0.f);
        } else {
          res[j] = ok[j] ? ld4nt(yv + HF + 4 * (lane + 64 * j)) : f4(0.f);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float4 o;
      if constexpr (MODE == 1) {  // head mean: heads summed in order (+ bias per head), / H, + R
        const int q = ql + (PAIR ? 32 : 64) * j;
        const int qc = ok[j] ? 4 * q : 0;
        float4 t[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h) t[h] = add4(acc[h][j], ld4(bias + (hp * NH + h) * F + qc));
        float4 tot = t[0];
#pragma unroll
        for (int h = 1; h < NH; ++h) tot = add4(tot, t[h]);
        if constexpr (PAIR) {  // + the upper half's heads, in order
#pragma unroll
          for (int h = 0; h < NH; ++h)
            tot = add4(tot, make_float4(__shfl_xor(t[h].x, 32, 64), __shfl_xor(t[h].y, 32, 64),
                                        __shfl_xor(t[h].z, 32, 64), __shfl_xor(t[h].w, 32, 64)));
        }
        if (!ok[j] || hp != 0) continue;
        const float invh = (float)H;
        o = make_float4(tot.x / invh + res[j].x, tot.y / invh + res[j].y, tot.z / invh + res[j].z,
                        tot.w / invh + res[j].w);
        st4nt(out + v * F + 4 * q, o);
      } else {
        if (!ok[j]) continue;
        o = add4(add4(acc[0][j], res[j]), ld4(bias + cz[j]));
        if (MODE == 0) o = make_float4(elu(o.x), elu(o.y), elu(o.z), elu(o.w));
        st4nt(out + v * HF + cz[j], o);
      }
      rmx = amax4(rmx, o);
    }
    const float wm = wave_max(rmx);
    omx = fmaxf(omx, wm);
    if (out_rows && lane == 0) out_rows[v] = __float_as_uint(wm);
  }
  if (out_amax) block_amax_commit<256>(omx, out_amax);
}

// *out = max(*out, max_i rows[i]) (bits of non-negative floats): the operand max of a product
// from the per-row maxima its producer already wrote, instead of one atomicMax per 4-atom block
// of a wave-per-atom kernel (a single word takes ~90 atomics per us: 440 k of them were most of
// the forward's 5 ms on config 5).  A few hundred blocks, one atomic each.
__global__ void __launch_bounds__(256)
rows_amax_kernel(int64_t n, const uint32_t* __restrict__ rows, uint32_t* __restrict__ out) {
  uint32_t m = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    m = max(m, rows[i]);
  block_amax_commit<256>(__uint_as_float(m), out);
}

inline int launch_rows_amax(int64_t n, const uint32_t* rows, uint32_t* out, hipStream_t st) {
  if (!rows || !out || n <= 0) return MVML_OK;
  rows_amax_kernel<<<(unsigned)std::min<int64_t>(ceil_div(n, 256 * 16), 512), 256, 0, st>>>(n, rows, out);
  return check_launch("rows_amax_kernel");
}

// H = 4: one thread per destination with the four heads as one float4 (el / er rows are 16 B),
// softmax_pair's per-head arithmetic and edge order, so attn is bitwise the same; the first DC
// logits stay in registers, later ones are recomputed (L2-resident el rows).
__global__ void __launch_bounds__(256)
gat_softmax_dst4_kernel(int64_t N, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ in_src,
                        const float* __restrict__ elr, float slope, float* __restrict__ attn) {
  const int64_t v = xcd_block(blockIdx.x, gridDim.x) * 256 + threadIdx.x;
  if (v >= N) return;
  const float4 er = ld4(elr + v * 8 + 4);
  const int eb = rowptr[v], ee = rowptr[v + 1];
  auto logit = [&](int e) {
    const float4 el = ld4(elr + (int64_t)in_src[e] * 8);
    return make_float4(leaky(el.x + er.x, slope), leaky(el.y + er.y, slope), leaky(el.z + er.z, slope),
                       leaky(el.w + er.w, slope));
  };
  constexpr int DC = 6;
  float4 sc[DC];
  float4 m = f4(-INFINITY), sum = f4(0.f);
#pragma unroll
  for (int t = 0; t < DC; ++t) {
    sc[t] = (eb + t < ee) ? logit(eb + t) : f4(-INFINITY);
    m = make_float4(fmaxf(m.x, sc[t].x), fmaxf(m.y, sc[t].y), fmaxf(m.z, sc[t].z), fmaxf(m.w, sc[t].w));
  }
  for (int e = eb + DC; e < ee; ++e) {
    const float4 c = logit(e);
    m = make_float4(fmaxf(m.x, c.x), fmaxf(m.y, c.y), fmaxf(m.z, c.z), fmaxf(m.w, c.w));
  }
  auto ex = [&](float4 c) {
    return make_float4(expf(c.x - m.x), expf(c.y - m.y), expf(c.z - m.z), expf(c.w - m.w));
  };
#pragma unroll
  for (int t = 0; t < DC; ++t)
    if (eb + t < ee) sum = add4(sum, ex(sc[t]));
  for (int e = eb + DC; e < ee; ++e) sum = add4(sum, ex(logit(e)));
  auto store = [&](int e, float4 c) {
    const float4 p = ex(c);
    st4(attn + (int64_t)e * 4, make_float4(p.x / sum.x, p.y / sum.y, p.z / sum.z, p.w / sum.w));
  };
#pragma unroll
  for (int t = 0; t < DC; ++t)
    if (eb + t < ee) store(eb + t, sc[t]);
  for (int e = eb + DC; e < ee; ++e) store(e, logit(e));
}

// The edge softmax alone, one thread per (destination, head) (softmax_pair: bitwise the fused
// kernels' attn), for gat_agg_fwd_dst_kernel<..., SM = false>.
template <int H>
__global__ void __launch_bounds__(256)
gat_softmax_dst_kernel(int64_t N, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ in_src,
                       const float* __restrict__ elr, float slope, float* __restrict__ attn) {
  const int64_t i = xcd_block(blockIdx.x, gridDim.x) * 256 + threadIdx.x;
  if (i >= N * H) return;
  softmax_pair<H>(i / H, (int)(i % H), rowptr, in_src, elr, slope, attn, nullptr, 0);
}

// --------------------------------------------------------------------------------- backward
// Backward contract (mvml_gat_agg_bwd): gY[n] = [dZ_agg | dR | d el | d er] where dZ_agg is
// dL/dZ through update_all(u_mul_e, sum) only; the el / er paths of dL/dZ (d el x attn_l +
// d er x attn_r) are NOT added to it: the projection backward takes them exactly through two
// extra GEMM rows / columns (A_l = attn_l . W_fc, see mvml_gat_fold_attn_rows), which keeps
// the backward to ONE pass over Z and dZ.
//
// The molecule case (group of <= kWinL atoms and <= kECap in-edges) is one workgroup per node
// group: the group's CSR, out-CSR and attention are staged in LDS, then the columns are swept
// CW at a time with Z and g_rst (= dL/d rst from g_out, ELU' or 1/H) staged in LDS:
//   * thread per in-edge e: g_a[e,h] += <Z[src_e], g_rst[dst_e]> over the chunk's columns;
//   * CW/4 lanes per source atom u: dZ_agg[u] = sum over u's out-edges of a_e g_rst[dst_e];
//   * dR (g_rst, or g_out for the head-mean residual) is written from the staged rows;
// then the softmax backward runs in LDS (g_s = a (g_a - sum a g_a), g_pre = g_s leaky') and
// d er / d el are its per-destination / per-source sums.  Z, g_out and dZ cross HBM once.
// Every other group (large molecules, edge-heavy hubs) takes the per-atom dst / src pair.
#ifndef MVML_BWD_WAVES
#define MVML_BWD_WAVES 4
#endif
// Backward LDS layout: Z and g_rst chunks of the group's rows, 16-B slot c of row r at
// r*LPD + (c ^ bwd_sw<LPD>(r)): 128-B rows (LPD = 8) are XOR-swizzled so whole-row reads of
// different atoms spread over the banks; 256-B rows (LPD = 16) already span all 64 banks.
template <int LPD>
__device__ __forceinline__ int bwd_sw(int r) { return LPD == 8 ? (r >> 1) & 7 : 0; }  // 4, 16: none

// DPP move within a row of 16 lanes (bound_ctrl: sources outside the row read 0).
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
// Sum over each aligned group of LPD (4, 8 or 16) lanes; valid in the group's last four lanes.
template <int LPD>
__device__ __forceinline__ float grp_sum_hi(float v) {
  v += dppf<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dppf<0x4E>(v);   // quad_perm [2,3,0,1]
  if (LPD >= 8) v += dppf<0x114>(v);  // row_shr:4
  if (LPD == 16) v += dppf<0x118>(v);  // row_shr:8
  return v;
}

// Chunk loop of the backward LDS kernel for a group of at most NPA * 64 atoms: 8 lanes per row
// (CW = 32 columns), NPA rows per lane octet.  The chunk rows (Z, g_out, and for ELU' the
// forward output) stream through a register ring (k+1 and k+2 in flight while chunk k is
// processed from LDS; k+1 only for two-pass groups).  Loads are unconditional (rows past the group read 0 through
// the buffer resource's range check; chunks past the end use an out-of-range offset), so the
// loop is straight-line and the vmcnt waits are exact; stores of rows past the group are
// skipped.
// Per chunk, the octet of destination atom d also forms g_a[e, h] += <Z[src_e], g_rst[d]> over
// the chunk's columns for d's in-edges: lane q dots its 16-B slice of the source row (LDS) with
// its slice of g_rst[d], a DPP octet sum finishes the dot, and one lane per edge adds it to
// s_ga (zeroed by the caller; every (edge, head) has exactly one writer).  That reads each
// source row slice once per in-edge: half the LDS bytes of an edge-per-thread dot.
// BIG: the out-CSR (s_odst / s_oslot) is read from global memory (g_odst / g_oslot, group
// edge base e0, first atom a0) instead of LDS, which the big window needs for its rows.
template <int H, int MODE, int NPA, int CW, int NT = 16 * CW, int WIN = kWinL, int ECAP = kECap,
          bool BIG = false>
__device__ __forceinline__ float bwd_lds_chunks(
    float4* zs, float4* gs, const float* s_att, const int* s_odst, const int* s_oslot,
    const int* s_orp, const int* s_rp, const uint16_t* s_src, float* s_ga,
    __amdgpu_buffer_rsrc_t rY, int ldyi, __amdgpu_buffer_rsrc_t rGo, __amdgpu_buffer_rsrc_t rO,
    __amdgpu_buffer_rsrc_t rG, int ldgi, int nr, int F, const int32_t* __restrict__ g_odst = nullptr,
    const int32_t* __restrict__ g_oslot = nullptr, int e0 = 0, int a0 = 0,
    const uint32_t* s_segI = nullptr, int nsegI = 0, const uint32_t* s_segO = nullptr,
    int nsegO = 0, const int* s_rs = nullptr, float4* s_part = nullptr,
    const uint32_t* s_oxe = nullptr, const uint16_t* s_oxb = nullptr, float* s_rmx = nullptr) {
  static_assert(kEC == 5, "in-edge writer lanes assume 5 cached in-edges");
  constexpr int LPD = CW / 4, DPP = NT / LPD;
  auto odst = [&](int o) -> int { if constexpr (BIG) return g_odst[e0 + o] - a0; else return s_odst[o]; };
  auto oslot = [&](int o) -> int { if constexpr (BIG) return g_oslot[e0 + o] - e0; else return s_oslot[o]; };
  const int tid = threadIdx.x, ds = tid / LPD, q = tid % LPD;
  const int HF = H * F, nfc = F / CW, nch = H * nfc;
  const int ocols = MODE == 1 ? F : HF;
  // row byte offsets (recomputed where used: registers are the constraint at NPA = 2)
  auto yrow = [&](int p) { return 4u * (uint32_t)((ds + DPP * p) * ldyi); };
  auto grow = [&](int p) { return 4u * (uint32_t)((ds + DPP * p) * ldgi); };
  auto gorow = [&](int p) { return 4u * (uint32_t)((ds + DPP * p) * ocols); };
  auto orow = [&](int p) { return 4u * (uint32_t)((ds + DPP * p) * HF); };
  // "no access" offsets just past each resource (see fwd_lds_chunks): every load and store is
  // unconditional, so the compiler's vmcnt counts are exact
  const uint32_t noY = 4u * (uint32_t)(nr * ldyi), noGo = 4u * (uint32_t)(nr * ocols);
  const uint32_t noO = 4u * (uint32_t)(nr * HF), noG = 4u * (uint32_t)(nr * ldgi);
  float gmx = 0.f;  // |max| of this thread's stores into gY (live rows, real chunks)
  float rmx[NPA];   // ... per row (s_rmx: the rows' |max| over dZ and dR, for per-row scales)
  bool live[NPA];
  // node role: the g_rst row slot (low 16 bits) and attention slot (high 16 bits) of the
  // first kEC out-edges of this octet's source atoms in registers (a missing edge reads the
  // atom's own row with a zero attention), so a chunk's gathers are independent LDS reads;
  // more out-edges (hubs) loop.
  static_assert(WIN * LPD <= 65536 && (ECAP + 1) * H <= 65536, "16-bit slots");
  uint32_t gsl[NPA][kEC];
  int ob[NPA], oend[NPA];
#pragma unroll
  for (int p = 0; p < NPA; ++p) {
    const int r = ds + DPP * p;
    live[p] = r < nr;
    rmx[p] = 0.f;
    ob[p] = live[p] ? s_orp[r] : 0;
    oend[p] = live[p] ? s_orp[r + 1] : 0;
#pragma unroll
    for (int i = 0; i < kEC; ++i) {
      const bool ok = ob[p] + i < oend[p];
      const int rr = ok ? odst(ob[p] + i) : r;
      gsl[p][i] = (uint32_t)(rr * LPD + (q ^ bwd_sw<LPD>(rr))) |
                  ((uint32_t)(ok ? oslot(ob[p] + i) * H : ECAP * H) << 16);
    }
  }
  // destination role: Z row slots of the first kEC in-edges (own row when missing; the dot is
  // then discarded), the in-edge base and in-degree
  uint32_t zsl[NPA][kEC];
  int ieb[NPA], ideg[NPA];
  // BIG: hub segments of this octet's rows — in-edges past kEC (segmented rows: none walked
  // here, bit 31) and out-edges past kEC (first | count << 12; their partials are added below)
  int rsg[NPA], oxb[NPA];
#pragma unroll
  for (int p = 0; p < NPA; ++p) {
    rsg[p] = 0;
    oxb[p] = 0xFFFF;
    if constexpr (BIG) {
      rsg[p] = live[p] ? s_rs[ds + DPP * p] : 0;
      oxb[p] = live[p] ? (int)s_oxb[ds + DPP * p] : 0xFFFF;
    }
  }
#pragma unroll
  for (int p = 0; p < NPA; ++p) {
    const int d = ds + DPP * p;
    ieb[p] = live[p] ? s_rp[d] : 0;
    ideg[p] = live[p] ? s_rp[d + 1] - ieb[p] : 0;
#pragma unroll
    for (int i = 0; i < kEC; ++i) {
      const int sr = i < ideg[p] ? s_src[ieb[p] + i] : d;
      zsl[p][i] = (uint32_t)(sr * LPD + (q ^ bwd_sw<LPD>(sr)));
    }
  }
  auto head_of = [&](int k) { return MODE == 1 ? k % H : k / nfc; };
  auto fch_of = [&](int k) { return MODE == 1 ? k / H : k % nfc; };
  auto col_of = [&](int k) { return head_of(k) * F + fch_of(k) * CW + 4 * q; };
  struct Rows { float4 z[NPA], g[NPA], o[NPA]; };
  // Mean mode: chunks are f-chunk-major (k = fc H + h), and g_rst = g_out / H is the same for
  // the H heads of an f-chunk, so g_out is loaded and gs staged only at h == 0 (the gs image of
  // chunk k stays valid for chunks k+1 .. k+H-1).
  auto load = [&](int k, Rows& R) {
    const bool ok = k < nch;
    const int col = col_of(k);
    const int gcol = MODE == 1 ? fch_of(k) * CW + 4 * q : col;
    const bool gload = MODE != 1 || head_of(k) == 0;  // uniform
#pragma unroll
    for (int p = 0; p < NPA; ++p) {
      R.z[p] = buf_ld4(rY, ok ? yrow(p) + 4u * (uint32_t)col : noY);
      if (gload) R.g[p] = buf_ld4(rGo, ok ? gorow(p) + 4u * (uint32_t)gcol : noGo);
      if (MODE == 0) R.o[p] = buf_ld4(rO, ok ? orow(p) + 4u * (uint32_t)col : noO);
    }
  };
  // stage chunk k: g_rst = g_out * ELU'(x) (ELU' = out + 1 for x <= 0, torch elu_backward on
  // the result) | g_out / H (head mean) | g_out; dR = g_rst, or g_out once per f-chunk (mean)
  auto stage = [&](int k, const Rows& R) {
    const bool ok = k < nch;
    const int h = head_of(k), fc = fch_of(k);
#pragma unroll
    for (int p = 0; p < NPA; ++p) {
      const int r = ds + DPP * p;
      float4 g = R.g[p];
      if (MODE == 0) {
        const float4 o = R.o[p];
        g.x *= o.x > 0.f ? 1.f : o.x + 1.f;
        g.y *= o.y > 0.f ? 1.f : o.y + 1.f;
        g.z *= o.z > 0.f ? 1.f : o.z + 1.f;
        g.w *= o.w > 0.f ? 1.f : o.w + 1.f;
      } else if (MODE == 1) {
        const float hh = (float)H;
        g = make_float4(g.x / hh, g.y / hh, g.z / hh, g.w / hh);
      }
      zs[r * LPD + (q ^ bwd_sw<LPD>(r))] = R.z[p];
      if (MODE != 1) {
        gs[r * LPD + (q ^ bwd_sw<LPD>(r))] = g;
        buf_st4(rG, ok ? grow(p) + 4u * (uint32_t)(HF + col_of(k)) : noG, g);
        if (ok && r < nr) rmx[p] = amax4(rmx[p], g);
      } else if (h == 0) {  // uniform branch: an all-out-of-range store is not free
        gs[r * LPD + (q ^ bwd_sw<LPD>(r))] = g;
        buf_st4(rG, ok ? grow(p) + 4u * (uint32_t)(HF + fc * CW + 4 * q) : noG, R.g[p]);
        if (ok && r < nr) rmx[p] = amax4(rmx[p], R.g[p]);
      }
    }
  };
  // chunks k+1 .. k+RB in flight (two-pass groups already move twice the bytes per chunk)
  constexpr int RB = NPA == 1 ? 2 : 1;
  Rows ring[RB];
  {
    Rows R0;
    load(0, R0);
#pragma unroll
    for (int i = 0; i < RB; ++i) load(1 + i, ring[i]);
    stage(0, R0);
  }
  __syncthreads();  // chunk 0
  for (int k = 0; k < nch; ++k) {
    const int h = head_of(k);
#ifndef MVML_BWD_NOEDGE
#pragma unroll
    for (int p = 0; p < NPA; ++p) {  // g_a partials of the in-edges of destination d
      const int d = ds + DPP * p;
      const float4 gd = gs[d * LPD + (q ^ bwd_sw<LPD>(d))];
      float t[kEC];
#pragma unroll
      for (int i = 0; i < kEC; ++i) t[i] = grp_sum_hi<LPD>(dot4(zs[zsl[p][i]], gd));
      if (q >= LPD - 4) {  // the group's last 4 lanes write in-edges 0..3, the first of them 4
        const int i0 = q - (LPD - 4);
        const float v = i0 == 0 ? t[0] : i0 == 1 ? t[1] : i0 == 2 ? t[2] : t[3];
        if (i0 < ideg[p]) s_ga[(ieb[p] + i0) * H + h] += v;
        if (i0 == 0 && ideg[p] > 4) s_ga[(ieb[p] + 4) * H + h] += t[4];
      }
      for (int i = kEC; i < (rsg[p] < 0 ? kEC : ideg[p]); ++i) {  // hubs (octet-uniform trip count)
        const int sr = s_src[ieb[p] + i];
        const float v = grp_sum_hi<LPD>(dot4(zs[sr * LPD + (q ^ bwd_sw<LPD>(sr))], gd));
        if (q == LPD - 4) s_ga[(ieb[p] + i) * H + h] += v;
      }
    }
    if constexpr (BIG) {  // hub in-edge segments: edge dots straight into s_ga (one writer each)
      for (int t = ds; t < nsegI; t += DPP) {
        const uint32_t sg = s_segI[t];
        const int d = (int)(sg >> 16), eb = (int)((sg >> 4) & 0xFFFu), c = (int)(sg & 15u) + 1;
        const float4 gd = gs[d * LPD + (q ^ bwd_sw<LPD>(d))];
        float v[kSegI];
#pragma unroll
        for (int j = 0; j < kSegI; ++j) {
          const int sr = s_src[eb + (j < c ? j : 0)];
          v[j] = grp_sum_hi<LPD>(dot4(zs[sr * LPD + (q ^ bwd_sw<LPD>(sr))], gd));
        }
        if (q >= LPD - 4) {  // lane i0 of the last four writes edges i0, i0 + 4
          const int i0 = q - (LPD - 4);
#pragma unroll
          for (int j = 0; j < kSegI; ++j)
            if (j % 4 == i0 && j < c) s_ga[(eb + j) * H + h] += v[j];
        }
      }
    }
#endif
    if constexpr (BIG) {  // hub out-edge segments: partial dZ sums to s_part
      for (int t = ds; t < nsegO; t += DPP) {
        const uint32_t sg = s_segO[t];
        const int c = (int)(sg & 15u) + 1;
        const uint32_t* oe = s_oxe + ((sg >> 4) & 0xFFFu);
        float4 part = f4(0.f);
        for (int j0 = 0; j0 < c; j0 += 4) {  // batches of 4 edges (registers)
          int od[4], sl[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t x = oe[j0 + j < c ? j0 + j : 0];
            od[j] = (int)(x >> 16);
            sl[j] = (int)(x & 0xFFFFu);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j)
            part = fma4(j0 + j < c ? s_att[sl[j] * H + h] : 0.f,
                        gs[od[j] * LPD + (q ^ bwd_sw<LPD>(od[j]))], part);
        }
        s_part[t * LPD + q] = part;
      }
    }
    float4 acc[NPA];  // dZ_agg of the source atoms over their out-edges
#pragma unroll
    for (int p = 0; p < NPA; ++p) {
      acc[p] = f4(0.f);
#ifndef MVML_BWD_NONODE
#pragma unroll
      for (int i = 0; i < kEC; ++i)
        acc[p] = fma4(s_att[(gsl[p][i] >> 16) + h], gs[gsl[p][i] & 0xFFFFu], acc[p]);
      for (int o = ob[p] + kEC; o < ((rsg[p] & 0xFFFFFF) ? ob[p] + kEC : oend[p]); ++o) {
        int od, sl;
        if (BIG && oxb[p] != 0xFFFF) {  // staged (hub partners: one or two edges past kEC)
          const uint32_t x = s_oxe[oxb[p] + o - ob[p] - kEC];
          od = (int)(x >> 16);
          sl = (int)(x & 0xFFFFu);
        } else {
          od = odst(o);
          sl = oslot(o);
        }
        acc[p] = fma4(s_att[sl * H + h], gs[od * LPD + (q ^ bwd_sw<LPD>(od))], acc[p]);
      }
#endif
    }
    __syncthreads();
    if constexpr (BIG) {  // this chunk's out-edge segment partials, in order
#pragma unroll
      for (int p = 0; p < NPA; ++p) {
        const int n = (rsg[p] >> 12) & 0xFFF, sb = rsg[p] & 0xFFF;
        for (int j = 0; j < n; ++j) acc[p] = add4(acc[p], s_part[(sb + j) * LPD + q]);
      }
    }
    stage(k + 1, ring[0]);
#pragma unroll
    for (int i = 0; i + 1 < RB; ++i) ring[i] = ring[i + 1];
    load(k + 1 + RB, ring[RB - 1]);
#pragma unroll
    for (int p = 0; p < NPA; ++p) {
      buf_st4(rG, grow(p) + 4u * (uint32_t)col_of(k), acc[p]);  // rows past the group: dropped
      if (ds + DPP * p < nr) rmx[p] = amax4(rmx[p], acc[p]);
    }
    __syncthreads();
  }
  // the rows' |max| over their LPD lanes (one writer per row; the caller adds d el / d er)
#pragma unroll
  for (int p = 0; p < NPA; ++p) {
    float m = rmx[p];
    gmx = fmaxf(gmx, m);
#pragma unroll
    for (int o = LPD / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (s_rmx && live[p] && q == 0) s_rmx[ds + DPP * p] = m;
  }
  return gmx;
}

// One workgroup of 512 threads per node group (2 per CU): the group's CSR, out-CSR and
// attention are staged in LDS, the column chunks stream through bwd_lds_chunks (one pass for
// groups of <= 64 atoms, two up to kWinL), then the softmax backward runs in LDS.
// BIG (kind bit 2): the big-window variant for the groups on the backward fallback list: 16-column
// chunks, 1024 threads (two passes of 256 rows), out-CSR and logits read from global memory
// (LDS holds the rows, the attention, the edge gradients and the in-CSR), one workgroup per CU
// walking the list.
template <int H, int MODE, int CW, int NT = 16 * CW, int WIN = kWinL, int ECAP = kECap, bool BIG = false>
__global__ void __launch_bounds__(NT, MVML_BWD_WAVES)
gat_agg_bwd_lds_kernel(const int32_t* __restrict__ plan, int64_t G, const int32_t* __restrict__ rowptr,
                       const int32_t* __restrict__ in_src, const int32_t* __restrict__ out_rowptr,
                       const int32_t* __restrict__ out_dst, const int32_t* __restrict__ out_inslot,
                       const float* __restrict__ Y, int64_t ldy, int F, const float* __restrict__ elr,
                       const float* __restrict__ attn, const float* __restrict__ out,
                       const float* __restrict__ g_out, float slope, float* __restrict__ gY,
                       int64_t ldgy, int C, uint32_t* __restrict__ gy_amax,
                       uint32_t* __restrict__ gy_rows) {
  constexpr int LPD = CW / 4;
  constexpr int DPP = NT / LPD;
  constexpr int NPM = WIN / DPP;  // passes over a full window
  static_assert(NPM * DPP == WIN && (NPM == 2 || NPM == 4), "the passes must tile the LDS rows exactly");
  __shared__ float4 zs[WIN * LPD];
  __shared__ float4 gs[WIN * LPD];
  __shared__ float s_att[(ECAP + 1) * H];  // + H zeros: the attention of a missing edge
  __shared__ float s_ga[ECAP * H];
  __shared__ uint16_t s_src[ECAP];
  __shared__ int s_odst[BIG ? 1 : ECAP], s_oslot[BIG ? 1 : ECAP];
  __shared__ int s_rp[WIN + 1], s_orp[WIN + 1];
  __shared__ float s_elr[BIG ? 1 : WIN * 2 * H];
  // BIG: hub segment tables (in-edges, out-edges), per-row segments, out-segment partials
  __shared__ uint32_t s_segI[BIG ? kSegCapI : 1], s_segO[BIG ? kSegCapO : 1];
  __shared__ int s_rs[BIG ? WIN : 1];
  __shared__ float4 s_part[BIG ? kSegCapO * LPD : 1];
  // out-edges past kEC of every row (dst row << 16 | in-slot), from row base s_oxb (0xFFFF:
  // past the table, read from global memory)
  __shared__ uint32_t s_oxe[BIG ? kOXCap : 1];
  __shared__ uint16_t s_oxb[BIG ? WIN : 1];
  __shared__ int s_wsum[BIG ? NT / 64 : 1];
  const GroupPlan gp(plan, G);
  const int nlist = BIG ? gp.count[1] : (int)blockIdx.x + 1;
  float gmx = 0.f;  // |max| of this thread's gY stores, committed once after the group loop
  for (int li = blockIdx.x; li < nlist; li += BIG ? gridDim.x : 1) {
  const int grp = BIG ? gp.bwd_list[li] : li;
  if (BIG) __syncthreads();  // the previous group's LDS reads are done
  if (!(gp.kind[grp] & (BIG ? 4 : 2))) continue;
  const int a0 = gp.start[grp], a1 = gp.start[grp + 1];
  const int tid = threadIdx.x;
  const int nr = a1 - a0, HF = H * F;
  const int ocols = MODE == 1 ? F : HF;
  const int e0 = rowptr[a0], ne = rowptr[a1] - e0;  // = the group's out-edge range too
  for (int i = tid; i <= nr; i += NT) {
    s_rp[i] = rowptr[a0 + i] - e0;
    s_orp[i] = out_rowptr[a0 + i] - e0;
  }
  for (int i = tid; i < ne; i += NT) {
    s_src[i] = (uint16_t)(in_src[e0 + i] - a0);
    if constexpr (!BIG) {
      s_odst[i] = out_dst[e0 + i] - a0;
      s_oslot[i] = out_inslot[e0 + i] - e0;
    }
  }
  for (int i = tid; i < ne * H; i += NT) s_att[i] = attn[(int64_t)e0 * H + i];
  if (tid < H) s_att[ECAP * H + tid] = 0.f;
  if constexpr (!BIG)
    for (int i = tid; i < nr * 2 * H; i += NT) s_elr[i] = elr[(int64_t)a0 * 2 * H + i];
  // BIG: after the chunk sweep the row buffers are free and hold the group's logits (zs) and
  // out-edge slots (gs) for the softmax backward and the d el sums
  float* s_elr_b = reinterpret_cast<float*>(zs);
  int* s_oslot_b = reinterpret_cast<int*>(gs);
  static_assert(!BIG || (WIN * 2 * H <= WIN * LPD * 4 && ECAP <= WIN * LPD * 4), "row buffers hold elr / slots");
  // gy_rows: the rows' |max| in the free row buffer after the sweep, past BIG's logits
  static_assert(WIN * 2 * H + WIN <= WIN * LPD * 4, "row buffer holds the logits and the row maxima");
  float* s_rmx = gy_rows ? reinterpret_cast<float*>(zs) + WIN * 2 * H : nullptr;
  auto elr_at = [&](int r, int c) -> float {  // elr of group row r, column c (el | er)
    if constexpr (BIG) return s_elr_b[r * 2 * H + c]; else return s_elr[r * 2 * H + c];
  };
  const int ldyi = (int)ldy, ldgi = (int)ldgy;
  const __amdgpu_buffer_rsrc_t rY = make_rsrc(Y + (int64_t)a0 * ldy, (uint32_t)(nr * ldyi) * 4u);
  const __amdgpu_buffer_rsrc_t rG = make_rsrc(gY + (int64_t)a0 * ldgy, (uint32_t)(nr * ldgi) * 4u);
  const __amdgpu_buffer_rsrc_t rGo = make_rsrc(g_out + (int64_t)a0 * ocols, (uint32_t)(nr * ocols) * 4u);
  const __amdgpu_buffer_rsrc_t rO = make_rsrc(out + (int64_t)a0 * HF, MODE == 0 ? (uint32_t)(nr * HF) * 4u : 0u);
  for (int i = tid; i < ne * H; i += NT) s_ga[i] = 0.f;
  __syncthreads();  // CSR / attention staged
  int nsegI = 0, nsegO = 0;
  if constexpr (BIG) {
    static_assert(NT >= WIN, "one row per thread for the segment scans");
    const bool lv = tid < nr;
    int rsI, rsO;
    nsegI = hub_segments<NT, kSegI, kSegCapI>(nr, lv ? s_rp[tid] : 0, lv ? s_rp[tid + 1] - s_rp[tid] : 0,
                                              s_segI, &rsI, s_wsum);
    const int ob = lv ? s_orp[tid] : 0, odeg = lv ? s_orp[tid + 1] - ob : 0;
    const int m = max(0, odeg - kEC);
    int mt;
    const int xb = block_excl_scan<NT>(m, s_wsum, &mt);
    const bool xok = xb + m <= kOXCap;
    for (int j = 0; j < (xok ? m : 0); ++j) {
      const int o = ob + kEC + j;
      s_oxe[xb + j] = (uint32_t)(out_dst[e0 + o] - a0) << 16 | (uint32_t)(out_inslot[e0 + o] - e0);
    }
    if (lv) s_oxb[tid] = (uint16_t)(xok && m ? xb : 0xFFFF);
    __syncthreads();  // s_wsum reads of the scan are done
    // out-edge segments index the table: "edge" e = xb + (out-edge - kEC)
    nsegO = hub_segments<NT, kSegO, kSegCapO, kSegMinO>(nr, xb - kEC, xok ? odeg : 0, s_segO, &rsO, s_wsum);
    if (lv) s_rs[tid] = rsO | (rsI ? (int)0x80000000 : 0);
    __syncthreads();
  }
#define MVML_BWD_CHUNKS(NPA)                                                                       \
  gmx = fmaxf(gmx, bwd_lds_chunks<H, MODE, NPA, CW, NT, WIN, ECAP, BIG>(zs, gs, s_att, s_odst, s_oslot, s_orp, s_rp,  \
                                                       s_src, s_ga, rY, ldyi, rGo, rO, rG, ldgi, nr, F, \
                                                       out_dst, out_inslot, e0, a0, s_segI, nsegI, \
                                                       s_segO, nsegO, s_rs, s_part, s_oxe, s_oxb, s_rmx))
  if (nr <= DPP) MVML_BWD_CHUNKS(1);
  else if (NPM == 2 || nr <= 2 * DPP) MVML_BWD_CHUNKS(2);
  else if (nr <= 3 * DPP) MVML_BWD_CHUNKS((NPM > 2 ? 3 : 2));
  else MVML_BWD_CHUNKS(NPM);
#undef MVML_BWD_CHUNKS
  __syncthreads();
  if constexpr (BIG) {
    for (int i = tid; i < nr * 2 * H; i += NT) s_elr_b[i] = elr[(int64_t)a0 * 2 * H + i];
    for (int i = tid; i < ne; i += NT) s_oslot_b[i] = out_inslot[e0 + i] - e0;
    __syncthreads();
  }
  // edge_softmax backward per (destination, head); g_pre replaces g_a in LDS
  for (int i = tid; i < nr * H; i += NT) {
    const int d = i / H, h = i % H;
    const int eb = s_rp[d], ee = s_rp[d + 1];
    const float er = elr_at(d, H + h);
    float dots = 0.f;
    for (int e = eb; e < ee; ++e) dots += s_att[e * H + h] * s_ga[e * H + h];
    float der = 0.f;
    for (int e = eb; e < ee; ++e) {
      const float g_s = s_att[e * H + h] * (s_ga[e * H + h] - dots);
      const float gp = (elr_at(s_src[e], h) + er) > 0.f ? g_s : g_s * slope;
      s_ga[e * H + h] = gp;
      der += gp;
    }
    gY[(int64_t)(a0 + d) * ldgy + C + H + h] = der;
    gmx = fmaxf(gmx, fabsf(der));
    if (s_rmx) atomicMax(reinterpret_cast<uint32_t*>(s_rmx) + d, __float_as_uint(fabsf(der)));
  }
  __syncthreads();
  for (int i = tid; i < nr * H; i += NT) {  // d el: sums over out-edges
    const int u = i / H, h = i % H;
    float del = 0.f;
    for (int o = s_orp[u]; o < s_orp[u + 1]; ++o) {
      int sl;
      if constexpr (BIG) sl = s_oslot_b[o]; else sl = s_oslot[o];
      del += s_ga[sl * H + h];
    }
    gY[(int64_t)(a0 + u) * ldgy + C + h] = del;
    gmx = fmaxf(gmx, fabsf(del));
    if (s_rmx) atomicMax(reinterpret_cast<uint32_t*>(s_rmx) + u, __float_as_uint(fabsf(del)));
  }
  if (s_rmx) {  // (LDS max of non-negative float bits: order-independent)
    __syncthreads();
    for (int r = tid; r < nr; r += NT) gy_rows[a0 + r] = __float_as_uint(s_rmx[r]);
  }
  }
  if (gy_amax) block_amax_commit<NT>(gmx, gy_amax);
}

// Pass A: one wave per destination v.
template <int H, int VPL>
__global__ void __launch_bounds__(kWavesPerBlock * 64)
gat_agg_bwd_dst_kernel(int64_t N, const int32_t* __restrict__ groups, int64_t G,
                       const int32_t* __restrict__ rowptr, const int32_t* __restrict__ in_src,
                       const float* __restrict__ Y, int64_t ldy, const float* __restrict__ elr,
                       const float* __restrict__ attn, const float* __restrict__ out,
                       const float* __restrict__ g_out, int F, float slope, int mode,
                       float* __restrict__ gpre, float* __restrict__ gY, int64_t ldgy,
                       float* __restrict__ gelr, int64_t ldgl, int skip_big,
                       uint32_t* __restrict__ gy_amax, uint32_t* __restrict__ gy_rows) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float gmx = 0.f;  // |max| of this thread's gY stores (block-uniform early returns only)
  // G > 0: one block per backward fallback group of the plan; G == 0: one wave per atom over
  // all atoms
  int64_t v, vend, vstep;
  if (G > 0) {
    const GroupPlan gp(groups, G);
    const int li = list_block(blockIdx.x, gridDim.x, gp.count[1]);
    if (li < 0) return;
    const int g = gp.bwd_list[li];
    if (skip_big && (gp.kind[g] & 4)) return;  // the big-window kernel takes it
    const int a0 = gp.start[g], a1 = gp.start[g + 1];
    v = a0 + wid;
    vend = a1;
    vstep = kWavesPerBlock;
  } else {
    v = xcd_block(blockIdx.x, gridDim.x) * kWavesPerBlock + wid;
    vend = min<int64_t>(v + 1, N);
    vstep = 1;
  }
  for (; v < vend; v += vstep) {
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
  float rmx = 0.f;  // this row's |max| (dR, d er) for gy_rows
#pragma unroll
  for (int c = 0; c < VPL; ++c) {
    const int col = 4 * (lane + 64 * c);
    if (mode != 1) {
      if (okc[c]) {
        st4(gyv + HF + col, gr[c]);
        rmx = amax4(rmx, gr[c]);
      }
    } else if (col < F) {
      const float4 go = ld4(g_out + v * F + col);
      st4(gyv + HF + col, go);
      rmx = amax4(rmx, go);
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
    for (int j = 0; j < cnt; j += 2) {  // two source rows in flight
      const int j1 = min(j + 1, cnt - 1);
      const float* zu0 = Y + (int64_t)rl(u_l, j) * ldy;
      const float* zu1 = Y + (int64_t)rl(u_l, j1) * ldy;
      float4 z0[VPL], z1[VPL];
#pragma unroll
      for (int c = 0; c < VPL; ++c) {
        z0[c] = okc[c] ? ld4(zu0 + 4 * (lane + 64 * c)) : f4(0.f);
        z1[c] = okc[c] ? ld4(zu1 + 4 * (lane + 64 * c)) : f4(0.f);
      }
      float p0[H], p1[H];
#pragma unroll
      for (int h = 0; h < H; ++h) { p0[h] = 0.f; p1[h] = 0.f; }
#pragma unroll
      for (int c = 0; c < VPL; ++c)
        if (okc[c]) {
          add_at<H>(p0, hc[c], dot4(z0[c], gr[c]));
          add_at<H>(p1, hc[c], dot4(z1[c], gr[c]));
        }
      HeadReduce<H>::template all<false>(p0, lane);
      HeadReduce<H>::template all<false>(p1, lane);
#pragma unroll
      for (int h = 0; h < H; ++h) ga_l[h] = (lane == j) ? p0[h] : (lane == j1) ? p1[h] : ga_l[h];
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
  store_heads<H>(gelr + v * ldgl + H, ger, lane);
#pragma unroll
  for (int h = 0; h < H; ++h) rmx = fmaxf(rmx, fabsf(ger[h]));
  gmx = fmaxf(gmx, rmx);
  if (gy_rows) {  // the first writer of the row's |max| (the source pass adds dZ, d el)
    rmx = wave_max(rmx);
    if (lane == 0) gy_rows[v] = __float_as_uint(rmx);
  }
  }
  if (gy_amax) block_amax_commit<kWavesPerBlock * 64>(gmx, gy_amax);
}

// Pass B: one wave per source u (out-CSR gather).
template <int H, int VPL>
__global__ void __launch_bounds__(kWavesPerBlock * 64)
gat_agg_bwd_src_kernel(int64_t N, const int32_t* __restrict__ groups, int64_t G,
                       const int32_t* __restrict__ rowptr, const int32_t* __restrict__ out_rowptr,
                       const int32_t* __restrict__ out_dst, const int32_t* __restrict__ out_inslot,
                       const float* __restrict__ attn, const float* __restrict__ gpre,
                       const float* __restrict__ out, const float* __restrict__ g_out, int F,
                       int mode, float* __restrict__ gY, int64_t ldgy, float* __restrict__ gelr,
                       int64_t ldgl, int skip_big, uint32_t* __restrict__ gy_amax,
                       uint32_t* __restrict__ gy_rows) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float gmx = 0.f;  // |max| of this thread's gY stores (block-uniform early returns only)
  // G > 0: one block per backward fallback group of the plan; G == 0: one wave per atom over
  // all atoms
  int64_t u, vend, vstep;
  if (G > 0) {
    const GroupPlan gp(groups, G);
    const int li = list_block(blockIdx.x, gridDim.x, gp.count[1]);
    if (li < 0) return;
    const int g = gp.bwd_list[li];
    if (skip_big && (gp.kind[g] & 4)) return;  // the big-window kernel takes it
    const int a0 = gp.start[g], a1 = gp.start[g + 1];
    u = a0 + wid;
    vend = a1;
    vstep = kWavesPerBlock;
  } else {
    u = xcd_block(blockIdx.x, gridDim.x) * kWavesPerBlock + wid;
    vend = min<int64_t>(u + 1, N);
    vstep = 1;
  }
  for (; u < vend; u += vstep) {
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
    for (int j = 0; j < cnt; j += 2) {  // two g_rst rows in flight
      const int j1 = min(j + 1, cnt - 1);
      const bool two = j + 1 < cnt;  // (uniform)
      const int w0 = rl(w_l, j), w1 = rl(w_l, j1);
      float a0[H], a1[H];
#pragma unroll
      for (int h = 0; h < H; ++h) { a0[h] = rl(a_l[h], j); a1[h] = rl(a_l[h], j1); }
      const float* gw0 = gY + (int64_t)w0 * ldgy + HF;  // g_rst rows written by the dst pass
      const float* gw1 = gY + (int64_t)w1 * ldgy + HF;
      float4 g0[VPL], g1[VPL];
#pragma unroll
      for (int c = 0; c < VPL; ++c) {
        const int col = 4 * (lane + 64 * c);
        g0[c] = !okc[c] ? f4(0.f) : (mode == 1) ? grst_of(g_out, out, w0, col, HF, F, H, mode) : ld4(gw0 + col);
        g1[c] = !okc[c] ? f4(0.f) : (mode == 1) ? grst_of(g_out, out, w1, col, HF, F, H, mode) : ld4(gw1 + col);
      }
#pragma unroll
      for (int c = 0; c < VPL; ++c)
        if (okc[c]) {
          gz[c] = fma4(pick<H>(a0, hc[c]), g0[c], gz[c]);
          if (two) gz[c] = fma4(pick<H>(a1, hc[c]), g1[c], gz[c]);
        }
    }
  }
  // dZ through the aggregation only; the el / er paths (d el x attn_l + d er x attn_r) reach
  // the projection's gradients through the [d el | d er] columns (mvml_gat_agg_bwd contract)
  float* gyu = gY + u * ldgy;
  float rmx = 0.f;
#pragma unroll
  for (int c = 0; c < VPL; ++c)
    if (okc[c]) {
      st4(gyu + 4 * (lane + 64 * c), gz[c]);
      rmx = amax4(rmx, gz[c]);
    }
  store_heads<H>(gelr + u * ldgl, gel, lane);
#pragma unroll
  for (int h = 0; h < H; ++h) rmx = fmaxf(rmx, fabsf(gel[h]));
  gmx = fmaxf(gmx, rmx);
  if (gy_rows) {  // the destination pass wrote this row's first part (stream order)
    rmx = wave_max(rmx);
    if (lane == 0) gy_rows[u] = max(gy_rows[u], __float_as_uint(rmx));
  }
  }
  if (gy_amax) block_amax_commit<kWavesPerBlock * 64>(gmx, gy_amax);
}

// ---- Head-mean layer backward by SOURCE atom (MVML_OPT_MEAN_SRC) -----------------------------
// In mean mode g_rst = g_out / H does not depend on the head, so both products of the backward
//   dZ[u, h, :] = sum_{e: u -> w} a_e,h g_out[w, :] / H          (update_all(u_mul_e, sum) backward)
//   g_a[e, h]   = <Z[u, h, :], g_out[w, :] / H>                   (the edge-weight gradient)
// are formed by the wave that owns SOURCE u: its projection row Z[u] (H F floats) is read once,
// straight from HBM into registers, and only the F-wide g_out rows of its out-neighbours are
// gathered (from the XCD's L2: xcd_block keeps neighbouring atoms on one XCD) — no LDS window,
// no chunk barriers, whatever the molecule size.  Lane l owns f-columns 4 (l + 64 j) of every
// head, so a g_out row is loaded once per edge (not once per head).  dZ walks the out-edges in
// out-CSR order with the atomwise pass's arithmetic (g_out / H, then fma), so it is bitwise
// the atomwise dZ; g_a is written per edge (one writer: the edge's source) for the softmax pass.
// (ld4nt / st4nt: the projection rows read once and the dZ rows written once pass through
// without displacing the g_out rows the XCD's waves share in L2)
template <int H, int NJ>
__global__ void __launch_bounds__(256)
gat_mean_bwd_src_kernel(int64_t N, const int32_t* __restrict__ out_rowptr,
                        const int32_t* __restrict__ out_dst, const int32_t* __restrict__ out_inslot,
                        const float* __restrict__ Y, int64_t ldy, const float* __restrict__ attn,
                        const float* __restrict__ g_out, int F, float* __restrict__ ga,
                        float* __restrict__ gY, int64_t ldgy, uint32_t* __restrict__ gy_amax,
                        uint32_t* __restrict__ gy_rows) {
  const int lane = threadIdx.x & 63;
  const int64_t u = xcd_block(blockIdx.x, gridDim.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float gmx = 0.f;
  if (u < N) {  // (no early return: block_amax_commit below has a barrier)
    const int nf4 = F / 4, HF = H * F;
    const float hh = (float)H;
    bool okj[NJ];
    float4 z[H][NJ], dz[H][NJ];
    const float* zu = Y + u * ldy;
    float* gyu = gY + u * ldgy;
    float rmx = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int fj = lane + 64 * j;
      okj[j] = fj < nf4;
#pragma unroll
      for (int h = 0; h < H; ++h) {
        z[h][j] = okj[j] ? ld4nt(zu + h * F + 4 * fj) : f4(0.f);
        dz[h][j] = f4(0.f);
      }
      if (okj[j]) {  // dR[u] = g_out[u] (the head-mean residual's gradient)
        const float4 go = ld4(g_out + u * F + 4 * fj);
        st4nt(gyu + HF + 4 * fj, go);
        rmx = amax4(rmx, go);
      }
    }
    const int ob = out_rowptr[u], oe = out_rowptr[u + 1];
    for (int base = ob; base < oe; base += 64) {
      const int cnt = min(64, oe - base);
      int w_l = 0, s_l = 0;
      float a_l[H];
#pragma unroll
      for (int h = 0; h < H; ++h) a_l[h] = 0.f;
      if (lane < cnt) {
        w_l = out_dst[base + lane];
        s_l = out_inslot[base + lane];
#pragma unroll
        for (int h = 0; h < H; ++h) a_l[h] = attn[(int64_t)s_l * H + h];
      }
      // two out-edges per trip: both g_out rows are loaded before either is used
      for (int j = 0; j < cnt; j += 2) {
        const int j1 = min(j + 1, cnt - 1);
        const bool two = j + 1 < cnt;  // (uniform)
        const float* gw0 = g_out + (int64_t)rl(w_l, j) * F;
        const float* gw1 = g_out + (int64_t)rl(w_l, j1) * F;
        float4 g0[NJ], g1[NJ];
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj) {
          g0[jj] = okj[jj] ? ld4(gw0 + 4 * (lane + 64 * jj)) : f4(0.f);
          g1[jj] = okj[jj] ? ld4(gw1 + 4 * (lane + 64 * jj)) : f4(0.f);
        }
        float a0[H], a1[H], p0[H], p1[H];
#pragma unroll
        for (int h = 0; h < H; ++h) { a0[h] = rl(a_l[h], j); a1[h] = rl(a_l[h], j1); p0[h] = 0.f; p1[h] = 0.f; }
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj) {
          const float4 ga4 = make_float4(g0[jj].x / hh, g0[jj].y / hh, g0[jj].z / hh, g0[jj].w / hh);
          const float4 gb4 = make_float4(g1[jj].x / hh, g1[jj].y / hh, g1[jj].z / hh, g1[jj].w / hh);
#pragma unroll
          for (int h = 0; h < H; ++h) {
            dz[h][jj] = fma4(a0[h], ga4, dz[h][jj]);
            p0[h] += dot4(z[h][jj], ga4);
            if (two) dz[h][jj] = fma4(a1[h], gb4, dz[h][jj]);
            p1[h] += dot4(z[h][jj], gb4);
          }
        }
        HeadReduce<H>::template all<false>(p0, lane);
        store_heads<H>(ga + (int64_t)rl(s_l, j) * H, p0, lane);
        if (two) {
          HeadReduce<H>::template all<false>(p1, lane);
          store_heads<H>(ga + (int64_t)rl(s_l, j1) * H, p1, lane);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      if (okj[j]) {
#pragma unroll
        for (int h = 0; h < H; ++h) {
          st4nt(gyu + h * F + 4 * (lane + 64 * j), dz[h][j]);
          rmx = amax4(rmx, dz[h][j]);
        }
      }
    const float wm = wave_max(rmx);
    gmx = fmaxf(gmx, wm);
    if (gy_rows && lane == 0) gy_rows[u] = __float_as_uint(wm);  // the first writer of the row
  }
  if (gy_amax) block_amax_commit<256>(gmx, gy_amax);
}

// edge_softmax + LeakyReLU backward per destination v (thread per atom, the LDS kernel's
// arithmetic and edge order): g_a -> g_pre in place, d er[v] -> gY[v, C + H ..]
template <int H>
__global__ void __launch_bounds__(256)
gat_mean_bwd_softmax_kernel(int64_t N, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ in_src,
                            const float* __restrict__ elr, const float* __restrict__ attn, float slope,
                            float* __restrict__ gpre, float* __restrict__ gY, int64_t ldgy, int C) {
  const int64_t v = xcd_block(blockIdx.x, gridDim.x) * 256 + threadIdx.x;
  if (v >= N) return;
  const int eb = rowptr[v], ee = rowptr[v + 1];
  float er[H], dots[H], der[H];
#pragma unroll
  for (int h = 0; h < H; ++h) { er[h] = elr[v * 2 * H + H + h]; dots[h] = 0.f; der[h] = 0.f; }
  for (int e = eb; e < ee; ++e)
#pragma unroll
    for (int h = 0; h < H; ++h) dots[h] += attn[(int64_t)e * H + h] * gpre[(int64_t)e * H + h];
  for (int e = eb; e < ee; ++e) {
    const float* el = elr + (int64_t)in_src[e] * 2 * H;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float g_s = attn[(int64_t)e * H + h] * (gpre[(int64_t)e * H + h] - dots[h]);
      const float gp = (el[h] + er[h]) > 0.f ? g_s : g_s * slope;
      gpre[(int64_t)e * H + h] = gp;
      der[h] += gp;
    }
  }
#pragma unroll
  for (int h = 0; h < H; ++h) gY[v * ldgy + C + H + h] = der[h];
}

// d el[u] = sum over u's out-edges of g_pre (out-CSR order); the row |max| gains d el / d er.
template <int H>
__global__ void __launch_bounds__(256)
gat_mean_bwd_gel_kernel(int64_t N, const int32_t* __restrict__ out_rowptr,
                        const int32_t* __restrict__ out_inslot, const float* __restrict__ gpre,
                        float* __restrict__ gY, int64_t ldgy, int C, uint32_t* __restrict__ gy_amax,
                        uint32_t* __restrict__ gy_rows) {
  const int64_t u = xcd_block(blockIdx.x, gridDim.x) * 256 + threadIdx.x;
  float m = 0.f;
  if (u < N) {
    float g[H];
#pragma unroll
    for (int h = 0; h < H; ++h) g[h] = 0.f;
    for (int o = out_rowptr[u]; o < out_rowptr[u + 1]; ++o) {
      const float* p = gpre + (int64_t)out_inslot[o] * H;
#pragma unroll
      for (int h = 0; h < H; ++h) g[h] += p[h];
    }
    float* row = gY + u * ldgy + C;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      row[h] = g[h];
      m = fmaxf(m, fmaxf(fabsf(g[h]), fabsf(row[H + h])));
    }
    if (gy_rows) gy_rows[u] = max(gy_rows[u], __float_as_uint(m));
  }
  if (gy_amax) block_amax_commit<256>(m, gy_amax);
}

// ---- Flatten layer backward by source atom (MVML_OPT_FLAT_SRC), for large molecules ----------
// The flatten layer's g_rst (= g_out x ELU'(out)) is per head, so the source-owned form needs
// the g_rst rows of the out-neighbours.  One pass: the wave of source u forms its own g_rst row
// once from g_out[u] and out[u] (ELU'(x) = out + 1 below 0) and writes it as dR[u];
// for each out-edge u -> w it gathers the g_out[w] (and out[w]) rows — read by w's own wave and by
// w's other in-neighbours' waves at about the same time, so from the XCD's L2 — and forms g_rst[w]
// in registers with the same arithmetic, then dZ[u] += a_e g_rst[w] (out-CSR order) and
// g_a[e] = <Z[u], g_rst[w]> per head.  (Round 4 had a two-pass form — every g_rst row written
// first, then gathered — with the same bits; measured slower, deleted in round 5.)
template <int H, int NJ, int MODE, int U = 2>
__global__ void __launch_bounds__(256)
gat_flat_bwd_src1_kernel(int64_t N, const int32_t* __restrict__ out_rowptr,
                         const int32_t* __restrict__ out_dst, const int32_t* __restrict__ out_inslot,
                         const float* __restrict__ Y, int64_t ldy, const float* __restrict__ attn,
                         const float* __restrict__ out, const float* __restrict__ g_out, int F,
                         float* __restrict__ ga, float* __restrict__ gY, int64_t ldgy,
                         uint32_t* __restrict__ gy_amax, uint32_t* __restrict__ gy_rows) {
  const int lane = threadIdx.x & 63;
  const int64_t u = xcd_block(blockIdx.x, gridDim.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float gmx = 0.f;
  if (u < N) {  // (no early return: block_amax_commit below has a barrier)
    const int HF = H * F;
    bool okc[NJ];
    int hc[NJ];
    float4 z[NJ], dz[NJ];
    float rmx = 0.f;
    auto grst = [&](int64_t w, int c) -> float4 {  // g_rst[w, 4 (lane + 64 c) ..]
      const int col = 4 * (lane + 64 * c);
      float4 g = ld4(g_out + w * HF + col);
      if (MODE == 0) {
        const float4 o = ld4(out + w * HF + col);
        g.x *= o.x > 0.f ? 1.f : o.x + 1.f;
        g.y *= o.y > 0.f ? 1.f : o.y + 1.f;
        g.z *= o.z > 0.f ? 1.f : o.z + 1.f;
        g.w *= o.w > 0.f ? 1.f : o.w + 1.f;
      }
      return g;
    };
#pragma unroll
    for (int c = 0; c < NJ; ++c) {
      const int col = 4 * (lane + 64 * c);
      okc[c] = col < HF;
      hc[c] = okc[c] ? col / F : 0;
      z[c] = okc[c] ? ld4nt(Y + u * ldy + col) : f4(0.f);
      dz[c] = f4(0.f);
      if (okc[c]) {  // dR[u] = g_rst[u]
        const float4 g = grst(u, c);
        st4nt(gY + u * ldgy + HF + col, g);
        rmx = amax4(rmx, g);
      }
    }
    const int ob = out_rowptr[u], oe = out_rowptr[u + 1];
    for (int base = ob; base < oe; base += 64) {
      const int cnt = min(64, oe - base);
      int w_l = 0, s_l = 0;
      float a_l[H];
#pragma unroll
      for (int h = 0; h < H; ++h) a_l[h] = 0.f;
      if (lane < cnt) {
        w_l = out_dst[base + lane];
        s_l = out_inslot[base + lane];
#pragma unroll
        for (int h = 0; h < H; ++h) a_l[h] = attn[(int64_t)s_l * H + h];
      }
      for (int j = 0; j < cnt; j += U) {  // U out-neighbours' rows in flight
        float4 g[U][NJ];
#pragma unroll
        for (int t = 0; t < U; ++t) {
          const int64_t wt = rl(w_l, min(j + t, cnt - 1));  // past the chunk: a duplicate row, unused
#pragma unroll
          for (int c = 0; c < NJ; ++c) g[t][c] = okc[c] ? grst(wt, c) : f4(0.f);
        }
#pragma unroll
        for (int t = 0; t < U; ++t) {
          if (j + t >= cnt) break;  // (uniform)
          float a[H], pd[H];
#pragma unroll
          for (int h = 0; h < H; ++h) { a[h] = rl(a_l[h], j + t); pd[h] = 0.f; }
#pragma unroll
          for (int c = 0; c < NJ; ++c)
            if (okc[c]) {
              dz[c] = fma4(pick<H>(a, hc[c]), g[t][c], dz[c]);
              add_at<H>(pd, hc[c], dot4(z[c], g[t][c]));
            }
          HeadReduce<H>::template all<false>(pd, lane);
          store_heads<H>(ga + (int64_t)rl(s_l, j + t) * H, pd, lane);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < NJ; ++c)
      if (okc[c]) {
        st4nt(gY + u * ldgy + 4 * (lane + 64 * c), dz[c]);
        rmx = amax4(rmx, dz[c]);
      }
    const float wm = wave_max(rmx);
    gmx = fmaxf(gmx, wm);
    if (gy_rows && lane == 0) gy_rows[u] = __float_as_uint(wm);  // the first writer of the row
  }
  if (gy_amax) block_amax_commit<256>(gmx, gy_amax);
}

template <int H>
int launch_flat_src1(int64_t N, const int32_t* rp, const int32_t* src, const int32_t* orp,
                     const int32_t* odst, const int32_t* oslot, const float* Y, int64_t ldy,
                     const float* elr, const float* attn, const float* out, const float* g_out, int F,
                     float slope, int mode, float* gpre, float* gY, int64_t ldgy, int C, uint32_t* gy_amax,
                     uint32_t* gy_rows, hipStream_t st) {
  const int HF = H * F;
  const int nj = (int)ceil_div(HF / 4, 64);
  const unsigned b4 = (unsigned)ceil_div(N, 4), b256 = (unsigned)ceil_div(N, 256);
  uint32_t* const blk_amax = gy_rows ? nullptr : gy_amax;  // (see launch_mean_src)
  const bool u1 = option(MVML_OPT_DST_UNR) != 2;  // one out-neighbour row per trip (2: two)
#define MVML_FLAT_SRC1(NJ)                                                                                   \
  do {                                                                                                       \
    if (mode == 0 && u1)                                                                                     \
      gat_flat_bwd_src1_kernel<H, NJ, 0, 1><<<b4, 256, 0, st>>>(                                              \
          N, orp, odst, oslot, Y, ldy, attn, out, g_out, F, gpre, gY, ldgy, blk_amax, gy_rows);               \
    else if (mode == 0)                                                                                      \
      gat_flat_bwd_src1_kernel<H, NJ, 0><<<b4, 256, 0, st>>>(                                                 \
          N, orp, odst, oslot, Y, ldy, attn, out, g_out, F, gpre, gY, ldgy, blk_amax, gy_rows);               \
    else if (u1)                                                                                             \
      gat_flat_bwd_src1_kernel<H, NJ, 2, 1><<<b4, 256, 0, st>>>(                                              \
          N, orp, odst, oslot, Y, ldy, attn, out, g_out, F, gpre, gY, ldgy, blk_amax, gy_rows);               \
    else                                                                                                     \
      gat_flat_bwd_src1_kernel<H, NJ, 2><<<b4, 256, 0, st>>>(                                                 \
          N, orp, odst, oslot, Y, ldy, attn, out, g_out, F, gpre, gY, ldgy, blk_amax, gy_rows);               \
  } while (0)
  switch (nj) {
    case 1: MVML_FLAT_SRC1(1); break;
    case 2: MVML_FLAT_SRC1(2); break;
    case 3: MVML_FLAT_SRC1(3); break;
    case 4: MVML_FLAT_SRC1(4); break;
    case 5: MVML_FLAT_SRC1(5); break;
    case 6: MVML_FLAT_SRC1(6); break;
    case 7: MVML_FLAT_SRC1(7); break;
    case 8: MVML_FLAT_SRC1(8); break;
    default: set_error("gat_agg_bwd: flat-src path needs H F <= 2048"); return MVML_ERR_INVALID;
  }
#undef MVML_FLAT_SRC1
  int rc = check_launch("gat_flat_bwd_src1_kernel");
  if (rc) return rc;
  gat_mean_bwd_softmax_kernel<H><<<b256, 256, 0, st>>>(N, rp, src, elr, attn, slope, gpre, gY, ldgy, C);
  rc = check_launch("gat_mean_bwd_softmax_kernel");
  if (rc) return rc;
  gat_mean_bwd_gel_kernel<H><<<b256, 256, 0, st>>>(N, orp, oslot, gpre, gY, ldgy, C, blk_amax, gy_rows);
  rc = check_launch("gat_mean_bwd_gel_kernel");
  if (rc) return rc;
  return launch_rows_amax(N, gy_rows, gy_amax, st);
}

template <int H>
int launch_mean_src(int64_t N, const int32_t* rp, const int32_t* src, const int32_t* orp,
                    const int32_t* odst, const int32_t* oslot, const float* Y, int64_t ldy,
                    const float* elr, const float* attn, const float* g_out, int F, float slope,
                    float* gpre, float* gY, int64_t ldgy, int C, uint32_t* gy_amax, uint32_t* gy_rows,
                    hipStream_t st) {
  const int nj = (int)ceil_div(F / 4, 64);
  const unsigned b4 = (unsigned)ceil_div(N, 4), b256 = (unsigned)ceil_div(N, 256);
  // with per-row maxima requested, max |gY| comes from them at the end (no per-block atomics)
  uint32_t* const blk_amax = gy_rows ? nullptr : gy_amax;
#define MVML_MEAN_SRC(NJ) \
  gat_mean_bwd_src_kernel<H, NJ><<<b4, 256, 0, st>>>( \
      N, orp, odst, oslot, Y, ldy, attn, g_out, F, gpre, gY, ldgy, blk_amax, gy_rows)
  switch (nj) {
    case 1: MVML_MEAN_SRC(1); break;
    case 2: MVML_MEAN_SRC(2); break;
    case 3: MVML_MEAN_SRC(3); break;
    case 4: MVML_MEAN_SRC(4); break;
    default: set_error("gat_agg_bwd: mean-src path needs F <= 1024"); return MVML_ERR_INVALID;
  }
#undef MVML_MEAN_SRC
  int rc = check_launch("gat_mean_bwd_src_kernel");
  if (rc) return rc;
  gat_mean_bwd_softmax_kernel<H><<<b256, 256, 0, st>>>(N, rp, src, elr, attn, slope, gpre, gY, ldgy, C);
  rc = check_launch("gat_mean_bwd_softmax_kernel");
  if (rc) return rc;
  gat_mean_bwd_gel_kernel<H><<<b256, 256, 0, st>>>(N, orp, oslot, gpre, gY, ldgy, C, blk_amax, gy_rows);
  rc = check_launch("gat_mean_bwd_gel_kernel");
  if (rc) return rc;
  return launch_rows_amax(N, gy_rows, gy_amax, st);
}

template <int H>
int launch_fwd(int64_t N, const int32_t* groups, int64_t G, const int32_t* rp, const int32_t* src,
               const float* Y, int64_t ldy, int F, const float* bias, float slope, int mode,
               float* out, float* attn, const float* elr, uint32_t* out_amax, uint32_t* out_rows,
               hipStream_t st) {
  if (option(MVML_OPT_DST_FWD) && H * F <= 2048) {  // one wave per destination atom, every atom
    const unsigned b4 = (unsigned)ceil_div(N, 4);
    const int HF = H * F;
    const bool sm = option(MVML_OPT_DST_FWD) == 1;  // 2: the softmax as its own launch first
    // with per-row maxima requested, max |out| comes from them afterwards (no per-block atomics)
    uint32_t* const blk_amax = out_rows ? nullptr : out_amax;
    if (!sm && H == 4) {
      gat_softmax_dst4_kernel<<<(unsigned)ceil_div(N, 256), 256, 0, st>>>(N, rp, src, elr, slope, attn);
      int rc = check_launch("gat_softmax_dst4_kernel");
      if (rc) return rc;
    } else if (!sm) {
      gat_softmax_dst_kernel<H><<<(unsigned)ceil_div(N * H, 256), 256, 0, st>>>(N, rp, src, elr, slope, attn);
      int rc = check_launch("gat_softmax_dst_kernel");
      if (rc) return rc;
    }
#define MVML_DST_FWD(M, NJ, U)                                                                    \
  do {                                                                                            \
    if (sm)                                                                                       \
      gat_agg_fwd_dst_kernel<H, M, NJ, U, true>                                                   \
          <<<b4, 256, 0, st>>>(   \
              N, rp, src, Y, ldy, F, bias, elr, slope, attn, out, blk_amax, out_rows);             \
    else                                                                                          \
      gat_agg_fwd_dst_kernel<H, M, NJ, U, false>                                                  \
          <<<b4, 256, 0, st>>>(  \
              N, rp, src, Y, ldy, F, bias, elr, slope, attn, out, blk_amax, out_rows);             \
  } while (0)
    // rows in flight per wave (MVML_OPT_DST_UNR, H = 4 at the GAT widths: tuning A/B)
    const int unr = option(MVML_OPT_DST_UNR);
    if (mode == 1) {  // mean: half-waves over the heads, lanes over F / 4
      const int nj = (int)ceil_div(F / 4, H >= 2 ? 32 : 64);
      if (nj == 1) MVML_DST_FWD(1, 1, 4);
      else if (nj == 2) MVML_DST_FWD(1, 2, 2);
      else if (nj == 3 && H == 4 && unr == 2) MVML_DST_FWD(1, 3, 2);
      else if (nj == 3 && H == 4 && unr == 3) MVML_DST_FWD(1, 3, 3);
      else if (nj == 3 && unr == 6) MVML_DST_FWD(1, 3, 1);  // (6: the residual loaded first)
      else if (nj == 3 && H == 4) {
        // one row in flight, the residual loaded after the gather: 90 VGPRs, five waves per SIMD
        // (residual first: 104, four) — config 5 layer 2 6.35 -> 6.08 ms, config 3 3.66 -> 3.60
        // (profiles/r05_agg_late_residual_config*.txt)
        if (sm)
          gat_agg_fwd_dst_kernel<H, 1, 3, 1, true, true><<<b4, 256, 0, st>>>(
              N, rp, src, Y, ldy, F, bias, elr, slope, attn, out, blk_amax, out_rows);
        else
          gat_agg_fwd_dst_kernel<H, 1, 3, 1, false, true><<<b4, 256, 0, st>>>(
              N, rp, src, Y, ldy, F, bias, elr, slope, attn, out, blk_amax, out_rows);
      }
      else if (nj == 3) MVML_DST_FWD(1, 3, 1);  // one row in flight: fewest registers, most waves
      else if (nj <= 4) MVML_DST_FWD(1, 4, 2);
      else { set_error("gat_agg_fwd: dst path needs F <= %d in mean mode", H >= 2 ? 512 : 1024); return MVML_ERR_INVALID; }
    } else {
      const int nj = (int)ceil_div(HF / 4, 64);
#define MVML_DST_FWD_F(NJ, U) do { if (mode == 0) MVML_DST_FWD(0, NJ, U); else MVML_DST_FWD(2, NJ, U); } while (0)
      if (nj == 1) MVML_DST_FWD_F(1, 4);
      else if (nj == 2) MVML_DST_FWD_F(2, 4);
      else if (nj == 3 && H == 4 && unr == 2) MVML_DST_FWD_F(3, 2);
      else if (nj == 3 && H == 4 && unr == 4) MVML_DST_FWD_F(3, 4);
      else if (nj == 3 && H == 4 && (unr == 5 || (unr == 0 && sm))) {
        // late residual (60 VGPRs, eight waves per SIMD instead of six): with the fused softmax
        // (large molecules) config-5 layer 1 4.90 -> 4.41 ms; the split-softmax form (small
        // molecules) measured even (profiles/r05_agg_late_residual_flatten_config*.txt)
#define MVML_DST_FWD_LR(M)                                                                        \
  do {                                                                                            \
    if (sm)                                                                                       \
      gat_agg_fwd_dst_kernel<H, M, 3, 1, true, true><<<b4, 256, 0, st>>>(                         \
          N, rp, src, Y, ldy, F, bias, elr, slope, attn, out, blk_amax, out_rows);                 \
    else                                                                                          \
      gat_agg_fwd_dst_kernel<H, M, 3, 1, false, true><<<b4, 256, 0, st>>>(                        \
          N, rp, src, Y, ldy, F, bias, elr, slope, attn, out, blk_amax, out_rows);                 \
  } while (0)
        if (mode == 0) MVML_DST_FWD_LR(0); else MVML_DST_FWD_LR(2);
#undef MVML_DST_FWD_LR
      }
      else if (nj == 3) MVML_DST_FWD_F(3, 1);  // fewer rows in flight, more waves: faster
      else if (nj == 4) MVML_DST_FWD_F(4, 2);
      else MVML_DST_FWD_F(8, 2);
#undef MVML_DST_FWD_F
    }
#undef MVML_DST_FWD
    int rc = check_launch("gat_agg_fwd_dst_kernel");
    if (rc) return rc;
    return launch_rows_amax(N, out_rows, out_amax, st);
  }
  if (G == 0) return MVML_OK;
  const bool big = use_big_window(H, F);
  // the edge_softmax runs inside each kernel for its own groups (no separate softmax launch)
#define MVML_AGG_FWD_M(CW, M)                                                                       \
  do {                                                                                              \
    gat_agg_fwd_lds_kernel<H, CW, M, CW * 16><<<(unsigned)G, CW * 16, 0, st>>>(groups, G, rp, src, Y, ldy, F, \
                                                                         bias, elr, slope, attn, out, out_amax, out_rows); \
    gat_agg_fwd_gather_kernel<H, CW, M><<<(unsigned)G, kAggThreads, 0, st>>>(groups, G, rp, src, Y, ldy, \
                                                                            F, bias, elr, slope, attn, out, big, out_amax, out_rows); \
    if constexpr (H <= 4)                                                                           \
      if (big)                                                                                      \
        gat_agg_fwd_lds_kernel<H, 16, M, kBigThreads, kPlanBigAtoms, kPlanBigEdgeCap, true>          \
            <<<(unsigned)std::min<int64_t>(G, kBigBlocks), kBigThreads, 0, st>>>(                    \
                groups, G, rp, src, Y, ldy, F, bias, elr, slope, attn, out, out_amax, out_rows);    \
  } while (0)
#define MVML_AGG_FWD(CW)                                  \
  do {                                                    \
    if (mode == 0) MVML_AGG_FWD_M(CW, 0);                 \
    else if (mode == 1) MVML_AGG_FWD_M(CW, 1);            \
    else MVML_AGG_FWD_M(CW, 2);                           \
  } while (0)
// Widest column chunk of the forward LDS kernel: 32 (two 512-thread workgroups per CU, so one
// group's softmax and first loads overlap the other's chunk sweep) measured 3-5 % faster than
// 64 (one 1024-thread workgroup per CU) on configs 2 and 3 (profiles/r04_fwd_chunk_width.txt).
#ifndef MVML_FWD_CWMAX
#define MVML_FWD_CWMAX 32
#endif
  if (MVML_FWD_CWMAX >= 64 && F % 64 == 0) MVML_AGG_FWD(64);
  else if (MVML_FWD_CWMAX >= 32 && F % 32 == 0) MVML_AGG_FWD(32);
  else if (F % 16 == 0) MVML_AGG_FWD(16);
  else if (F % 8 == 0) MVML_AGG_FWD(8);
  else MVML_AGG_FWD(4);
#undef MVML_AGG_FWD
#undef MVML_AGG_FWD_M
  return check_launch("gat_agg_fwd_kernel");
}

template <int H, int VPL>
int launch_bwd(int64_t N, const int32_t* groups, int64_t G, const int32_t* rp, const int32_t* src,
               const int32_t* orp, const int32_t* odst, const int32_t* oslot, const float* Y,
               int64_t ldy, const float* elr, const float* attn, const float* out,
               const float* g_out, int F, float slope, int mode, float* gpre, float* gY,
               int64_t ldgy, int C, uint32_t* gy_amax, uint32_t* gy_rows, hipStream_t st) {
  if (mode == 1 && option(MVML_OPT_MEAN_SRC) && F <= 1024)  // head-mean layer by source atom
    return launch_mean_src<H>(N, rp, src, orp, odst, oslot, Y, ldy, elr, attn, g_out, F, slope, gpre, gY,
                              ldgy, C, gy_amax, gy_rows, st);
  // flatten layer by source atom, one pass (round 5; the round-4 two-pass form — g_rst rows
  // written first, then gathered — computed the same bits and was measured slower: deleted)
  if (mode != 1 && option(MVML_OPT_FLAT_SRC))
    return launch_flat_src1<H>(N, rp, src, orp, odst, oslot, Y, ldy, elr, attn, out, g_out, F, slope, mode,
                               gpre, gY, ldgy, C, gy_amax, gy_rows, st);
  if (option(MVML_OPT_BWD_ATOMWISE)) G = 0;  // tests: the per-atom pair over every atom
  if (F % 32 == 0 && G > 0) {  // molecule groups: one pass over Z / g_out / dZ per group
#ifndef MVML_BWD_CW64
#define MVML_BWD_CW64 0
#endif
    // 32-column chunks (two 512-thread workgroups per CU); MVML_BWD_CW64=1: 64-column chunks
    // (256-B row segments, half the chunks and barriers; one 1024-thread workgroup per CU),
    // measured 1-2 % slower in round 4 (profiles/r04_fwd_chunk_width.txt, second part)
#define MVML_BWD_LDS(M, CW)                                                                       \
    gat_agg_bwd_lds_kernel<H, M, CW><<<(unsigned)G, 16 * CW, 0, st>>>(groups, G, rp, src, orp, odst, \
                                                                      oslot, Y, ldy, F, elr, attn, \
                                                                      out, g_out, slope, gY, ldgy, C, gy_amax, gy_rows)
    if (MVML_BWD_CW64 && F % 64 == 0) {
      if (mode == 0) MVML_BWD_LDS(0, 64);
      else if (mode == 1) MVML_BWD_LDS(1, 64);
      else MVML_BWD_LDS(2, 64);
    } else {
      if (mode == 0) MVML_BWD_LDS(0, 32);
      else if (mode == 1) MVML_BWD_LDS(1, 32);
      else MVML_BWD_LDS(2, 32);
    }
#undef MVML_BWD_LDS
    int rc = check_launch("gat_agg_bwd_lds_kernel");
    if (rc) return rc;
  } else {
    G = 0;  // no LDS groups: the per-atom pair covers every atom
  }
  const int big = G > 0 && use_big_window(H, F);
  if constexpr (H <= 4) {
    if (big) {
#define MVML_BWD_BIG(M)                                                                             \
      gat_agg_bwd_lds_kernel<H, M, 16, kBigThreads, kPlanBigAtoms, kPlanBigEdgeCap, true>            \
          <<<(unsigned)std::min<int64_t>(G, kBigBlocks), kBigThreads, 0, st>>>(                      \
              groups, G, rp, src, orp, odst, oslot, Y, ldy, F, elr, attn, out, g_out, slope, gY, ldgy, C, gy_amax, gy_rows)
      if (mode == 0) MVML_BWD_BIG(0);
      else if (mode == 1) MVML_BWD_BIG(1);
      else MVML_BWD_BIG(2);
#undef MVML_BWD_BIG
      int rc = check_launch("gat_agg_bwd_lds_kernel(big)");
      if (rc) return rc;
    }
  }
  const unsigned blocks = G > 0 ? (unsigned)G : (unsigned)ceil_div(N, kWavesPerBlock);
  gat_agg_bwd_dst_kernel<H, VPL><<<blocks, kWavesPerBlock * 64, 0, st>>>(
      N, groups, G, rp, src, Y, ldy, elr, attn, out, g_out, F, slope, mode, gpre, gY, ldgy, gY + C, ldgy, big,
      gy_amax, gy_rows);
  int rc = check_launch("gat_agg_bwd_dst_kernel");
  if (rc) return rc;
  gat_agg_bwd_src_kernel<H, VPL><<<blocks, kWavesPerBlock * 64, 0, st>>>(
      N, groups, G, rp, orp, odst, oslot, attn, gpre, out, g_out, F, mode, gY, ldgy, gY + C, ldgy, big,
      gy_amax, gy_rows);
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
  MVML_REQUIRE(ldy < (1 << 20), "%s: leading dimension too large", who);
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
                                         int64_t ldy, const float* __restrict__ gelr, int64_t ldgl,
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
      const float* g = gelr + (r + j) * ldgl;
      sl[j] = fmaf(g[h], z, sl[j]);
      sr[j] = fmaf(g[H + h], z, sr[j]);
    }
  }
  for (; r < r1; ++r) {
    const float z = Y[r * ldy + col];
    const float* g = gelr + r * ldgl;
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
                                    const float* __restrict__ attn_lr, int H, int F, int Fin,
                                    int ldw, int mean_res, float* __restrict__ Wcat) {
  const int HF = H * F;
  const int RW = mean_res ? F : HF;
  const int64_t total = (int64_t)(HF + RW + (attn_lr ? 2 * H : 0)) * ldw;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)(e / ldw), k = (int)(e % ldw);
    float v;
    if (k >= Fin) {
      v = 0.f;
    } else if (row < HF) {
      v = fc_w[(int64_t)row * Fin + k];
    } else if (row >= HF + RW) {  // A_l / A_r rows: sum_f attn[h, f] fc.weight[h F + f, k]
      const int side = (row - HF - RW) / H, h = (row - HF - RW) % H;
      const float* a = attn_lr + side * HF + h * F;
      float acc = 0.f;
      for (int f = 0; f < F; ++f) acc = fmaf(a[f], fc_w[(int64_t)(h * F + f) * Fin + k], acc);
      v = acc;
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

// dL/dfc.weight = gWcat[0:HF] (+ attn_l[h,f] gWcat[C+h] + attn_r[h,f] gWcat[C+H+h]: the el / er
// paths, when the backward folded them into the GEMM);  dL/dres_fc.weight[hF+f] =
// gWcat[HF+hF+f] or gWcat[HF+f] / H.
__global__ void unfold_w_kernel(const float* __restrict__ gW, const float* __restrict__ attn_lr,
                                int H, int F, int Fin, int ldg, int mean_res,
                                float* __restrict__ g_fc, float* __restrict__ g_res) {
  const int HF = H * F;
  const int C = HF + (mean_res ? F : HF);
  const int64_t total = (int64_t)HF * Fin;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)(e / Fin), k = (int)(e % Fin);
    float gf = gW[(int64_t)row * ldg + k];
    if (attn_lr) {
      const int h = row / F;
      gf = fmaf(attn_lr[row], gW[(int64_t)(C + h) * ldg + k], gf);
      gf = fmaf(attn_lr[HF + row], gW[(int64_t)(C + H + h) * ldg + k], gf);
    }
    g_fc[e] = gf;
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

extern "C" size_t mvml_gat_proj_fwd_workspace_size(int64_t num_nodes, int H, int F) {
  // logit partials, then 256 B for the split-fp16 operand maxima
  return carve_size((size_t)num_nodes * 2 * (H * F / (1 << proj_logw(F))) * sizeof(float)) + 256;
}

extern "C" int mvml_gat_proj_fwd(int64_t num_nodes, const float* X, int64_t ldx, int64_t K,
                                 const float* Wcat, int64_t ldw, const float* attn_lr, int H,
                                 int F, int mean_residual, int algo, float* Y, int64_t ldy,
                                 float* elr, const uint32_t* amax_x, const uint32_t* amax_w,
                                 const uint16_t* w_planes, int64_t w_plane, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  clear_error();
  MVML_REQUIRE(H == 1 || H == 2 || H == 4 || H == 8, "gat_proj_fwd: num_heads must be 1, 2, 4 or 8 (got %d)", H);
  MVML_REQUIRE(F > 0 && F % 4 == 0, "gat_proj_fwd: out_feats must be a positive multiple of 4 (got %d)", F);
  MVML_REQUIRE(num_nodes >= 0 && K > 0 && ldx >= K && ldw >= K, "gat_proj_fwd: bad shape");
  const int C = mvml_gat_proj_cols(H, F, mean_residual);
  MVML_REQUIRE(ldy >= C, "gat_proj_fwd: ldy < %d", C);
  if (num_nodes == 0) return MVML_OK;
  if (!workspace || workspace_bytes < mvml_gat_proj_fwd_workspace_size(num_nodes, H, F)) {
    set_error("gat_proj_fwd: workspace of mvml_gat_proj_fwd_workspace_size bytes required");
    return MVML_ERR_WORKSPACE;
  }
  MVML_REQUIRE(attn_lr != nullptr && elr != nullptr, "gat_proj_fwd: attn_lr and elr are required");
  hipStream_t st = as_stream(stream);
  float* part = static_cast<float*>(workspace);
  MVML_REQUIRE(algo == MVML_GEMM_F32 || algo == MVML_GEMM_F32X3 || algo == MVML_GEMM_BF16 ||
                   algo == MVML_GEMM_F16X2,
               "gat_proj_fwd: bad algo %d", algo);
  uint32_t* amax_ws = reinterpret_cast<uint32_t*>(
      static_cast<uint8_t*>(workspace) +
      carve_size((size_t)num_nodes * 2 * (H * F / (1 << proj_logw(F))) * sizeof(float)));
  int rc = gemm_proj_epi(algo, num_nodes, C, K, X, ldx, Wcat, ldw, Y, ldy,
                         attn_lr, H * F, proj_logw(F), part, amax_ws, amax_x, amax_w, w_planes,
                         w_plane, st);
  if (rc) return rc;
  const int W = 1 << proj_logw(F);
  const unsigned blocks = (unsigned)ceil_div(num_nodes * 2 * H, 256);
  switch (H) {
    case 1: gat_logits_finalize_kernel<1><<<blocks, 256, 0, st>>>(num_nodes, F, W, part, elr); break;
    case 2: gat_logits_finalize_kernel<2><<<blocks, 256, 0, st>>>(num_nodes, F, W, part, elr); break;
    case 4: gat_logits_finalize_kernel<4><<<blocks, 256, 0, st>>>(num_nodes, F, W, part, elr); break;
    case 8: gat_logits_finalize_kernel<8><<<blocks, 256, 0, st>>>(num_nodes, F, W, part, elr); break;
  }
  return check_launch("gat_logits_finalize_kernel");
}

extern "C" int mvml_gat_agg_fwd(int64_t num_nodes, const int32_t* node_groups, int64_t num_groups,
                                const int32_t* in_rowptr, const int32_t* in_src, const float* Y,
                                int64_t ldy, int H, int F, const float* elr, const float* bias,
                                float slope, int mode, float* out, float* attn, uint32_t* out_amax,
                                uint32_t* out_row_amax, void* stream) {
  clear_error();
  int rc = check_shapes(H, F, mode, ldy, Y, "gat_agg_fwd");
  if (rc) return rc;
  MVML_REQUIRE(((uintptr_t)out & 15) == 0 && ((uintptr_t)bias & 15) == 0,
               "gat_agg_fwd: out / bias must be 16-byte aligned");
  MVML_REQUIRE(attn != nullptr && elr != nullptr, "gat_agg_fwd: elr input and attn output are required");
  MVML_REQUIRE(num_groups == mvml_node_group_count(num_nodes) && (num_groups == 0 || node_groups),
               "gat_agg_fwd: node_groups must come from mvml_build_node_groups (%lld groups expected)",
               (long long)mvml_node_group_count(num_nodes));
  if (num_nodes == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  switch (H) {
    case 1: return launch_fwd<1>(num_nodes, node_groups, num_groups, in_rowptr, in_src, Y, ldy, F, bias, slope, mode, out, attn, elr, out_amax, out_row_amax, st);
    case 2: return launch_fwd<2>(num_nodes, node_groups, num_groups, in_rowptr, in_src, Y, ldy, F, bias, slope, mode, out, attn, elr, out_amax, out_row_amax, st);
    case 4: return launch_fwd<4>(num_nodes, node_groups, num_groups, in_rowptr, in_src, Y, ldy, F, bias, slope, mode, out, attn, elr, out_amax, out_row_amax, st);
    case 8: return launch_fwd<8>(num_nodes, node_groups, num_groups, in_rowptr, in_src, Y, ldy, F, bias, slope, mode, out, attn, elr, out_amax, out_row_amax, st);
  }
  set_error("gat_agg_fwd: unsupported shape");
  return MVML_ERR_INVALID;
}

extern "C" size_t mvml_gat_agg_bwd_workspace_size(int64_t num_edges, int H) {
  return carve_size((size_t)num_edges * H * sizeof(float));
}

extern "C" int mvml_gat_agg_bwd(int64_t num_nodes, const int32_t* node_groups, int64_t num_groups,
                                const int32_t* in_rowptr, const int32_t* in_src,
                                const int32_t* out_rowptr, const int32_t* out_dst,
                                const int32_t* out_inslot, const float* Y, int64_t ldy,
                                const float* elr, const float* attn, const float* out,
                                const float* g_out, int H, int F, float slope, int mode, float* gY,
                                int64_t ldgy, uint32_t* gy_amax, uint32_t* gy_row_amax, void* workspace,
                                size_t workspace_bytes, void* stream) {
  clear_error();
  int rc = check_shapes(H, F, mode, ldy, Y, "gat_agg_bwd");
  if (rc) return rc;
  const int C = mvml_gat_proj_cols(H, F, mode == 1);
  MVML_REQUIRE(ldgy >= C + 2 * H && ldgy % 4 == 0 && ldgy < (1 << 20),
               "gat_agg_bwd: ldgy must be >= proj_cols + 2H = %d and a multiple of 4", C + 2 * H);
  MVML_REQUIRE(attn != nullptr && elr != nullptr, "gat_agg_bwd: attn / elr from the forward are required");
  MVML_REQUIRE(mode != 0 || out != nullptr, "gat_agg_bwd: mode 0 needs the forward output");
  MVML_REQUIRE(num_groups == mvml_node_group_count(num_nodes) && (num_groups == 0 || node_groups),
               "gat_agg_bwd: node_groups must come from mvml_build_node_groups");
  if (num_nodes == 0) return MVML_OK;
  if (!workspace || workspace_bytes == 0) {
    set_error("gat_agg_bwd: workspace of mvml_gat_agg_bwd_workspace_size(E, H) bytes required");
    return MVML_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  float* gpre = static_cast<float*>(workspace);
  const int vpl = (int)ceil_div(H * F, 256);
  switch (H) {
    case 1: { MVML_VPL_CASES(launch_bwd, 1, num_nodes, node_groups, num_groups, in_rowptr, in_src, out_rowptr, out_dst, out_inslot, Y, ldy, elr, attn, out, g_out, F, slope, mode, gpre, gY, ldgy, C, gy_amax, gy_row_amax, st) break; }
    case 2: { MVML_VPL_CASES(launch_bwd, 2, num_nodes, node_groups, num_groups, in_rowptr, in_src, out_rowptr, out_dst, out_inslot, Y, ldy, elr, attn, out, g_out, F, slope, mode, gpre, gY, ldgy, C, gy_amax, gy_row_amax, st) break; }
    case 4: { MVML_VPL_CASES(launch_bwd, 4, num_nodes, node_groups, num_groups, in_rowptr, in_src, out_rowptr, out_dst, out_inslot, Y, ldy, elr, attn, out, g_out, F, slope, mode, gpre, gY, ldgy, C, gy_amax, gy_row_amax, st) break; }
    case 8: { MVML_VPL_CASES(launch_bwd, 8, num_nodes, node_groups, num_groups, in_rowptr, in_src, out_rowptr, out_dst, out_inslot, Y, ldy, elr, attn, out, g_out, F, slope, mode, gpre, gY, ldgy, C, gy_amax, gy_row_amax, st) break; }
  }
  set_error("gat_agg_bwd: unsupported shape");
  return MVML_ERR_INVALID;
}

extern "C" size_t mvml_gat_attn_grad_workspace_size(int64_t num_nodes, int H, int F) {
  return carve_size((size_t)attn_grad_splits(num_nodes, H * F) * 2 * H * F * sizeof(float));
}

extern "C" int mvml_gat_attn_grad(int64_t num_nodes, int H, int F, const float* Y, int64_t ldy,
                                  const float* gelr, int64_t ldgl, float* g_attn_l, float* g_attn_r,
                                  void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  MVML_REQUIRE(H > 0 && F > 0 && num_nodes >= 0 && ldy >= (int64_t)H * F && ldgl >= 2 * H,
               "gat_attn_grad: bad shape");
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
  attn_grad_partial_kernel<<<g1, 256, 0, st>>>(num_nodes, H, F, Y, ldy, gelr, ldgl, rows_per, part);
  attn_grad_final_kernel<<<(unsigned)ceil_div(2 * HF, 256), 256, 0, st>>>(HF, S, part, g_attn_l, g_attn_r);
  return check_launch("attn_grad");
}

extern "C" int mvml_gat_fold_weights(const float* fc_w, const float* res_fc_w, const float* attn_lr,
                                     int H, int F, int Fin, int ldw, int mean_residual, float* Wcat,
                                     void* stream) {
  clear_error();
  MVML_REQUIRE(H > 0 && F > 0 && Fin > 0 && ldw >= Fin, "gat_fold_weights: bad shape");
  hipStream_t st = as_stream(stream);
  const int64_t total = (int64_t)(mvml_gat_proj_cols(H, F, mean_residual) + (attn_lr ? 2 * H : 0)) * ldw;
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(total, 256), 8192);
  fold_weights_kernel<<<blocks, 256, 0, st>>>(fc_w, res_fc_w, attn_lr, H, F, Fin, ldw, mean_residual, Wcat);
  return check_launch("fold_weights_kernel");
}

extern "C" int mvml_gat_unfold_grads(const float* gWcat, const float* attn_lr, int H, int F,
                                     int Fin, int ldg, int mean_residual, float* g_fc_w,
                                     float* g_res_fc_w, void* stream) {
  clear_error();
  MVML_REQUIRE(H > 0 && F > 0 && Fin > 0 && ldg >= Fin, "gat_unfold_grads: bad shape");
  hipStream_t st = as_stream(stream);
  const int64_t total = (int64_t)H * F * Fin;
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(total, 256), 8192);
  unfold_w_kernel<<<blocks, 256, 0, st>>>(gWcat, attn_lr, H, F, Fin, ldg, mean_residual, g_fc_w, g_res_fc_w);
  return check_launch("unfold_w_kernel");
}
