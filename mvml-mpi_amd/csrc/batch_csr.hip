// Device-side graph batching: dgl.batch (dataset.py:52-54) + in/out CSR construction.
//
// Layout produced (all int32 unless noted), N = sum of nodes, E = sum of edges:
//   node_offsets/edge_offsets int64[B+1]  exclusive cumsum of batch_num_nodes / _edges
//   src/dst[E]        global ids, edge order = graph order then each graph's local order
//   node_graph[N]     molecule id of every atom (Set2Set / readout segments)
//   in_rowptr[N+1], in_src[E], in_eid[E]       rows = dst, stable in edge id
//   out_rowptr[N+1], out_dst[E], out_inslot[E]  rows = src, stable in edge id; out_inslot
//                                               is the in-CSR slot of the same edge
// Molecules are independent and small, so the CSR is built by ONE WAVE per molecule
// (build_csr_wave_kernel, molecules up to 256 atoms / 1024 edges); larger graphs take ONE
// workgroup each (build_csr_kernel): the per-graph degree histogram lives in LDS (graphs above
// kLdsNodes atoms fall back to a workspace histogram) and the stable placement walks the edges
// in 256-edge chunks, ranking equal keys inside a chunk by lane order.  Integer atomics are used only for histogram
// counts (order-independent), so the output is deterministic and bit-exact with the oracle
// (oracle/graph_ref.py: csr_ref).
#include "common.h"

namespace mvml {
namespace {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 4;
constexpr int kScanTile = kScanThreads * kScanItems;  // 1024 items per block
constexpr int kCsrThreads = 256;
constexpr int kLdsNodes = 4096;
constexpr int kWaveMolAtoms = 128;   // build_csr_wave_kernel: one wave per molecule up to these
constexpr int kWaveMolEdges = 512;   // ... sizes (LDS: 3 KB per wave, 4 waves per workgroup: 8
                                     // workgroups per CU; 6 KB slices held occupancy to 6)
constexpr int kBigMolAtoms = 1024;   // build_csr_bigwave_kernel: one wave per molecule up to
constexpr int kBigMolEdges = 4096;   // ... these sizes (LDS: 24 KB per one-wave workgroup)

template <typename T>
__device__ T block_exclusive_scan(T v, T* lds_waves /*[kWaves]*/, T* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  T x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) lds_waves[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    T run = 0;
    for (int w = 0; w < nw; ++w) {
      T t = lds_waves[w];
      lds_waves[w] = run;
      run += t;
    }
    lds_waves[nw] = run;
  }
  __syncthreads();
  T res = x - v + lds_waves[wid];
  *total = lds_waves[nw];
  __syncthreads();
  return res;
}

// Both offset scans (atoms, edges) in one set of launches: grid y / block index picks the array.
struct Scan2 {
  const int64_t* in[2];
  int64_t* out[2];
  int64_t* tmp[2];
  int32_t* zero[2] = {nullptr, nullptr};  // two words each, zeroed by the first kernel (the
                                          // CSR build's status flags and list counts: no memsets)
};
__global__ void scan2_tile_sums(Scan2 a, int64_t n) {
  const int y = blockIdx.y;
  if (blockIdx.x == 0 && threadIdx.x < 2 && a.zero[y]) a.zero[y][threadIdx.x] = 0;
  __shared__ int64_t w[kScanThreads / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i)
    if (base + i < n) s += a.in[y][base + i];
  int64_t tot;
  block_exclusive_scan<int64_t>(s, w, &tot);
  if (threadIdx.x == 0) a.tmp[y][blockIdx.x] = tot;
}
__global__ void scan2_sums_single(Scan2 a, int64_t nt) {
  int64_t* sums = a.tmp[blockIdx.x];
  __shared__ int64_t w[kScanThreads / 64 + 1];
  int64_t carry = 0;
  for (int64_t b = 0; b < nt; b += kScanThreads) {
    const int64_t i = b + threadIdx.x;
    const int64_t v = i < nt ? sums[i] : 0;
    int64_t tot;
    const int64_t ex = block_exclusive_scan<int64_t>(v, w, &tot);
    if (i < nt) sums[i] = ex + carry;
    carry += tot;
  }
}
__global__ void scan2_tile_apply(Scan2 a, int64_t n) {
  const int y = blockIdx.y;
  __shared__ int64_t w[kScanThreads / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  int64_t v[kScanItems];
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    v[i] = (base + i < n) ? a.in[y][base + i] : 0;
    s += v[i];
  }
  int64_t tot;
  int64_t ex = block_exclusive_scan<int64_t>(s, w, &tot) + a.tmp[y][blockIdx.x];
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    if (base + i < n) a.out[y][base + i] = ex;
    ex += v[i];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == blockDim.x - 1) a.out[y][n] = a.tmp[y][blockIdx.x] + tot;
}

int exclusive_scan2_i64(const Scan2& a, int64_t n, hipStream_t st) {
  if (n == 0) {
    (void)hipMemsetAsync(a.out[0], 0, sizeof(int64_t), st);
    (void)hipMemsetAsync(a.out[1], 0, sizeof(int64_t), st);
    return check_launch("scan2(empty)");
  }
  const int64_t nt = ceil_div(n, kScanTile);
  scan2_tile_sums<<<dim3((unsigned)nt, 2), kScanThreads, 0, st>>>(a, n);
  scan2_sums_single<<<2, kScanThreads, 0, st>>>(a, nt);
  scan2_tile_apply<<<dim3((unsigned)nt, 2), kScanThreads, 0, st>>>(a, n);
  return check_launch("exclusive_scan2_i64");
}


// Stable placement of one graph's edges into the CSR keyed by `key_local` (dst for the
// in-CSR, src for the out-CSR).  cursor[] holds each row's next free local slot.
// For the in-CSR pass (IN = true) it records every edge's in-slot in inslot_ws; the out
// pass reads it back to fill out_inslot.
template <bool IN>
__device__ void place_edges(int ne, int64_t eoff, int64_t noff, const int32_t* __restrict__ key_local,
                            const int32_t* __restrict__ val_local, int* cursor, int* chunk_key,
                            int32_t* __restrict__ out_val, int32_t* __restrict__ out_aux,
                            int32_t* __restrict__ inslot_ws, int n) {
  for (int base = 0; base < ne; base += kCsrThreads) {
    const int i = base + threadIdx.x;
    int k = -1, v = 0;
    if (i < ne) {
      k = key_local[eoff + i];
      v = val_local[eoff + i];
      if (k < 0 || k >= n || v < 0 || v >= n) k = -1;  // invalid edges are skipped (flagged)
    }
    chunk_key[threadIdx.x] = k;
    __syncthreads();
    int rank = 0;
    bool last = true;
    if (k >= 0) {
      for (int j = 0; j < (int)threadIdx.x; ++j) rank += (chunk_key[j] == k);
      const int lim = min(kCsrThreads, ne - base);
      for (int j = threadIdx.x + 1; j < lim; ++j)
        if (chunk_key[j] == k) { last = false; break; }
    }
    int slot = 0;
    if (k >= 0) slot = cursor[k] + rank;
    __syncthreads();
    if (k >= 0) {
      if (last) cursor[k] = slot + 1;
      const int64_t g = eoff + slot;
      out_val[g] = v + (int32_t)noff;
      if (IN) {
        out_aux[g] = (int32_t)(eoff + i);     // in_eid
        inslot_ws[eoff + i] = (int32_t)g;     // in-slot of edge eoff+i
      } else {
        out_aux[g] = inslot_ws[eoff + i];     // out_inslot
      }
    }
    __syncthreads();
  }
}

// Block-wide exclusive scan of cnt[0..n) in place; writes rowptr[noff + j] = eoff + excl[j].
__device__ void rows_from_counts(int* cnt, int n, int64_t noff, int64_t eoff,
                                 int32_t* __restrict__ rowptr, int* zero_rows) {
  __shared__ int w[kCsrThreads / 64 + 1];
  int carry = 0, zeros = 0;
  for (int b = 0; b < n; b += kCsrThreads) {
    const int j = b + threadIdx.x;
    const int c = j < n ? cnt[j] : 0;
    if (j < n && c == 0) ++zeros;
    int tot;
    const int ex = block_exclusive_scan<int>(c, w, &tot);
    if (j < n) {
      cnt[j] = carry + ex;
      rowptr[noff + j] = (int32_t)(eoff + carry + ex);
    }
    carry += tot;
  }
  if (zero_rows && zeros) atomicAdd(zero_rows, zeros);
}

// One WAVE per molecule: the wave's degree histograms and the in-slot of every edge live in its
// own LDS slice, the row starts come from a wave scan, and the stable placement walks the edges
// 64 at a time in edge order — a lane's rank among the chunk's equal keys is the number of
// earlier lanes holding its key, found by matching the key bit by bit over ballots (log2(n)
// steps, no loop over lanes), its slot the row's cursor plus that rank, and the cursors then
// advance by LDS adds (order-independent).  No block barriers.  Two sizes:
//  * build_csr_wave_kernel: four molecules per 256-thread workgroup, <= kWaveMolAtoms atoms and
//    <= kWaveMolEdges edges (every KEGG-like molecule); larger ones go to a list;
//  * build_csr_bigwave_kernel: one molecule per 64-thread workgroup, <= kBigMolAtoms atoms and
//    <= kBigMolEdges edges (config 5's 150-400-atom hub molecules), walking that list; the rest
//    to a second list for build_csr_kernel (one workgroup per graph, any size).
// A stable counting sort has one result, so every path gives the same output.
__device__ __forceinline__ void wave_lds_sync_b() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// exclusive wave scan of cnt[0..n) in place (+ the row starts), returns the zero-count rows
__device__ __forceinline__ int wave_rows_from_counts(int* cnt, int n, int64_t noff, int64_t eoff,
                                                     int32_t* __restrict__ rowptr) {
  const int lane = threadIdx.x & 63;
  int carry = 0, zeros = 0;
  for (int b = 0; b < n; b += 64) {
    const int j = b + lane;
    const int c = j < n ? cnt[j] : 0;
    zeros += (j < n && c == 0) ? 1 : 0;
    int x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (j < n) {
      cnt[j] = carry + x - c;
      rowptr[noff + j] = (int32_t)(eoff + carry + x - c);
    }
    carry += __shfl(x, 63, 64);
  }
  return zeros;
}

// stable placement of the molecule's edges keyed by key_local (dst: in-CSR, src: out-CSR)
template <bool IN>
__device__ __forceinline__ void wave_place_edges(int ne, int n, int64_t eoff, int64_t noff,
                                                 const int32_t* __restrict__ key_local,
                                                 const int32_t* __restrict__ val_local, int* cursor,
                                                 int* s_inslot, int32_t* __restrict__ out_val,
                                                 int32_t* __restrict__ out_aux) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));  // lanes < this one
  int nbits = 0;
  while ((1 << nbits) < n) ++nbits;  // keys are in [0, n)
  // the next chunk's keys are loaded before this chunk is placed (one load latency per chunk
  // hidden: the big molecules walk ~27 chunks per pass)
  auto load = [&](int base, int& k, int& v) {
    const int i = base + lane;
    k = -1;
    v = 0;
    if (i < ne) {
      k = key_local[eoff + i];
      v = val_local[eoff + i];
      if (k < 0 || k >= n || v < 0 || v >= n) k = -1;  // invalid edges are skipped (flagged)
    }
  };
  int kn, vn;
  load(0, kn, vn);
  for (int base = 0; base < ne; base += 64) {
    const int i = base + lane;
    const int k = kn, v = vn;
    if (base + 64 < ne) load(base + 64, kn, vn);
    // lanes holding this lane's key: intersect, bit by bit, the ballots that agree with it
    uint64_t same = __ballot(k >= 0);
    for (int b = 0; b < nbits; ++b) {
      const bool bit = ((k >> b) & 1) != 0;
      const uint64_t on = __ballot(bit);
      same &= bit ? on : ~on;
    }
    const int rank = __popcll(same & below);
    const int slot = k >= 0 ? cursor[k] + rank : 0;
    wave_lds_sync_b();  // every lane read its cursor before any advances
    if (k >= 0) {
      atomicAdd(&cursor[k], 1);
      const int64_t gs = eoff + slot;
      out_val[gs] = v + (int32_t)noff;
      if (IN) {
        out_aux[gs] = (int32_t)(eoff + i);  // in_eid
        s_inslot[i] = (int32_t)gs;          // in-slot of edge eoff + i
      } else {
        out_aux[gs] = s_inslot[i];          // out_inslot
      }
    }
    wave_lds_sync_b();
  }
}

// The same placement from registers: the wave kernel's molecules have <= kWaveMolEdges edges,
// so the lane's <= NCH (src, dst) pairs loaded once for the counts are kept and both passes
// place them without reloading (two dependent global round trips fewer per molecule).
template <bool IN, int NCH>
__device__ __forceinline__ void wave_place_edges_reg(int ne, int n, int64_t eoff, int64_t noff,
                                                     const int (&sv)[NCH], const int (&dv)[NCH], int* cursor,
                                                     int* s_inslot, int32_t* __restrict__ out_val,
                                                     int32_t* __restrict__ out_aux) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int nbits = 0;
  while ((1 << nbits) < n) ++nbits;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int base = 64 * c;
    if (base >= ne) break;
    const int i = base + lane;
    int k = IN ? dv[c] : sv[c];
    const int v = IN ? sv[c] : dv[c];
    if (i >= ne || k < 0 || k >= n || v < 0 || v >= n) k = -1;
    uint64_t same = __ballot(k >= 0);
    for (int b = 0; b < nbits; ++b) {
      const bool bit = ((k >> b) & 1) != 0;
      const uint64_t on = __ballot(bit);
      same &= bit ? on : ~on;
    }
    const int rank = __popcll(same & below);
    const int slot = k >= 0 ? cursor[k] + rank : 0;
    wave_lds_sync_b();
    if (k >= 0) {
      atomicAdd(&cursor[k], 1);
      const int64_t gs = eoff + slot;
      out_val[gs] = v + (int32_t)noff;
      if (IN) {
        out_aux[gs] = (int32_t)(eoff + i);
        s_inslot[i] = (int32_t)gs;
      } else {
        out_aux[gs] = s_inslot[i];
      }
    }
    wave_lds_sync_b();
  }
}

struct CsrArgs {
  const int32_t* src_local;
  const int32_t* dst_local;
  const int64_t* num_nodes;
  const int64_t* num_edges;
  const int64_t* node_off;
  const int64_t* edge_off;
  int32_t* src;
  int32_t* dst;
  int32_t* node_graph;
  int32_t* in_rowptr;
  int32_t* in_src;
  int32_t* in_eid;
  int32_t* out_rowptr;
  int32_t* out_dst;
  int32_t* out_inslot;
  int32_t* flags;
};

// the whole CSR build of molecule g by the calling wave (LDS slices cin / cout [n], slot [ne]);
// NCH > 0 (ne <= 64 NCH): the edges stay in registers between the count and the two placements
template <int NCH = 0>
__device__ __forceinline__ void wave_build_molecule(const CsrArgs& a, int64_t g, int n, int ne, int64_t noff,
                                                    int64_t eoff, int* cin, int* cout, int* slot) {
  const int lane = threadIdx.x & 63;
  constexpr int NR = NCH > 0 ? NCH : 1;
  int sv[NR], dv[NR];
  if constexpr (NCH > 0) {  // issue every edge load first
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int i = 64 * c + lane;
      sv[c] = i < ne ? a.src_local[eoff + i] : -1;
      dv[c] = i < ne ? a.dst_local[eoff + i] : -1;
    }
  }
  for (int j = lane; j < n; j += 64) {
    cin[j] = 0;
    cout[j] = 0;
    a.node_graph[noff + j] = (int32_t)g;
  }
  wave_lds_sync_b();
  int bad = 0;
  auto count_edge = [&](int i, int s, int d) {
    a.src[eoff + i] = s + (int32_t)noff;
    a.dst[eoff + i] = d + (int32_t)noff;
    if (s < 0 || s >= n || d < 0 || d >= n) {
      ++bad;
      return;
    }
    atomicAdd(&cin[d], 1);
    atomicAdd(&cout[s], 1);
  };
  if constexpr (NCH > 0) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      if (64 * c + lane < ne) count_edge(64 * c + lane, sv[c], dv[c]);
  } else {
#pragma unroll 4
    for (int i = lane; i < ne; i += 64) count_edge(i, a.src_local[eoff + i], a.dst_local[eoff + i]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o, 64);
  if (lane == 0 && bad) atomicAdd(&a.flags[1], bad);
  wave_lds_sync_b();
  int zeros = wave_rows_from_counts(cin, n, noff, eoff, a.in_rowptr);
  wave_rows_from_counts(cout, n, noff, eoff, a.out_rowptr);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) zeros += __shfl_xor(zeros, o, 64);
  if (lane == 0) {
    if (zeros) atomicAdd(&a.flags[0], zeros);
    a.in_rowptr[noff + n] = (int32_t)(eoff + ne);  // == the next molecule's first row start
    a.out_rowptr[noff + n] = (int32_t)(eoff + ne);
  }
  wave_lds_sync_b();
  if constexpr (NCH > 0) {
    wave_place_edges_reg<true>(ne, n, eoff, noff, sv, dv, cin, slot, a.in_src, a.in_eid);
    wave_place_edges_reg<false>(ne, n, eoff, noff, sv, dv, cout, slot, a.out_dst, a.out_inslot);
  } else {
    wave_place_edges<true>(ne, n, eoff, noff, a.dst_local, a.src_local, cin, slot, a.in_src, a.in_eid);
    wave_place_edges<false>(ne, n, eoff, noff, a.src_local, a.dst_local, cout, slot, a.out_dst, a.out_inslot);
  }
}

__global__ void __launch_bounds__(256)
build_csr_wave_kernel(CsrArgs a, int64_t B, int32_t* __restrict__ big_list, int* __restrict__ big_count) {
  __shared__ int s_cin[4][kWaveMolAtoms];
  __shared__ int s_cout[4][kWaveMolAtoms];
  __shared__ int s_slot[4][kWaveMolEdges];
  const int w = threadIdx.x >> 6;
  const int64_t g = (int64_t)blockIdx.x * 4 + w;
  if (g >= B) return;  // (wave-level only: no block barriers below)
  // sizes and offsets in one round trip (the offsets are the scan's, already written)
  const int n = (int)a.num_nodes[g];
  const int ne = (int)a.num_edges[g];
  const int64_t noff = a.node_off[g], eoff = a.edge_off[g];
  if (n > kWaveMolAtoms || ne > kWaveMolEdges) {  // the next size class
    if ((threadIdx.x & 63) == 0) big_list[atomicAdd(big_count, 1)] = (int32_t)g;
    return;
  }
  wave_build_molecule<kWaveMolEdges / 64>(a, g, n, ne, noff, eoff, s_cin[w], s_cout[w], s_slot[w]);
}

// persistent over the first list; one wave per workgroup (24 KB of LDS)
__global__ void __launch_bounds__(64)
build_csr_bigwave_kernel(CsrArgs a, const int32_t* __restrict__ list, const int* __restrict__ count,
                         int32_t* __restrict__ huge_list, int* __restrict__ huge_count) {
  __shared__ int s_cin[kBigMolAtoms];
  __shared__ int s_cout[kBigMolAtoms];
  __shared__ int s_slot[kBigMolEdges];
  const int cnt = *count;
  for (int li = blockIdx.x; li < cnt; li += gridDim.x) {
    const int64_t g = list[li];
    const int n = (int)a.num_nodes[g];
    const int ne = (int)a.num_edges[g];
    if (n > kBigMolAtoms || ne > kBigMolEdges) {
      if (threadIdx.x == 0) huge_list[atomicAdd(huge_count, 1)] = (int32_t)g;
      continue;
    }
    wave_build_molecule(a, g, n, ne, a.node_off[g], a.edge_off[g], s_cin, s_cout, s_slot);
    wave_lds_sync_b();  // this molecule's LDS reads are done before the next one's zeroing
  }
}

__global__ void __launch_bounds__(kCsrThreads)
build_csr_kernel(const int32_t* __restrict__ src_local, const int32_t* __restrict__ dst_local,
                 const int64_t* __restrict__ num_nodes, const int64_t* __restrict__ num_edges,
                 const int64_t* __restrict__ node_off, const int64_t* __restrict__ edge_off,
                 int64_t N, int64_t E, int32_t* __restrict__ src, int32_t* __restrict__ dst,
                 int32_t* __restrict__ node_graph, int32_t* __restrict__ in_rowptr,
                 int32_t* __restrict__ in_src, int32_t* __restrict__ in_eid,
                 int32_t* __restrict__ out_rowptr, int32_t* __restrict__ out_dst,
                 int32_t* __restrict__ out_inslot, int32_t* __restrict__ flags,
                 int32_t* __restrict__ inslot_ws, int* __restrict__ big_cnt,
                 const int32_t* __restrict__ list, const int* __restrict__ count) {
  __shared__ int cnt_in_l[kLdsNodes];
  __shared__ int cnt_out_l[kLdsNodes];
  __shared__ int chunk_key[kCsrThreads];
  const int lcount = *count;
  for (int li = blockIdx.x; li < lcount; li += gridDim.x) {
  __syncthreads();  // the previous graph's LDS use is done
  const int64_t g = list[li];
  const int n = (int)num_nodes[g];
  const int ne = (int)num_edges[g];
  const int64_t noff = node_off[g], eoff = edge_off[g];
  int* cnt_in = cnt_in_l;
  int* cnt_out = cnt_out_l;
  if (n > kLdsNodes) {  // large graph: histogram in the workspace slice of this graph
    cnt_in = big_cnt + 2 * noff;
    cnt_out = cnt_in + n;
  }
  for (int j = threadIdx.x; j < n; j += kCsrThreads) {
    cnt_in[j] = 0;
    cnt_out[j] = 0;
    node_graph[noff + j] = (int32_t)g;
  }
  __syncthreads();
  int bad = 0;
  for (int i = threadIdx.x; i < ne; i += kCsrThreads) {
    const int s = src_local[eoff + i], d = dst_local[eoff + i];
    src[eoff + i] = s + (int32_t)noff;
    dst[eoff + i] = d + (int32_t)noff;
    if (s < 0 || s >= n || d < 0 || d >= n) {
      ++bad;
      continue;
    }
    atomicAdd(&cnt_in[d], 1);
    atomicAdd(&cnt_out[s], 1);
  }
  if (bad) atomicAdd(&flags[1], bad);
  __syncthreads();
  rows_from_counts(cnt_in, n, noff, eoff, in_rowptr, &flags[0]);
  __syncthreads();
  rows_from_counts(cnt_out, n, noff, eoff, out_rowptr, nullptr);
  if (threadIdx.x == 0) {  // row end of this graph == next graph's first row start
    in_rowptr[noff + n] = (int32_t)(eoff + ne);
    out_rowptr[noff + n] = (int32_t)(eoff + ne);
  }
  __syncthreads();
  place_edges<true>(ne, eoff, noff, dst_local, src_local, cnt_in, chunk_key, in_src, in_eid,
                    inslot_ws, n);
  // inslot_ws written above by this workgroup; __syncthreads in place_edges orders it.
  place_edges<false>(ne, eoff, noff, src_local, dst_local, cnt_out, chunk_key, out_dst,
                     out_inslot, inslot_ws, n);
  }
}

// Node groups: group g starts at the first atom of the molecule that contains atom
// g * kNodeGroupAtoms, so every group is a range of whole molecules (possibly empty when a
// molecule spans several multiples).  group_start[G] = N.  One thread per MOLECULE writes the
// starts of the groups whose first multiple it contains (every multiple of kNodeGroupAtoms
// below N lies in exactly one molecule, so each start is written once) — no per-group binary
// search over node_offsets (16 dependent loads per group: ~30 us per 65,536-molecule batch).
__global__ void node_group_start_kernel(int64_t B, int64_t N, const int64_t* __restrict__ node_offsets,
                                        int64_t G, int32_t* __restrict__ plan) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m == 0) plan[G] = (int32_t)N;
  if (m >= B) return;
  const int64_t a = node_offsets[m], b = m + 1 < B ? node_offsets[m + 1] : N;
  for (int64_t g = (a + kNodeGroupAtoms - 1) / kNodeGroupAtoms; g * kNodeGroupAtoms < b; ++g)
    plan[g] = (int32_t)a;
}

// Group kinds, one wave per group.  Kind bits: bit 0 = the forward LDS kernel takes the group
// (<= kPlanWinAtoms atoms, <= kPlanEdgeCap in-edges, in-degree <= kPlanDegCap everywhere),
// bit 1 = the backward LDS kernel does (atom and edge caps only), bit 2 = the group fits the big
// LDS window (<= kPlanBigAtoms atoms, <= kPlanBigEdgeCap in-edges, any in-degree): groups on a
// fallback list with bit 2 are taken by the big-window kernels.  Non-empty groups without a bit
// are appended to that direction's fallback list.
__global__ void node_group_kind_kernel(int64_t G, const int32_t* __restrict__ rowptr,
                                       int32_t* __restrict__ plan) {
  const int64_t g = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (g >= G) return;
  int32_t* kind = plan + G + 1;
  const int a0 = plan[g], a1 = plan[g + 1];
  int dmax = 0;
  for (int v = a0 + lane; v < a1; v += 64) dmax = max(dmax, rowptr[v + 1] - rowptr[v]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) dmax = max(dmax, __shfl_xor(dmax, o, 64));
  if (lane != 0) return;
  int k = 0;
  if (a1 > a0) {
    const bool fits = a1 - a0 <= kPlanWinAtoms && rowptr[a1] - rowptr[a0] <= kPlanEdgeCap;
    const bool big = a1 - a0 <= kPlanBigAtoms && rowptr[a1] - rowptr[a0] <= kPlanBigEdgeCap;
    k = (fits && dmax <= kPlanDegCap ? 1 : 0) | (fits ? 2 : 0) | (big ? 4 : 0);
  }
  kind[g] = k;
}

// The fallback lists in group order, one workgroup: thread t owns the contiguous groups
// [t R, (t + 1) R), R = ceil(G / 1024).  Its starts and kinds are read 8 groups per round with
// every load independent (a loop with the kind load behind the emptiness test paid two load
// latencies per group: ~30 us per 65,536-molecule batch), the flags kept as bit masks (R <= 64;
// larger plans re-read them in a second pass), the counts exclusive-scanned across the
// workgroup (shuffles within a wave, the 16 wave totals through LDS) and the entries written
// in group order.
constexpr int kListUnroll = 8;
__device__ __forceinline__ void group_flag_masks(const int32_t* __restrict__ start, const int32_t* __restrict__ kind,
                                                 int64_t G, int64_t g0, int64_t g1, uint64_t& m0, uint64_t& m1,
                                                 int& c0, int& c1) {
  m0 = m1 = 0;
  c0 = c1 = 0;
  for (int64_t base = g0; base < g1; base += kListUnroll) {
    int32_t sv[kListUnroll + 1], kv[kListUnroll];
#pragma unroll
    for (int u = 0; u <= kListUnroll; ++u) sv[u] = start[min(base + u, G)];
#pragma unroll
    for (int u = 0; u < kListUnroll; ++u) kv[u] = kind[min(base + u, G - 1)];
#pragma unroll
    for (int u = 0; u < kListUnroll; ++u) {
      const bool live = base + u < g1 && sv[u + 1] > sv[u];
      const bool f0 = live && (kv[u] & 1) == 0, f1 = live && (kv[u] & 2) == 0;
      c0 += f0;
      c1 += f1;
      const int sh = (int)(base + u - g0);
      if (sh < 64) {
        m0 |= (uint64_t)f0 << sh;
        m1 |= (uint64_t)f1 << sh;
      }
    }
  }
}
__global__ void __launch_bounds__(1024) node_group_lists_kernel(int64_t G, int32_t* __restrict__ plan) {
  const int32_t* start = plan;
  const int32_t* kind = plan + G + 1;
  int32_t* count = plan + 2 * G + 1;
  __shared__ int s_w[2][16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t R = (G + 1023) / 1024, g0 = min(G, tid * R), g1 = min(G, g0 + R);
  uint64_t m0, m1;
  int c0, c1;
  group_flag_masks(start, kind, G, g0, g1, m0, m1, c0, c1);
  int i0 = c0, i1 = c1;  // inclusive wave scans
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u0 = __shfl_up(i0, o, 64), u1 = __shfl_up(i1, o, 64);
    if (lane >= o) {
      i0 += u0;
      i1 += u1;
    }
  }
  if (lane == 63) {
    s_w[0][w] = i0;
    s_w[1][w] = i1;
  }
  __syncthreads();
  int o0 = i0 - c0, o1 = i1 - c1, t0 = 0, t1 = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    o0 += k < w ? s_w[0][k] : 0;
    o1 += k < w ? s_w[1][k] : 0;
    t0 += s_w[0][k];
    t1 += s_w[1][k];
  }
  for (int64_t cb = g0; cb < g1 && (c0 | c1); cb += 64) {  // 64 groups per mask
    if (cb > g0) {  // (R > 64 only) the next 64 groups' flags again
      int d0, d1;
      group_flag_masks(start, kind, G, cb, min(g1, cb + 64), m0, m1, d0, d1);
    }
    for (uint64_t m = m0; m; m &= m - 1) plan[2 * G + 3 + o0++] = (int32_t)(cb + __builtin_ctzll(m));
    for (uint64_t m = m1; m; m &= m - 1) plan[3 * G + 3 + o1++] = (int32_t)(cb + __builtin_ctzll(m));
  }
  if (tid == 0) {
    count[0] = t0;
    count[1] = t1;
  }
}

}  // namespace
}  // namespace mvml

using namespace mvml;

extern "C" size_t mvml_build_csr_workspace_size(int64_t num_graphs, int64_t num_nodes,
                                                int64_t num_edges) {
  size_t nt = (size_t)ceil_div(num_graphs > 0 ? num_graphs : 1, kScanTile);
  return 2 * carve_size(nt * sizeof(int64_t)) + carve_size((size_t)num_edges * sizeof(int32_t)) +
         carve_size((size_t)2 * num_nodes * sizeof(int)) +
         2 * carve_size((size_t)(num_graphs > 0 ? num_graphs : 1) * sizeof(int32_t)) +
         carve_size(2 * sizeof(int)) + 256;
}

extern "C" int mvml_build_csr(const int32_t* src_local, const int32_t* dst_local,
                              const int64_t* batch_num_nodes, const int64_t* batch_num_edges,
                              int64_t num_graphs, int64_t num_nodes, int64_t num_edges,
                              int64_t* node_offsets, int64_t* edge_offsets, int32_t* src,
                              int32_t* dst, int32_t* node_graph, int32_t* in_rowptr,
                              int32_t* in_src, int32_t* in_eid, int32_t* out_rowptr,
                              int32_t* out_dst, int32_t* out_inslot, int32_t* status_flags,
                              void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  MVML_REQUIRE(num_graphs >= 0 && num_nodes >= 0 && num_edges >= 0, "build_csr: negative size");
  MVML_REQUIRE(num_nodes < (int64_t(1) << 31) && num_edges < (int64_t(1) << 31),
               "build_csr: int32 index overflow (N=%lld, E=%lld)", (long long)num_nodes,
               (long long)num_edges);
  MVML_REQUIRE(num_graphs < (int64_t(1) << 31), "build_csr: too many graphs");
  if (workspace_bytes < mvml_build_csr_workspace_size(num_graphs, num_nodes, num_edges)) {
    set_error("build_csr: workspace too small");
    return MVML_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  Carver cv(workspace, workspace_bytes);
  int64_t* tmp = cv.take<int64_t>((size_t)ceil_div(num_graphs > 0 ? num_graphs : 1, kScanTile));
  int64_t* tmp2 = cv.take<int64_t>((size_t)ceil_div(num_graphs > 0 ? num_graphs : 1, kScanTile));
  int32_t* inslot = cv.take<int32_t>((size_t)num_edges);
  int* big = cv.take<int>((size_t)2 * num_nodes);
  int32_t* list1 = cv.take<int32_t>((size_t)(num_graphs > 0 ? num_graphs : 1));
  int32_t* list2 = cv.take<int32_t>((size_t)(num_graphs > 0 ? num_graphs : 1));
  int* counts = cv.take<int>(2);
  if (num_graphs == 0) (void)hipMemsetAsync(status_flags, 0, 2 * sizeof(int32_t), st);
  const Scan2 sc{{batch_num_nodes, batch_num_edges}, {node_offsets, edge_offsets}, {tmp, tmp2},
                 {status_flags, reinterpret_cast<int32_t*>(counts)}};
  int rc = exclusive_scan2_i64(sc, num_graphs, st);
  if (rc) return rc;
  if (num_nodes == 0) {
    (void)hipMemsetAsync(in_rowptr, 0, sizeof(int32_t), st);
    (void)hipMemsetAsync(out_rowptr, 0, sizeof(int32_t), st);
    return check_launch("build_csr(empty)");
  }
  if (num_graphs > 0) {
    const CsrArgs a{src_local, dst_local, batch_num_nodes, batch_num_edges, node_offsets, edge_offsets,
                    src, dst, node_graph, in_rowptr, in_src, in_eid, out_rowptr, out_dst,
                    out_inslot, status_flags};
    build_csr_wave_kernel<<<(unsigned)ceil_div(num_graphs, 4), 256, 0, st>>>(a, num_graphs, list1, counts);
    int rc2 = check_launch("build_csr_wave_kernel");
    if (rc2) return rc2;
    // the molecules past the wave kernel's sizes (a device-side list: persistent grids)
    build_csr_bigwave_kernel<<<(unsigned)std::min<int64_t>(num_graphs, 2048), 64, 0, st>>>(a, list1, counts,
                                                                                         list2, counts + 1);
    rc2 = check_launch("build_csr_bigwave_kernel");
    if (rc2) return rc2;
    build_csr_kernel<<<(unsigned)std::min<int64_t>(num_graphs, 512), kCsrThreads, 0, st>>>(
        src_local, dst_local, batch_num_nodes, batch_num_edges, node_offsets, edge_offsets,
        num_nodes, num_edges, src, dst, node_graph, in_rowptr, in_src, in_eid, out_rowptr,
        out_dst, out_inslot, status_flags, inslot, big, list2, counts + 1);
  }
  return check_launch("build_csr_kernel");
}

extern "C" int64_t mvml_node_group_count(int64_t num_nodes) {
  return num_nodes > 0 ? ceil_div(num_nodes, kNodeGroupAtoms) : 0;
}

extern "C" int64_t mvml_node_group_plan_size(int64_t num_nodes) {
  const int64_t G = mvml_node_group_count(num_nodes);
  return G > 0 ? 4 * G + 3 : 1;
}

extern "C" int mvml_build_node_groups(int64_t num_graphs, int64_t num_nodes,
                                      const int64_t* node_offsets, const int32_t* in_rowptr,
                                      int32_t* plan, void* stream) {
  clear_error();
  MVML_REQUIRE(num_graphs >= 0 && num_nodes >= 0 && num_nodes < (int64_t(1) << 31),
               "build_node_groups: bad sizes");
  const int64_t G = mvml_node_group_count(num_nodes);
  if (G == 0) return MVML_OK;
  MVML_REQUIRE(num_graphs > 0 && node_offsets && in_rowptr && plan, "build_node_groups: null input");
  hipStream_t st = as_stream(stream);
  node_group_start_kernel<<<(unsigned)ceil_div(num_graphs, 256), 256, 0, st>>>(num_graphs, num_nodes,
                                                                              node_offsets, G, plan);
  int rc = check_launch("node_group_start_kernel");
  if (rc) return rc;
  // fallback counts and lists: node_group_lists_kernel
  node_group_kind_kernel<<<(unsigned)ceil_div(G, 4), 256, 0, st>>>(G, in_rowptr, plan);
  rc = check_launch("node_group_kind_kernel");
  if (rc) return rc;
  node_group_lists_kernel<<<1, 1024, 0, st>>>(G, plan);
  return check_launch("node_group_lists_kernel");
}
