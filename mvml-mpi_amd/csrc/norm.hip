// GraphNorm (torch_geometric 2.2.0, model.py:85 and 93) forward/backward with per-group
// statistics, the ReLU backward of GNNModule.fc (model.py:86-87) and the Dropout that follows
// it (and the fusion head's two, model.py:36, 46), and a narrow column-slice copy.
//
// Reference semantics with batch=None: the normalisation group is the whole mini-batch passed
// to GNNModule.forward (64 molecules, config.py:21).  Groups are rows [off[g], off[g+1]).
//   mean = sum(x)/n;  o = x - mean*mean_scale;  var = sum(o^2)/n;  std = sqrt(var + eps)
//   y = weight*o/std + bias
// One thread per (group, column): column reads of a 768-wide row are coalesced across the
// workgroup.  Parameter gradients are reduced over groups in fixed order (no atomics).
// Statistics and per-element arithmetic run in fp64 (inputs/outputs fp32): GraphNorm over a
// small group is ill-conditioned (x - mean cancels), the layer is tiny ((B, 768) per step, no
// measurable cost), and fp64 keeps its own rounding out of the gradients it sends upstream.
#include <type_traits>

#include "common.h"
#include "dropout.h"

namespace mvml {
namespace {

__global__ void graphnorm_fwd_kernel(int D, const int64_t* __restrict__ off, const float* __restrict__ x,
                                     const float* __restrict__ w, const float* __restrict__ b,
                                     const float* __restrict__ ms, float eps, float* __restrict__ y) {
  const int col = blockIdx.y * blockDim.x + threadIdx.x;
  if (col >= D) return;
  const int64_t g = blockIdx.x;
  const int64_t r0 = off[g], r1 = off[g + 1];
  if (r1 <= r0) return;
  const double n = (double)(r1 - r0);
  double s = 0.0;
  for (int64_t r = r0; r < r1; ++r) s += x[r * D + col];
  const double mean = s / n;
  const double msc = ms[col];
  double v = 0.0;
  for (int64_t r = r0; r < r1; ++r) {
    const double o = x[r * D + col] - mean * msc;
    v += o * o;
  }
  const double k = (double)w[col] / sqrt(v / n + (double)eps);
  const double bc = b[col];
  for (int64_t r = r0; r < r1; ++r) {
    const double o = x[r * D + col] - mean * msc;
    y[r * D + col] = (float)(k * o + bc);
  }
}

// Per (group, column): g_x and the group's partial parameter gradients.
__global__ void graphnorm_bwd_kernel(int D, const int64_t* __restrict__ off, const float* __restrict__ x,
                                     const float* __restrict__ w, const float* __restrict__ ms, float eps,
                                     const float* __restrict__ gy, float* __restrict__ gx,
                                     double* __restrict__ part /* [3][G][D] */, int64_t G) {
  const int col = blockIdx.y * blockDim.x + threadIdx.x;
  if (col >= D) return;
  const int64_t g = blockIdx.x;
  const int64_t r0 = off[g], r1 = off[g + 1];
  double pw = 0.0, pb = 0.0, pms = 0.0;
  if (r1 > r0) {
    const double n = (double)(r1 - r0);
    double s = 0.0;
    for (int64_t r = r0; r < r1; ++r) s += x[r * D + col];
    const double mean = s / n;
    const double msc = ms[col], wc = w[col];
    double v = 0.0, so = 0.0, sgy = 0.0, sgyo = 0.0;
    for (int64_t r = r0; r < r1; ++r) {
      const double o = x[r * D + col] - mean * msc;
      const double gyr = gy[r * D + col];
      v += o * o;
      so += o;
      sgy += gyr;
      sgyo += gyr * o;
    }
    const double var = v / n + (double)eps;
    const double inv = 1.0 / sqrt(var);
    // g_o_j = w/std * (g_y_j - S1 * o_j / (n std^2)),  S1 = sum g_y o
    const double k1 = wc * inv;
    const double k2 = sgyo / (n * var);
    const double sum_go = k1 * (sgy - k2 * so);
    for (int64_t r = r0; r < r1; ++r) {
      const double o = x[r * D + col] - mean * msc;
      const double go = k1 * (gy[r * D + col] - k2 * o);
      gx[r * D + col] = (float)(go - msc * sum_go / n);
    }
    pw = sgyo * inv;
    pb = sgy;
    pms = -mean * sum_go;
  }
  part[(0 * G + g) * D + col] = pw;
  part[(1 * G + g) * D + col] = pb;
  part[(2 * G + g) * D + col] = pms;
}

// Sum of the G group partials of one parameter gradient: a workgroup per 16 columns, 16 group
// stripes per column (g = stripe, stripe + 16, ...; four independent accumulators so the loads
// stay in flight), then a fixed-order tree over the stripes in LDS — deterministic.  (One thread
// per column walking all G groups took 0.36 ms for G = 1024, D = 768: latency, not bytes.)
__global__ void __launch_bounds__(256) graphnorm_param_reduce(int D, int64_t G, const double* __restrict__ part,
                                                              float* __restrict__ gw, float* __restrict__ gb,
                                                              float* __restrict__ gms) {
  const int c = threadIdx.x & 15, stripe = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + c;
  const int which = blockIdx.y;
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  if (col < D) {
    const double* p = part + (int64_t)which * G * D + col;
    int64_t g = stripe;
    for (; g + 48 < G; g += 64) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += p[(g + 16 * u) * D];
    }
    for (; g < G; g += 16) a[0] += p[g * D];
  }
  __shared__ double red[16][17];
  red[stripe][c] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  for (int h = 8; h > 0; h >>= 1) {
    if (stripe < h) red[stripe][c] += red[stripe + h][c];
    __syncthreads();
  }
  if (stripe == 0 && col < D) {
    float* dst = which == 0 ? gw : (which == 1 ? gb : gms);
    if (dst) dst[col] = (float)red[0][c];
  }
}

__global__ void relu_bwd_kernel(int64_t n, const float* __restrict__ y, const float* __restrict__ gy,
                                float* __restrict__ gx, float scale) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    gx[i] = y[i] > 0.f ? (scale == 1.f ? gy[i] : gy[i] * scale) : 0.f;
}

// y = x * keep * scale (x == y allowed), four elements per thread (16-B accesses when x, y and
// n are 4-aligned; the scalar tail otherwise)
__global__ void dropout_fwd_kernel(int64_t n, const float* x, float* y, uint32_t thr, float scale,
                                   uint64_t seed, bool vec) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; 4 * q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t a = dropout_pair_bits(seed, 2 * q), b = dropout_pair_bits(seed, 2 * q + 1);
    const uint32_t u[4] = {(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
    const int64_t i0 = 4 * q;
    if (vec && i0 + 4 <= n) {
      float4 v = *reinterpret_cast<const float4*>(x + i0);
      v.x = u[0] >= thr ? v.x * scale : 0.f;
      v.y = u[1] >= thr ? v.y * scale : 0.f;
      v.z = u[2] >= thr ? v.z * scale : 0.f;
      v.w = u[3] >= thr ? v.w * scale : 0.f;
      *reinterpret_cast<float4*>(y + i0) = v;
    } else {
      for (int e = 0; e < 4 && i0 + e < n; ++e) y[i0 + e] = u[e] >= thr ? x[i0 + e] * scale : 0.f;
    }
  }
}

// dst[r][c] = src[r][c] for c < cols: the narrow column slice of a wide row-pitched matrix
// (the 2H logit columns of the projection output) into a dense [rows][cols] array
// (V = 4: 16-B accesses, when cols, both pitches and both pointers are 4-float aligned)
template <int V>
__global__ void copy_cols_kernel(int64_t rows, int cols, const float* __restrict__ src, int64_t lds,
                                 float* __restrict__ dst, int64_t ldd) {
  using vec = typename std::conditional<V == 4, float4, float>::type;
  const int cv = cols / V;
  const int64_t total = rows * cv;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cv;
    const int c = (int)(i - r * cv) * V;
    *reinterpret_cast<vec*>(dst + r * ldd + c) = *reinterpret_cast<const vec*>(src + r * lds + c);
  }
}

// Set2Set's LSTM weights as the gates products read them: wcat [4D][kin + D] = [w_ih | w_hh]
// and (wperm not NULL) the cell epilogue's interleaved rows, wperm row 4 j + q = wcat row q D + j
__global__ void lstm_pack_weights_kernel(int D, int kin, const float* __restrict__ w_ih,
                                         const float* __restrict__ w_hh, float* __restrict__ wcat,
                                         float* __restrict__ wperm) {
  const int K = kin + D;
  const int64_t total = (int64_t)4 * D * K;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / K), c = (int)(i - (int64_t)r * K);
    const float v = c < kin ? w_ih[(int64_t)r * kin + c] : w_hh[(int64_t)r * D + (c - kin)];
    wcat[i] = v;
    if (wperm) {
      const int q = r / D, j = r - q * D;
      wperm[(int64_t)(4 * j + q) * K + c] = v;
    }
  }
}

// dst[c][r] = src[r][c] through a 32 x 33 LDS tile (both sides coalesced)
__global__ void transpose_kernel(int64_t rows, int64_t cols, const float* __restrict__ src, int64_t lds,
                                 float* __restrict__ dst, int64_t ldd) {
  __shared__ float tile[32][33];
  const int64_t r0 = (int64_t)blockIdx.y * 32, c0 = (int64_t)blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 rows per pass
  for (int k = ty; k < 32; k += 8)
    if (r0 + k < rows && c0 + tx < cols) tile[k][tx] = src[(r0 + k) * lds + c0 + tx];
  __syncthreads();
  for (int k = ty; k < 32; k += 8)
    if (c0 + k < cols && r0 + tx < rows) dst[(c0 + k) * ldd + r0 + tx] = tile[tx][k];
}

// y[i] = x[i] * s[0] (a device scalar: the upstream gradient of a scalar loss)
__global__ void scale_by_kernel(int64_t n, const float* __restrict__ x, const float* __restrict__ s,
                                float* __restrict__ y) {
  const float a = s[0];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = x[i] * a;
}

// Zero a pitched block of rows with 16-B vector stores (row_bytes, pitch and base 16-B aligned):
// the runtime's 2-D memset ran at ~0.8 TB/s on Set2Set's [B, D] recurrent-state slices
__global__ void fill_zero_2d_kernel(int64_t rows, int64_t row_vecs, int64_t pitch_vecs, float4* __restrict__ p) {
  const int64_t total = rows * row_vecs;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / row_vecs;
    p[r * pitch_vecs + (i - r * row_vecs)] = z;
  }
}

}  // namespace
}  // namespace mvml

using namespace mvml;

extern "C" int mvml_graphnorm_fwd(int64_t G, int D, const int64_t* group_offsets, const float* x,
                                  const float* weight, const float* bias, const float* mean_scale,
                                  float eps, float* y, void* stream) {
  clear_error();
  MVML_REQUIRE(G >= 0 && D > 0 && G < (int64_t(1) << 31), "graphnorm_fwd: bad shape");
  if (G == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  dim3 grid((unsigned)G, (unsigned)ceil_div(D, 256));
  graphnorm_fwd_kernel<<<grid, 256, 0, st>>>(D, group_offsets, x, weight, bias, mean_scale, eps, y);
  return check_launch("graphnorm_fwd_kernel");
}

extern "C" size_t mvml_graphnorm_bwd_workspace_size(int64_t G, int D) {
  return carve_size((size_t)3 * G * D * sizeof(double));
}

extern "C" int mvml_graphnorm_bwd(int64_t G, int D, const int64_t* group_offsets, const float* x,
                                  const float* weight, const float* mean_scale, float eps,
                                  const float* g_y, float* g_x, float* g_weight, float* g_bias,
                                  float* g_mean_scale, void* workspace, size_t workspace_bytes,
                                  void* stream) {
  clear_error();
  MVML_REQUIRE(G >= 0 && D > 0 && G < (int64_t(1) << 31), "graphnorm_bwd: bad shape");
  if (G == 0) return MVML_OK;
  if (!workspace || workspace_bytes < mvml_graphnorm_bwd_workspace_size(G, D)) {
    set_error("graphnorm_bwd: workspace too small");
    return MVML_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  dim3 grid((unsigned)G, (unsigned)ceil_div(D, 256));
  graphnorm_bwd_kernel<<<grid, 256, 0, st>>>(D, group_offsets, x, weight, mean_scale, eps, g_y, g_x,
                                             part, G);
  int rc = check_launch("graphnorm_bwd_kernel");
  if (rc) return rc;
  dim3 g2((unsigned)ceil_div(D, 16), 3);
  graphnorm_param_reduce<<<g2, 256, 0, st>>>(D, G, part, g_weight, g_bias, g_mean_scale);
  return check_launch("graphnorm_param_reduce");
}

extern "C" int mvml_relu_bwd(int64_t n, const float* y, const float* g_y, float* g_x, float scale,
                             void* stream) {
  clear_error();
  MVML_REQUIRE(n >= 0, "relu_bwd: bad size");
  if (n == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(n, 256), 16384);
  relu_bwd_kernel<<<blocks, 256, 0, st>>>(n, y, g_y, g_x, scale);
  return check_launch("relu_bwd_kernel");
}

extern "C" int mvml_dropout_fwd(int64_t n, const float* x, float* y, double p, int64_t seed, void* stream) {
  clear_error();
  MVML_REQUIRE(n >= 0 && x && y && p >= 0.0 && p < 1.0, "dropout_fwd: bad arguments (0 <= p < 1)");
  if (n == 0) return MVML_OK;
  // keep iff the element's 32-bit draw u >= thr = round(p 2^32): P(keep) = 1 - p to 2^-32
  const uint32_t thr = dropout_threshold(p);
  const float scale = dropout_scale(p);  // 1 / (1 - p) in double, rounded once
  const bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0;
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(ceil_div(n, 4), 256), 8192);
  dropout_fwd_kernel<<<blocks, 256, 0, as_stream(stream)>>>(n, x, y, thr, scale, (uint64_t)seed, vec);
  return check_launch("dropout_fwd_kernel");
}

extern "C" int mvml_copy_cols(int64_t rows, int cols, const float* src, int64_t lds, float* dst, int64_t ldd,
                              void* stream) {
  clear_error();
  MVML_REQUIRE(rows >= 0 && cols > 0 && (lds >= cols || lds == 0) && ldd >= cols && src && dst,
               "copy_cols: bad shape");
  if (rows == 0) return MVML_OK;
  const bool v4 = (cols % 4 == 0) && (lds % 4 == 0) && (ldd % 4 == 0) &&
                  ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(rows * cols / (v4 ? 4 : 1), 256), 16384);
  if (v4)
    copy_cols_kernel<4><<<blocks, 256, 0, as_stream(stream)>>>(rows, cols, src, lds, dst, ldd);
  else
    copy_cols_kernel<1><<<blocks, 256, 0, as_stream(stream)>>>(rows, cols, src, lds, dst, ldd);
  return check_launch("copy_cols_kernel");
}

extern "C" int mvml_fill_zero(void* p, int64_t rows, int64_t row_bytes, int64_t pitch_bytes, void* stream) {
  clear_error();
  MVML_REQUIRE(rows >= 0 && row_bytes >= 0 && pitch_bytes >= row_bytes && (p || rows == 0 || row_bytes == 0),
               "fill_zero: bad shape");
  if (rows == 0 || row_bytes == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  if (pitch_bytes != row_bytes && row_bytes % 16 == 0 && pitch_bytes % 16 == 0 && (uintptr_t)p % 16 == 0) {
    const int64_t total = rows * (row_bytes / 16);
    fill_zero_2d_kernel<<<(unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(total, 256), 8192)), 256, 0, st>>>(
        rows, row_bytes / 16, pitch_bytes / 16, static_cast<float4*>(p));
    return check_launch("fill_zero_2d_kernel");
  }
  const hipError_t e = (pitch_bytes == row_bytes)
                           ? hipMemsetAsync(p, 0, (size_t)(rows * row_bytes), st)
                           : hipMemset2DAsync(p, (size_t)pitch_bytes, 0, (size_t)row_bytes, (size_t)rows, st);
  if (e != hipSuccess) {
    set_error("fill_zero: %s", hipGetErrorString(e));
    return MVML_ERR_LAUNCH;
  }
  return MVML_OK;
}

extern "C" int mvml_lstm_pack_weights(int D, int kin, const float* w_ih, const float* w_hh, float* wcat,
                                      float* wperm, void* stream) {
  clear_error();
  MVML_REQUIRE(D > 0 && kin > 0 && w_ih && w_hh && wcat, "lstm_pack_weights: bad arguments");
  const int64_t total = (int64_t)4 * D * (kin + D);
  lstm_pack_weights_kernel<<<(unsigned)std::min<int64_t>(ceil_div(total, 256), 8192), 256, 0, as_stream(stream)>>>(
      D, kin, w_ih, w_hh, wcat, wperm);
  return check_launch("lstm_pack_weights_kernel");
}

extern "C" int mvml_transpose(int64_t rows, int64_t cols, const float* src, int64_t lds, float* dst, int64_t ldd,
                              void* stream) {
  clear_error();
  MVML_REQUIRE(rows >= 0 && cols >= 0 && lds >= cols && ldd >= rows && ceil_div(rows, 32) < 65536,
               "transpose: bad shape");
  if (rows == 0 || cols == 0) return MVML_OK;
  dim3 grid((unsigned)ceil_div(cols, 32), (unsigned)ceil_div(rows, 32));
  transpose_kernel<<<grid, 256, 0, as_stream(stream)>>>(rows, cols, src, lds, dst, ldd);
  return check_launch("transpose_kernel");
}

extern "C" int mvml_scale_by(int64_t n, const float* x, const float* s, float* y, void* stream) {
  clear_error();
  MVML_REQUIRE(n >= 0 && (n == 0 || (x && s && y)), "scale_by: bad arguments");
  if (n == 0) return MVML_OK;
  scale_by_kernel<<<(unsigned)std::min<int64_t>(ceil_div(n, 256), 8192), 256, 0, as_stream(stream)>>>(n, x, s, y);
  return check_launch("scale_by_kernel");
}
