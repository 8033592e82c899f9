// GraphNorm (torch_geometric 2.2.0, model.py:85 and 93) forward/backward with per-group
// statistics, and the ReLU backward of GNNModule.fc (model.py:86-87).
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
#include "common.h"

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

__global__ void graphnorm_param_reduce(int D, int64_t G, const double* __restrict__ part,
                                       float* __restrict__ gw, float* __restrict__ gb,
                                       float* __restrict__ gms) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  const int which = blockIdx.y;
  if (col >= D) return;
  double s = 0.0;
  for (int64_t g = 0; g < G; ++g) s += part[((int64_t)which * G + g) * D + col];
  float* dst = which == 0 ? gw : (which == 1 ? gb : gms);
  if (dst) dst[col] = (float)s;
}

__global__ void relu_bwd_kernel(int64_t n, const float* __restrict__ y, const float* __restrict__ gy,
                                float* __restrict__ gx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    gx[i] = y[i] > 0.f ? gy[i] : 0.f;
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
  dim3 g2((unsigned)ceil_div(D, 256), 3);
  graphnorm_param_reduce<<<g2, 256, 0, st>>>(D, G, part, g_weight, g_bias, g_mean_scale);
  return check_launch("graphnorm_param_reduce");
}

extern "C" int mvml_relu_bwd(int64_t n, const float* y, const float* g_y, float* g_x, void* stream) {
  clear_error();
  MVML_REQUIRE(n >= 0, "relu_bwd: bad size");
  if (n == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(n, 256), 16384);
  relu_bwd_kernel<<<blocks, 256, 0, st>>>(n, y, g_y, g_x);
  return check_launch("relu_bwd_kernel");
}
