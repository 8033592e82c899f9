// GraphNorm (torch_geometric 2.2.0, model.py:85 and 93) forward/backward with per-group
// statistics, and the ReLU backward of GNNModule.fc (model.py:86-87).
//
// Reference semantics with batch=None: the normalisation group is the whole mini-batch passed
// to GNNModule.forward (64 molecules, config.py:21).  Groups are rows [off[g], off[g+1]).
//   mean = sum(x)/n;  o = x - mean*mean_scale;  var = sum(o^2)/n;  std = sqrt(var + eps)
//   y = weight*o/std + bias
// One thread per (group, column): column reads of a 768-wide row are coalesced across the
// workgroup.  Parameter gradients are reduced over groups in fixed order (no atomics).
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
  const float n = (float)(r1 - r0);
  float s = 0.f;
  for (int64_t r = r0; r < r1; ++r) s += x[r * D + col];
  const float mean = s / n;
  const float msc = ms[col];
  float v = 0.f;
  for (int64_t r = r0; r < r1; ++r) {
    const float o = x[r * D + col] - mean * msc;
    v += o * o;
  }
  const float stdv = sqrtf(v / n + eps);
  const float wc = w[col], bc = b[col];
  for (int64_t r = r0; r < r1; ++r) {
    const float o = x[r * D + col] - mean * msc;
    y[r * D + col] = wc * o / stdv + bc;
  }
}

// Per (group, column): g_x and the group's partial parameter gradients.
__global__ void graphnorm_bwd_kernel(int D, const int64_t* __restrict__ off, const float* __restrict__ x,
                                     const float* __restrict__ w, const float* __restrict__ ms, float eps,
                                     const float* __restrict__ gy, float* __restrict__ gx,
                                     float* __restrict__ part /* [3][G][D] */, int64_t G) {
  const int col = blockIdx.y * blockDim.x + threadIdx.x;
  if (col >= D) return;
  const int64_t g = blockIdx.x;
  const int64_t r0 = off[g], r1 = off[g + 1];
  float pw = 0.f, pb = 0.f, pms = 0.f;
  if (r1 > r0) {
    const float n = (float)(r1 - r0);
    float s = 0.f;
    for (int64_t r = r0; r < r1; ++r) s += x[r * D + col];
    const float mean = s / n;
    const float msc = ms[col], wc = w[col];
    float v = 0.f, so = 0.f, sgy = 0.f, sgyo = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
      const float o = x[r * D + col] - mean * msc;
      const float gyr = gy[r * D + col];
      v += o * o;
      so += o;
      sgy += gyr;
      sgyo += gyr * o;
    }
    const float stdv = sqrtf(v / n + eps);
    const float inv = 1.f / stdv;
    // g_o_j = w/std * (g_y_j - S1 * o_j / (n std^2)),  S1 = sum g_y o
    const float k1 = wc * inv;
    const float k2 = sgyo / (n * stdv * stdv);
    const float sum_go = k1 * (sgy - k2 * so);
    for (int64_t r = r0; r < r1; ++r) {
      const float o = x[r * D + col] - mean * msc;
      const float go = k1 * (gy[r * D + col] - k2 * o);
      gx[r * D + col] = go - msc * sum_go / n;
    }
    pw = sgyo * inv;
    pb = sgy;
    pms = -mean * sum_go;
  }
  part[(0 * G + g) * D + col] = pw;
  part[(1 * G + g) * D + col] = pb;
  part[(2 * G + g) * D + col] = pms;
}

__global__ void graphnorm_param_reduce(int D, int64_t G, const float* __restrict__ part,
                                       float* __restrict__ gw, float* __restrict__ gb,
                                       float* __restrict__ gms) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  const int which = blockIdx.y;
  if (col >= D) return;
  float s = 0.f;
  for (int64_t g = 0; g < G; ++g) s += part[((int64_t)which * G + g) * D + col];
  float* dst = which == 0 ? gw : (which == 1 ? gb : gms);
  if (dst) dst[col] = s;
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
  return carve_size((size_t)3 * G * D * sizeof(float));
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
  float* part = static_cast<float*>(workspace);
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
