// The training step's optimizer update on flat buffers (round 6): main.py:88's
// torch.optim.Adam(model.parameters(), lr, weight_decay) as three launches over every
// parameter, with the per-parameter "has a gradient" decision kept on the device.
//
// torch skips a parameter whose .grad is None (the reference's never-used LayerNorms,
// model.py:42, 120); under data parallelism only the all-reduced presence flags say whether
// ANY rank produced one, and reading them on the host costs a blocking copy per step.  Here
// the flags travel in the gradient buffer (after the gradients, one all-reduce for both) and
// the update kernel reads them: no host synchronisation anywhere in the step.
//  * mvml_grad_gather: this step's gradient tensors (a device table of pointers, NULL = no
//    gradient on this rank) -> the flat gradient buffer (zeros for absent ones) + 1.0 / 0.0
//    presence flags.
//  * mvml_adam_flat: for every parameter whose flag is > 0: torch's Adam arithmetic (L2 weight
//    decay into the gradient, exp_avg lerp, exp_avg_sq, bias corrections of the parameter's
//    own step count in double as torch's host-side step does), the gradient scaled by
//    grad_scale first (1 / world for a mean over ranks).
//  * mvml_adam_steps: the per-parameter step counters advance (after the update read them).
// Workgroup c works on chunk c of a static chunk table (a chunk never straddles parameters).
#include "common.h"

namespace mvml {
namespace {

constexpr int kOptThreads = 256;

__global__ void __launch_bounds__(kOptThreads)
grad_gather_kernel(const int32_t* __restrict__ chunk_param, const int64_t* __restrict__ chunk_beg,
                   const int64_t* __restrict__ chunk_end, const int64_t* __restrict__ param_off,
                   const uint64_t* __restrict__ src, int P, float* __restrict__ flat, int64_t numel) {
  const int c = blockIdx.x;
  const int i = chunk_param[c];
  const int64_t b = chunk_beg[c], e = chunk_end[c], off = param_off[i];
  const float* s = reinterpret_cast<const float*>(src[i]);
  if (c == 0)
    for (int q = threadIdx.x; q < P; q += kOptThreads) flat[numel + q] = src[q] ? 1.f : 0.f;
  // segments start 16-B aligned (host: param_off % 4 == 0) but a gradient tensor need not be
  for (int64_t k = b + threadIdx.x; k < e; k += kOptThreads) flat[k] = s ? s[k - off] : 0.f;
}

__global__ void __launch_bounds__(kOptThreads)
adam_flat_kernel(const int32_t* __restrict__ chunk_param, const int64_t* __restrict__ chunk_beg,
                 const int64_t* __restrict__ chunk_end, const float* __restrict__ flags,
                 const int32_t* __restrict__ steps, float* __restrict__ param, const float* __restrict__ grad,
                 float* __restrict__ m, float* __restrict__ v, double lr, double beta1, double beta2,
                 float eps, float weight_decay, float grad_scale) {
  const int c = blockIdx.x;
  const int i = chunk_param[c];
  if (!(flags[i] > 0.f)) return;  // no rank produced a gradient: torch skips the parameter
  const int64_t b = chunk_beg[c], e = chunk_end[c];
  const int step = steps[i] + 1;
  // torch (non-capturable Adam): the hyper-parameters are Python doubles, the bias corrections
  // and 1 - beta are formed in double and only then rounded to the tensor's float (1 - 0.999f
  // in float would be 1.3e-5 off 0.001, a systematic offset of exp_avg_sq)
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2 = 1.0 - pow(beta2, (double)step);
  const float step_size = (float)(lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  const float w1 = (float)(1.0 - beta1), w2 = (float)(1.0 - beta2), b2 = (float)beta2;
  for (int64_t k = b + threadIdx.x; k < e; k += kOptThreads) {
    float g = grad[k];
    if (grad_scale != 1.f) g *= grad_scale;
    float p = param[k];
    if (weight_decay != 0.f) g = g + weight_decay * p;  // grad.add(param, alpha=weight_decay)
    float mk = m[k];
    mk = mk + w1 * (g - mk);                            // exp_avg.lerp_(grad, 1 - beta1)
    const float vk = v[k] * b2 + w2 * g * g;             // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
    const float denom = sqrtf(vk) / bc2_sqrt + eps;
    p = p - step_size * (mk / denom);                   // param.addcdiv_(exp_avg, denom, -step_size)
    m[k] = mk;
    v[k] = vk;
    param[k] = p;
  }
}

__global__ void adam_steps_kernel(int P, const float* __restrict__ flags, int32_t* __restrict__ steps) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < P && flags[i] > 0.f) steps[i] += 1;
}

}  // namespace
}  // namespace mvml

using namespace mvml;

extern "C" int mvml_grad_gather(int64_t nchunks, const int32_t* chunk_param, const int64_t* chunk_beg,
                                const int64_t* chunk_end, const int64_t* param_off, const uint64_t* src,
                                int P, float* flat, int64_t numel, void* stream) {
  clear_error();
  MVML_REQUIRE(nchunks >= 0 && nchunks < (int64_t(1) << 31) && P >= 0 && numel >= 0 && flat,
               "grad_gather: bad arguments");
  if (nchunks == 0) return MVML_OK;
  grad_gather_kernel<<<(unsigned)nchunks, kOptThreads, 0, as_stream(stream)>>>(
      chunk_param, chunk_beg, chunk_end, param_off, src, P, flat, numel);
  return check_launch("grad_gather_kernel");
}

extern "C" int mvml_adam_flat(int64_t nchunks, const int32_t* chunk_param, const int64_t* chunk_beg,
                              const int64_t* chunk_end, const float* flags, int32_t* steps, int P,
                              float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                              double lr, double beta1, double beta2, double eps, double weight_decay,
                              float grad_scale, void* stream) {
  clear_error();
  MVML_REQUIRE(nchunks >= 0 && nchunks < (int64_t(1) << 31) && P >= 0 && flags && steps,
               "adam_flat: bad arguments");
  MVML_REQUIRE(beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && eps >= 0.0 && lr >= 0.0,
               "adam_flat: bad hyper-parameters");
  if (nchunks == 0 || P == 0) return MVML_OK;
  hipStream_t st = as_stream(stream);
  adam_flat_kernel<<<(unsigned)nchunks, kOptThreads, 0, st>>>(chunk_param, chunk_beg, chunk_end, flags, steps,
                                                              param, grad, exp_avg, exp_avg_sq, lr, beta1,
                                                              beta2, (float)eps, (float)weight_decay,
                                                              grad_scale);
  int rc = check_launch("adam_flat_kernel");
  if (rc) return rc;
  adam_steps_kernel<<<(unsigned)ceil_div(P, 256), 256, 0, st>>>(P, flags, steps);
  return check_launch("adam_steps_kernel");
}
