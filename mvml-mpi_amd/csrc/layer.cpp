// One GATConv's whole backward behind one C entry point (SURVEY §8(b)'s `proj_bwd`, round 6):
// the sequence mvml_gat.functional.GATLayerFunction.backward runs (aggregation backward, the
// weight-gradient product, the unfolding into fc / res_fc, the re-associated attention-vector
// gradients, the bias column sums and the per-row-scaled data-gradient product), enqueued by
// native code over a caller-sized workspace, so a C caller needs no re-derivation of the
// operand maxima, row maxima and scratch the pieces share.  Reference: dgllife GATLayer /
// dgl GATConv backward (/root/reference/model.py:81, 91; autograd of GATConv.forward, dgl 0.9.1).
#include <stdint.h>

#include "common.h"

namespace mvml {
namespace {

int64_t round4(int64_t x) { return (x + 3) / 4 * 4; }
int64_t row_pitch(int64_t c) { return (c + 63) / 64 * 64; }  // functional._row_pitch

struct LayerBwdPlan {
  int64_t Fp, C, CE, ldg, outc;
  size_t gy, gyr, amx, gW, wil, agg, gemm, total;
};

LayerBwdPlan layer_bwd_plan(int64_t N, int64_t E, int H, int F, int Fin, int mean) {
  LayerBwdPlan p{};
  p.Fp = round4(Fin);
  p.C = mvml_gat_proj_cols(H, F, mean);
  p.CE = p.C + 2 * H;
  p.ldg = row_pitch(p.CE);
  p.outc = mean ? F : (int64_t)H * F;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += carve_size(bytes);
    return o;
  };
  p.amx = take(4 * sizeof(uint32_t));
  p.gy = take((size_t)N * p.ldg * sizeof(float));
  p.gyr = take((size_t)std::max<int64_t>(N, 1) * sizeof(uint32_t));
  p.gW = take((size_t)p.CE * p.Fp * sizeof(float));
  p.wil = take((size_t)p.CE * p.Fp * sizeof(float));
  p.agg = take(mvml_gat_agg_bwd_workspace_size(E, H));
  p.gemm = take(std::max(mvml_gemm_colsum_workspace_size(p.CE, p.Fp, N, (int64_t)H * F),
                         mvml_gemm_workspace_size(N, Fin, p.CE)));
  p.total = off;
  return p;
}

}  // namespace
}  // namespace mvml

using namespace mvml;

extern "C" size_t mvml_gat_layer_bwd_workspace_size(int64_t num_nodes, int64_t num_edges, int H, int F,
                                                    int Fin, int mean) {
  if (num_nodes < 0 || num_edges < 0 || H <= 0 || F <= 0 || Fin <= 0) return 0;
  return layer_bwd_plan(num_nodes, num_edges, H, F, Fin, mean ? 1 : 0).total;
}

extern "C" int mvml_gat_layer_bwd(int64_t N, const int32_t* node_groups, int64_t num_groups,
                                  const int32_t* in_rowptr, const int32_t* in_src, const int32_t* out_rowptr,
                                  const int32_t* out_dst, const int32_t* out_inslot, int64_t num_edges,
                                  int H, int F, int Fin, int mean, float slope, const float* X,
                                  const float* Wcat, const float* attn_lr, const float* Y, int64_t ldy,
                                  const float* elr, const float* attn, const float* out, const float* g_out,
                                  float* g_X, float* g_fc, float* g_res, float* g_attn, float* g_bias,
                                  void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  MVML_REQUIRE(N >= 0 && num_edges >= 0 && H > 0 && F > 0 && Fin > 0 && X && Wcat && attn_lr && Y && elr &&
                   attn && out && g_out && g_fc && g_res && g_attn && g_bias,
               "gat_layer_bwd: bad arguments");
  const LayerBwdPlan p = layer_bwd_plan(N, num_edges, H, F, Fin, mean ? 1 : 0);
  if (!workspace || workspace_bytes < p.total) {
    set_error("gat_layer_bwd: workspace too small (need %zu)", p.total);
    return MVML_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  uint32_t* amx = reinterpret_cast<uint32_t*>(ws + p.amx);  // [max |X|, max |Wcat|, max |gY|, -]
  float* gY = reinterpret_cast<float*>(ws + p.gy);
  uint32_t* gyr = reinterpret_cast<uint32_t*>(ws + p.gyr);
  float* gW = reinterpret_cast<float*>(ws + p.gW);
  float* wil = reinterpret_cast<float*>(ws + p.wil);
  const int64_t HF = (int64_t)H * F;
  const int mode = mean ? 1 : 0;  // 0: flatten + ELU (dgllife's hidden layers), 1: head mean
  int rc;
#define MVML_TRY(call)    \
  do {                    \
    rc = (call);          \
    if (rc) return rc;    \
  } while (0)
  if (hipMemsetAsync(amx, 0, 4 * sizeof(uint32_t), st) != hipSuccess) {
    set_error("gat_layer_bwd: hipMemsetAsync failed");
    return MVML_ERR_LAUNCH;
  }
  // operand maxima of the split-fp16 products: X (the weight gradient's B), Wcat (the data
  // gradient's B, split once into its interleaved image), gY (folded by the aggregation backward)
  MVML_TRY(mvml_absmax_f32(N, p.Fp, X, p.Fp, amx + 0, 1, stream));
  MVML_TRY(mvml_absmax_f32(p.CE, p.Fp, Wcat, p.Fp, amx + 1, 1, stream));
  // gY = [dZ | dR | d el | d er] with per-row maxima (the data gradient's per-row scales)
  MVML_TRY(mvml_gat_agg_bwd(N, node_groups, num_groups, in_rowptr, in_src, out_rowptr, out_dst, out_inslot, Y,
                            ldy, elr, attn, out, g_out, H, F, slope, mode, gY, p.ldg, amx + 2,
                            g_X ? gyr : nullptr, ws + p.agg, mvml_gat_agg_bwd_workspace_size(num_edges, H),
                            stream));
  // dL/d[Wcat ; A_l ; A_r] = gY^T X (split-K over atoms), unfolded into fc / res_fc; with it the
  // bias gradient: column sums of g_rst = gY's residual columns (mean: g_out / H, the same for
  // every head)
  const size_t gws = std::max(mvml_gemm_colsum_workspace_size(p.CE, p.Fp, N, HF),
                              mvml_gemm_workspace_size(N, Fin, p.CE));
  MVML_TRY(mvml_gemm_f16x2_amax_colsum(p.CE, p.Fp, N, gY, p.ldg, X, p.Fp, amx + 2, amx + 0, gW, p.Fp, HF,
                                       mean ? F : HF, mean ? 1.f / H : 1.f, g_bias, ws + p.gemm, gws, stream));
  MVML_TRY(mvml_gat_unfold_grads(gW, attn_lr, H, F, Fin, (int)p.Fp, mean ? 1 : 0, g_fc, g_res, stream));
  // attention vectors, re-associated: per head, rows [G_l ; G_r] of gW times its F rows of Wcat
  MVML_TRY(mvml_gemm_f32x3_batched(0, 0, 2, F, p.Fp, H, gW + p.C * p.Fp, (int64_t)H * p.Fp, p.Fp, Wcat, p.Fp,
                                   (int64_t)F * p.Fp, nullptr, 0.f, 0, g_attn, HF, F, stream));
  if (mean) {
    for (int h = 1; h < H; ++h)
      if (hipMemcpyAsync(g_bias + (int64_t)h * F, g_bias, F * sizeof(float), hipMemcpyDeviceToDevice, st) !=
          hipSuccess) {
        set_error("gat_layer_bwd: hipMemcpyAsync failed");
        return MVML_ERR_LAUNCH;
      }
  }
  // dL/dX = gY Wcat, every atom's row at its own scale, Wcat from its interleaved image
  if (g_X) {
    MVML_TRY(mvml_split_f16x2_il4(p.CE, p.Fp, Wcat, p.Fp, amx + 1, wil, stream));
    MVML_TRY(mvml_gemm_f16x2_rows(N, Fin, p.CE, gY, p.ldg, Wcat, p.Fp, 1, wil, gyr, amx + 1, nullptr, 0.f, 0, g_X,
                                  Fin, ws + p.gemm, gws, stream));
  }
#undef MVML_TRY
  return MVML_OK;
}
