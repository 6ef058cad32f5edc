// blend.hip — ensemble epilogue for a batch of per-model probability columns (the per-model path; the
// fused ensemble kernel runs the same blend_row in its own epilogue). Semantics and reference lines:
// blend_row.h.
#include "blend_row.h"

namespace fd {
namespace {

__global__ void __launch_bounds__(256) blend_kernel(BlendConsts a, Cols cols, int64_t n, double* __restrict__ out_fp,
                                                     double* __restrict__ out_conf, uint8_t* __restrict__ out_dec,
                                                     uint8_t* __restrict__ out_risk) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double raw[FD_MAX_MODELS];
#pragma unroll
  for (int m = 0; m < FD_MAX_MODELS; ++m) raw[m] = m < a.n_models ? cols.p[m][i] : 0.0;
  double fp, conf;
  uint8_t dec, risk;
  blend_row(a, raw, fp, conf, dec, risk);
  out_fp[i] = fp;
  if (out_conf) out_conf[i] = conf;
  if (out_dec) out_dec[i] = dec;
  if (out_risk) out_risk[i] = risk;
}

}  // namespace

void launch_blend(Engine& e, const fd_blend_params& p, int64_t n, const double* const* d_probs,
                  const uint8_t* present, double* d_fp, double* d_conf, uint8_t* d_dec, uint8_t* d_risk) {
  FD_REQUIRE(p.n_models >= 0 && p.n_models <= FD_MAX_MODELS, FD_ERR_INVALID_ARG, "n_models out of range");
  FD_REQUIRE(d_fp != nullptr, FD_ERR_INVALID_ARG, "null output");
  if (n == 0) return;
  const BlendConsts a = blend_consts(p, present);
  FD_REQUIRE(a.n_models > 0, FD_ERR_INVALID_ARG, "No model predictions available");
  Cols cols{};
  int k = 0;
  for (int m = 0; m < p.n_models; ++m) {
    if (present && !present[m]) continue;
    FD_REQUIRE(d_probs && d_probs[m], FD_ERR_INVALID_ARG, "null probability column");
    cols.p[k++] = d_probs[m];
  }
  const int64_t blocks = (n + 255) / 256;
  Engine::Timed* ev = e.timing ? e.next_event_pair(FD_TIMING_BLEND) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, e.stream));
  hipLaunchKernelGGL(blend_kernel, dim3((unsigned)blocks), dim3(256), 0, e.stream, a, cols, n, d_fp, d_conf, d_dec,
                     d_risk);
  FD_HIP(hipGetLastError());
  if (ev) FD_HIP(hipEventRecord(ev->b, e.stream));
}

}  // namespace fd
