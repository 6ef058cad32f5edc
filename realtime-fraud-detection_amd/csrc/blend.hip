// blend.hip — ensemble epilogue for a batch: per-model clamp + confidence, weighted-average /
// voting / stacking combination, decision and risk level.
// Reference: ml/models/ensemble_predictor.py
//   _predict_single_model clamp            :202-203   fraud_prob = max(0.0, min(1.0, p))
//   _calculate_model_confidence            :325-342   min(1.0, |p-0.5| * 2 * mult)
//   _weighted_average_ensemble             :263-284
//   _voting_ensemble                       :286-303
//   _stacking_ensemble                     :305-323
//   _make_decision / _calculate_risk_level :344-369
// Arithmetic is f64 with FP contraction off and the reference's evaluation order, so every output
// is the value the Python float code computes for the same inputs.
#include "fd_internal.h"

namespace fd {
namespace {

struct BlendArgs {
  const double* probs[FD_MAX_MODELS];
  double weight[FD_MAX_MODELS];
  double mult[FD_MAX_MODELS];
  int n_models;
  int strategy;
  double fraud_threshold;
  double confidence_threshold;
};

// Python's min(a, b) returns a unless b < a; max(a, b) returns a unless b > a.
__device__ __forceinline__ double py_min(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double py_max(double a, double b) { return (b > a) ? b : a; }

__global__ void __launch_bounds__(256) blend_kernel(BlendArgs a, int64_t n, double* __restrict__ out_fp,
                                                     double* __restrict__ out_conf,
                                                     uint8_t* __restrict__ out_dec,
                                                     uint8_t* __restrict__ out_risk) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double p[FD_MAX_MODELS], c[FD_MAX_MODELS];
#pragma unroll
  for (int m = 0; m < FD_MAX_MODELS; ++m) {
    if (m < a.n_models) {
      const double raw = a.probs[m][i];
      const double q = py_max(0.0, py_min(1.0, raw));
      p[m] = q;
      const double dist = fabs(q - 0.5);
      c[m] = py_min(1.0, (dist * 2.0) * a.mult[m]);
    }
  }
  double fp = 0.0, conf = 0.0;
  const int nm = a.n_models;
  auto weighted = [&](double& f, double& cf) {
    double tw = 0.0, ws = 0.0, cs = 0.0;
    for (int m = 0; m < nm; ++m) {
      ws = ws + p[m] * a.weight[m];
      cs = cs + c[m] * a.weight[m];
      tw = tw + a.weight[m];
    }
    if (tw == 0.0) {
      f = 0.5;
      cf = 0.0;
    } else {
      f = ws / tw;
      cf = cs / tw;
    }
  };
  if (a.strategy == FD_BLEND_VOTING) {
    int votes = 0;
    double cs = 0.0;
    for (int m = 0; m < nm; ++m) {
      if (p[m] > a.fraud_threshold) ++votes;
      cs = cs + c[m];
    }
    fp = nm > 0 ? (double)votes / (double)nm : 0.0;
    conf = nm > 0 ? cs / (double)nm : 0.0;
  } else if (a.strategy == FD_BLEND_STACKING) {
    double tc = 0.0;
    for (int m = 0; m < nm; ++m) tc = tc + c[m];  // sum(): starts at int 0, same value
    if (tc == 0.0) {
      weighted(fp, conf);
    } else {
      double ws = 0.0;
      for (int m = 0; m < nm; ++m) ws = ws + p[m] * c[m];
      fp = ws / tc;
      conf = tc / (double)nm;
    }
  } else {
    weighted(fp, conf);
  }
  uint8_t dec;
  if (conf < a.confidence_threshold) dec = FD_REVIEW;
  else if (fp >= 0.95) dec = FD_DECLINE;
  else if (fp >= 0.8) dec = FD_REVIEW;
  else if (fp >= 0.6) dec = FD_APPROVE_WITH_MONITORING;
  else dec = FD_APPROVE;
  uint8_t risk;
  if (fp >= 0.95) risk = FD_CRITICAL;
  else if (fp >= 0.8) risk = FD_HIGH;
  else if (fp >= 0.6) risk = FD_MEDIUM;
  else if (fp >= 0.3) risk = FD_LOW;
  else risk = FD_VERY_LOW;
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
  BlendArgs a{};
  int k = 0;
  for (int m = 0; m < p.n_models; ++m) {
    if (present && !present[m]) continue;  // failed model: dropped, weights renormalise over the rest
    FD_REQUIRE(d_probs && d_probs[m], FD_ERR_INVALID_ARG, "null probability column");
    a.probs[k] = d_probs[m];
    a.weight[k] = p.weight[m];
    a.mult[k] = p.conf_mult[m];
    ++k;
  }
  FD_REQUIRE(k > 0, FD_ERR_INVALID_ARG, "No model predictions available");
  a.n_models = k;
  a.strategy = p.strategy;
  a.fraud_threshold = p.fraud_threshold;
  a.confidence_threshold = p.confidence_threshold;
  const int64_t blocks = (n + 255) / 256;
  Engine::Timed* ev = e.timing ? e.next_event_pair(FD_TIMING_BLEND) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, e.stream));
  hipLaunchKernelGGL(blend_kernel, dim3((unsigned)blocks), dim3(256), 0, e.stream, a, n, d_fp, d_conf,
                     d_dec, d_risk);
  FD_HIP(hipGetLastError());
  if (ev) FD_HIP(hipEventRecord(ev->b, e.stream));
}

}  // namespace fd
