// blend_row.h — one transaction's ensemble epilogue, shared by the blend kernel (blend.hip) and the fused
// ensemble kernel (ensemble.hip): per-model clamp + confidence, weighted-average / voting / stacking,
// decision and risk level.
// Reference: ml/models/ensemble_predictor.py
//   _predict_single_model clamp            :202-203   fraud_prob = max(0.0, min(1.0, p))
//   _calculate_model_confidence            :325-342   min(1.0, |p-0.5| * 2 * mult)
//   _weighted_average_ensemble             :263-284
//   _voting_ensemble                       :286-303
//   _stacking_ensemble                     :305-323
//   _make_decision / _calculate_risk_level :344-369
// Arithmetic is f64 with FP contraction off and the reference's evaluation order, so every output is the
// value the Python float code computes for the same inputs.
#pragma once

#include "fd_internal.h"

namespace fd {

struct BlendConsts {  // the present models only, in the caller's model order
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

__device__ __forceinline__ void blend_row(const BlendConsts& a, const double* raw, double& fp, double& conf,
                                          uint8_t& dec, uint8_t& risk) {
#pragma clang fp contract(off)
  double p[FD_MAX_MODELS], c[FD_MAX_MODELS];
  const int nm = a.n_models;
#pragma unroll
  for (int m = 0; m < FD_MAX_MODELS; ++m) {
    if (m < nm) {
      const double q = py_max(0.0, py_min(1.0, raw[m]));
      p[m] = q;
      const double dist = fabs(q - 0.5);
      c[m] = py_min(1.0, (dist * 2.0) * a.mult[m]);
    }
  }
  fp = 0.0;
  conf = 0.0;
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
  if (conf < a.confidence_threshold) dec = FD_REVIEW;
  else if (fp >= 0.95) dec = FD_DECLINE;
  else if (fp >= 0.8) dec = FD_REVIEW;
  else if (fp >= 0.6) dec = FD_APPROVE_WITH_MONITORING;
  else dec = FD_APPROVE;
  if (fp >= 0.95) risk = FD_CRITICAL;
  else if (fp >= 0.8) risk = FD_HIGH;
  else if (fp >= 0.6) risk = FD_MEDIUM;
  else if (fp >= 0.3) risk = FD_LOW;
  else risk = FD_VERY_LOW;
}

struct Cols {
  const double* p[FD_MAX_MODELS];
};

// the present models of fd_blend_params (failed / absent models dropped: weights renormalise over the rest)
inline BlendConsts blend_consts(const fd_blend_params& p, const uint8_t* present) {
  BlendConsts a{};
  int k = 0;
  for (int m = 0; m < p.n_models; ++m) {
    if (present && !present[m]) continue;
    a.weight[k] = p.weight[m];
    a.mult[k] = p.conf_mult[m];
    ++k;
  }
  a.n_models = k;
  a.strategy = p.strategy;
  a.fraud_threshold = p.fraud_threshold;
  a.confidence_threshold = p.confidence_threshold;
  return a;
}

}  // namespace fd
