/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into or called by the product path
 * (realtime-fraud-detection_amd/). Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it, as the checker / CPU baseline.
 *
 * Plain-C restatement of the reference's tree-ensemble scoring, walking the ORIGINAL node arrays
 * (not the engine's repacked layout):
 *
 *  orc_xgb_predict   xgboost 2.0.3 gbtree CPU predictor for binary:logistic, as called by
 *                    ml/models/model_manager.py:309-311 (XGBClassifier.predict_proba(X)[:, 1]).
 *                    Third-party algorithm (xgboost==2.0.3, services/ml-models/requirements.txt:3,
 *                    absent here): per row, margin = ProbToMargin(base_score) in f32, then for each
 *                    tree in order walk `fvalue < split_cond ? left : right` (missing -> default
 *                    child) and add the f32 leaf weight; p = common::Sigmoid(margin).
 *                    PARITY UNPINNED against the library itself (not installable offline); pinned
 *                    by hand-computed known-answer trees in tests/test_oracle_forest.py.
 *  orc_iforest_predict  sklearn IsolationForest.decision_function + the reference's
 *                    1/(1+exp(s)) (ml/models/model_manager.py:338-346): tree.apply compares
 *                    (double)x_f32 <= threshold_f64 (NaN -> missing_go_to_left), depths += (dpl +
 *                    apl - 1) in estimator order (f64), score = 2**(-depths/denominator).
 *                    Pinned against sklearn 1.7.2 outputs in tests/golden/ (make_golden.py).
 *
 * Rows are independent; OpenMP parallelises over rows only, never inside a row's sum.
 */
#include <math.h>
#include <stdint.h>
#include <stddef.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static inline float xgb_sigmoid(float x) {
  /* xgboost src/common/math.h common::Sigmoid */
  const float kEps = 1e-16f;
  float xm = -x;
  if (xm > 88.7f) xm = 88.7f;
  const float denom = expf(xm) + 1.0f + kEps;
  return 1.0f / denom;
}

float orc_xgb_base_margin(double base_score) {
  const float bs = (float)base_score;
  return -logf(1.0f / bs - 1.0f);
}

int orc_xgb_predict(int64_t n, int32_t ld, const float* X, int32_t n_trees, const int64_t* offs,
                    const int32_t* left, const int32_t* right, const int32_t* feature,
                    const double* thr, const uint8_t* dl, const double* leafv, double base_score,
                    int32_t nthreads, float* margin_out, float* prob_out, int32_t* leaf_out) {
  const float base = orc_xgb_base_margin(base_score);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static) if (nthreads != 1)
#endif
  for (int64_t r = 0; r < n; ++r) {
    const float* x = X + r * (int64_t)ld;
    float m = base;
    for (int32_t t = 0; t < n_trees; ++t) {
      const int64_t o = offs[t];
      int32_t nid = 0;
      while (left[o + nid] != -1) {
        const int32_t f = feature[o + nid];
        const float fv = (f < ld) ? x[f] : NAN;
        if (isnan(fv)) {
          nid = (dl && dl[o + nid]) ? left[o + nid] : right[o + nid];
        } else {
          nid = (fv < (float)thr[o + nid]) ? left[o + nid] : right[o + nid];
        }
      }
      m += (float)leafv[o + nid];
      if (leaf_out) leaf_out[r * n_trees + t] = nid;
    }
    if (margin_out) margin_out[r] = m;
    if (prob_out) prob_out[r] = xgb_sigmoid(m);
  }
  return 0;
}

int orc_iforest_predict(int64_t n, int32_t ld, const float* X, int32_t n_trees, const int64_t* offs,
                        const int32_t* left, const int32_t* right, const int32_t* feature,
                        const double* thr, const uint8_t* dl, const double* leafv, double offset,
                        double denominator, int32_t nthreads, double* depth_out, double* prob_out,
                        int32_t* leaf_out) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static) if (nthreads != 1)
#endif
  for (int64_t r = 0; r < n; ++r) {
    const float* x = X + r * (int64_t)ld;
    double depths = 0.0;
    for (int32_t t = 0; t < n_trees; ++t) {
      const int64_t o = offs[t];
      int32_t nid = 0;
      while (left[o + nid] != -1) {
        const int32_t f = feature[o + nid];
        const float fv = (f < ld) ? x[f] : NAN;
        if (isnan(fv)) {
          nid = (dl && dl[o + nid]) ? left[o + nid] : right[o + nid];
        } else if ((double)fv <= thr[o + nid]) {
          nid = left[o + nid];
        } else {
          nid = right[o + nid];
        }
      }
      depths += leafv[o + nid];
      if (leaf_out) leaf_out[r * n_trees + t] = nid;
    }
    const double q = (denominator != 0.0) ? depths / denominator : 1.0;
    const double score = pow(2.0, -q);
    const double decision = -score - offset;
    if (depth_out) depth_out[r] = depths;
    if (prob_out) prob_out[r] = 1.0 / (1.0 + exp(decision));
  }
  return 0;
}

/* Ensemble blend, weighted-average strategy (ensemble_predictor.py:263-284 with the clamp :203 and
   confidence :325-342), f64 in the reference's order. Used only by bench.py's full-pipeline CPU
   baseline; the exact restatement tested against the reference is scoring_ref.py. */
int orc_blend_weighted(int64_t n, int32_t n_models, const double* probs /* n_models x n */,
                       const double* weight, const double* mult, double confidence_threshold,
                       int32_t nthreads, double* fp_out, double* conf_out, uint8_t* dec_out,
                       uint8_t* risk_out) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static) if (nthreads != 1)
#endif
  for (int64_t i = 0; i < n; ++i) {
    double tw = 0.0, ws = 0.0, cs = 0.0;
    for (int m = 0; m < n_models; ++m) {
      double p = probs[(int64_t)m * n + i];
      p = (p < 1.0) ? p : 1.0;
      p = (p > 0.0) ? p : 0.0;
      double c = fabs(p - 0.5) * 2.0 * mult[m];
      c = (c < 1.0) ? c : 1.0;
      ws += p * weight[m];
      cs += c * weight[m];
      tw += weight[m];
    }
    const double fp = tw == 0.0 ? 0.5 : ws / tw, conf = tw == 0.0 ? 0.0 : cs / tw;
    fp_out[i] = fp;
    conf_out[i] = conf;
    dec_out[i] = conf < confidence_threshold ? 1 : (fp >= 0.95 ? 2 : (fp >= 0.8 ? 1 : (fp >= 0.6 ? 3 : 0)));
    risk_out[i] = fp >= 0.95 ? 4 : (fp >= 0.8 ? 3 : (fp >= 0.6 ? 2 : (fp >= 0.3 ? 1 : 0)));
  }
  return 0;
}
