/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). Never linked into the product.
 *
 * C restatement of the feature half of the hot path, sequential in arrival order, for large
 * batches (the pure-Python chain oracle/velocity_ref.py + features_ref.py covers small cases and is
 * what this file is cross-checked against in tests/test_oracle_features.py):
 *
 *   Java FeatureExtractor (services/flink-jobs/.../features/FeatureExtractor.java:92-363) for the
 *   bridged features, velocity read (RedisService.java:198-207) BEFORE the sink's write
 *   (RedisTransactionSink.java:116-135, TTL 3600 s RedisService.java:47,188), then
 *   FeatureProcessor.process_features (services/ml-models/src/models/feature_processor.py:161-402)
 *   and EnsemblePredictor._prepare_features (ensemble_predictor.py:221-250) for the bridged dict.
 *
 * Declared engine semantics and the parity status: oracle/velocity_ref.py header, DESIGN.md.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_RAW 16
#define ORC_VEC 64

typedef struct {
  int64_t cap;  /* power of two */
  uint64_t* keys;
  int mode, K;
  /* per card */
  int32_t* cnt;
  int64_t* sum;
  int64_t* last_ts;
  uint8_t* has_ts;
  int32_t* ring_n;
  int32_t* ring_head;
  int64_t* ring_ts;    /* cap * K */
  int64_t* ring_cents; /* cap * K */
  /* profiles */
  uint8_t* has_user;
  double* avg;
  int32_t* age;
  uint64_t* fps; /* cap * 3 */
  /* merchants */
  int64_t n_merchants;
  double* m_fr;
  double* m_mult;
} orc_state;

static uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

static int64_t find_or_insert(orc_state* s, uint64_t key) {
  if (key == 0) key = 1; /* 0 marks an empty slot */
  int64_t i = (int64_t)(mix64(key) & (uint64_t)(s->cap - 1));
  for (int64_t probes = 0; probes < s->cap; ++probes) {
    if (s->keys[i] == key) return i;
    if (s->keys[i] == 0) {
      s->keys[i] = key;
      return i;
    }
    i = (i + 1) & (s->cap - 1);
  }
  return -1;
}

void* orc_state_new(int64_t cap, int32_t mode, int32_t K) {
  orc_state* s = calloc(1, sizeof(orc_state));
  s->cap = cap;
  s->mode = mode;
  s->K = K;
  s->keys = calloc(cap, 8);
  s->cnt = calloc(cap, 4);
  s->sum = calloc(cap, 8);
  s->last_ts = calloc(cap, 8);
  s->has_ts = calloc(cap, 1);
  s->ring_n = calloc(cap, 4);
  s->ring_head = calloc(cap, 4);
  s->ring_ts = calloc((size_t)cap * K, 8);
  s->ring_cents = calloc((size_t)cap * K, 8);
  s->has_user = calloc(cap, 1);
  s->avg = calloc(cap, 8);
  s->age = calloc(cap, 4);
  s->fps = calloc((size_t)cap * 3, 8);
  return s;
}

void orc_state_free(void* p) {
  orc_state* s = p;
  if (!s) return;
  free(s->keys); free(s->cnt); free(s->sum); free(s->last_ts); free(s->has_ts); free(s->ring_n);
  free(s->ring_head); free(s->ring_ts); free(s->ring_cents); free(s->has_user); free(s->avg);
  free(s->age); free(s->fps); free(s->m_fr); free(s->m_mult);
  free(s);
}

int orc_state_load_users(void* p, int64_t n, const uint64_t* keys, const double* avg, const int32_t* age,
                         const uint64_t* fps) {
  orc_state* s = p;
  for (int64_t i = 0; i < n; ++i) {
    int64_t j = find_or_insert(s, keys[i]);
    if (j < 0) return 1;
    s->has_user[j] = 1;
    s->avg[j] = avg[i];
    s->age[j] = age[i];
    for (int f = 0; f < 3; ++f) s->fps[j * 3 + f] = fps[i * 3 + f];
  }
  return 0;
}

int orc_state_load_merchants(void* p, int64_t n, const double* fr, const double* mult) {
  orc_state* s = p;
  free(s->m_fr);
  free(s->m_mult);
  s->n_merchants = n;
  s->m_fr = malloc(n * 8);
  s->m_mult = malloc(n * 8);
  memcpy(s->m_fr, fr, n * 8);
  memcpy(s->m_mult, mult, n * 8);
  return 0;
}

/* Python max(x, lo) / min(x, hi) (feature_processor.py:231-234) */
static double pmax(double x, double lo) { return (lo > x) ? lo : x; }
static double pmin(double x, double hi) { return (hi < x) ? hi : x; }

/* bridged raw values -> the 64-wide vector (FeatureProcessor + _prepare_features) */
void orc_vector_from_raw(const double* r, float* out) {
  double v[ORC_VEC];
  int k = 0;
  const double amount = pmax(r[0], 0.0);
  double alog = r[1];
  if (isnan(alog) || isinf(alog)) alog = 0.0;
  const double hour = pmin(pmax(r[2], 0.0), 23.0);
  const double dow = pmin(pmax(r[3], 0.0), 6.0);
  double mfr = pmin(pmax(r[5], 0.0), 1.0);
  if (isnan(mfr)) mfr = 0.0;
  const double ip = isnan(r[7]) ? 0.5 : pmin(pmax(r[7], 0.0), 1.0);
  const double uavg = isnan(r[8]) ? 0.0 : pmax(r[8], 0.0);
  const double c5 = pmax(r[9], 0.0), c1 = pmax(r[10], 0.0), c24 = pmax(r[11], 0.0);
  const double s1 = pmax(r[12], 0.0), s24 = pmax(r[13], 0.0);
  double mrisk = pmin(pmax(r[14], 0.0), 1.0);
  if (isnan(mrisk)) mrisk = 0.5;
  const double age = pmax(r[15], 0.0);
  v[k++] = amount;         /* 0 amount */
  v[k++] = alog;           /* 1 amount_log (overwritten below if amount > 0) */
  v[k++] = 0.0;            /* amount_percentile */
  v[k++] = 0.0;            /* amount_zscore */
  v[k++] = 0.0;            /* rounded_amount_frequency */
  v[k++] = hour;           /* 5 hour_of_day */
  v[k++] = dow;            /* 6 day_of_week */
  v[k++] = r[4] > 0.5 ? 1.0 : 0.0; /* is_weekend */
  v[k++] = 0.0;            /* is_holiday */
  v[k++] = 0.0;            /* time_since_last_transaction */
  v[k++] = 0.0;            /* distance_from_home */
  v[k++] = 0.0;            /* location_risk_score */
  v[k++] = 0.5;            /* country_risk_score */
  v[k++] = 0.0;            /* timezone_mismatch */
  v[k++] = c1;             /* 14 user_transaction_count_1h */
  v[k++] = c24;            /* 15 user_transaction_count_24h */
  v[k++] = s24;            /* 16 user_total_amount_24h */
  v[k++] = uavg;           /* 17 user_avg_amount */
  v[k++] = 0.0;            /* user_unique_merchants_24h */
  v[k++] = age;            /* 19 user_account_age_days */
  v[k++] = 0.0;            /* merchant_transaction_count_1h */
  v[k++] = mfr;            /* 21 merchant_fraud_rate */
  v[k++] = 0.0;            /* merchant_avg_amount */
  v[k++] = mrisk;          /* 23 merchant_risk_score */
  v[k++] = 0.5;            /* merchant_category_risk */
  v[k++] = 0.5;            /* device_risk_score */
  v[k++] = r[6] > 0.5 ? 1.0 : 0.0; /* 26 is_new_device */
  v[k++] = ip;             /* 27 ip_risk_score */
  v[k++] = 0.0;            /* is_tor_ip */
  v[k++] = 0.0;            /* is_vpn_ip */
  v[k++] = 0.0;            /* velocity_score */
  v[k++] = s1;             /* 31 amount_velocity_1h */
  v[k++] = c5;             /* 32 transaction_velocity_5m */
  v[k++] = 0.5;            /* payment_method_risk */
  v[k++] = 0.5;            /* card_type_risk */
  v[k++] = 0.0;            /* is_crypto_merchant */
  v[k++] = 0.0;            /* is_gift_card_merchant */
  v[k++] = 0.0;            /* cross_border_transaction */
  v[k++] = 0.0;            /* payment_method_encoded */
  v[k++] = 0.0;            /* merchant_category_encoded */
  v[k++] = 0.0;            /* card_type_encoded */
  /* derived (feature_processor.py:330-363), appended in order when present */
  if (amount > 0) {
    v[1] = log1p(amount);
    v[k++] = sqrt(amount);
  }
  if (uavg > 0) v[k++] = amount / uavg;
  /* merchant_avg_amount is 0 on this path: no amount_to_merchant_avg_ratio */
  if (c24 > 0) v[k++] = c1 / (c24 / 24);
  v[k++] = (0.5 + ip) / 2;
  v[k++] = (9 <= hour && hour <= 17) ? 1.0 : 0.0;
  v[k++] = (hour < 6 || hour > 22) ? 1.0 : 0.0;
  while (k < ORC_VEC) v[k++] = 0.0;
  for (int i = 0; i < ORC_VEC; ++i) {
    double x = v[i];
    if (x < -10.0) x = -10.0;
    if (x > 10.0) x = 10.0;
    out[i] = (float)x;
  }
}

/* also returns velocity_5min_amount (5-minute window sum / 100) per transaction when vel5_out != NULL */
int orc_features_run_ex(void* p, int64_t n, const uint64_t* key, const int64_t* ts, const int64_t* cents,
                        const int32_t* merchant, const uint64_t* dfp, const uint8_t* ipc, const uint8_t* hour_in,
                        const uint8_t* wk_in, double* raw_out, float* vec_out, double* vel5_out) {
  orc_state* s = p;
  const int64_t W[3] = {300000, 3600000, 86400000};
  for (int64_t i = 0; i < n; ++i) {
    double r[ORC_RAW];
    const int64_t t = ts[i];
    const double amount = (double)cents[i] / 100.0;
    int64_t days = t / 86400000;
    if (t % 86400000 < 0) days -= 1;
    int hour = (int)((t - days * 86400000) / 3600000);
    int64_t dw = (days + 3) % 7;
    if (dw < 0) dw += 7;
    const int dow = (int)dw + 1;
    if (hour_in[i] != 255) hour = hour_in[i];
    const int weekend = (wk_in[i] == 255) ? (dow >= 6) : (wk_in[i] != 0);
    const int64_t j = find_or_insert(s, key[i]);
    if (j < 0) return 1;
    double mfr, mult;
    if (merchant[i] >= 0 && merchant[i] < s->n_merchants) {
      mfr = isnan(s->m_fr[merchant[i]]) ? 0.05 : s->m_fr[merchant[i]];
      mult = s->m_mult[merchant[i]];
    } else {
      mfr = 0.1;
      mult = 2.0;
    }
    int known = 0;
    if (s->has_user[j] && dfp[i] != 0)
      for (int f = 0; f < 3; ++f) known |= (s->fps[j * 3 + f] == dfp[i]);
    r[0] = amount;
    r[1] = (amount + 1 > 0) ? log(amount + 1) : ((amount + 1 == 0) ? -INFINITY : NAN);
    r[2] = hour;
    r[3] = dow;
    r[4] = weekend ? 1.0 : 0.0;
    r[5] = mfr;
    r[6] = known ? 0.0 : 1.0;
    r[7] = ipc[i] == 0 ? NAN : (ipc[i] == 1 ? 0.1 : 0.3);
    r[8] = s->has_user[j] ? (isnan(s->avg[j]) ? 0.0 : s->avg[j]) : NAN;
    int64_t c[3] = {0, 0, 0}, sm[3] = {0, 0, 0};
    if (s->mode == 0) {
      const int live = s->has_ts[j] && (t - s->last_ts[j] <= 3600000);
      const int64_t cc = live ? s->cnt[j] : 0, ss = live ? s->sum[j] : 0;
      c[0] = c[1] = c[2] = cc;
      sm[0] = sm[1] = sm[2] = ss;
      s->cnt[j] = (int32_t)(cc + 1);
      s->sum[j] = ss + cents[i];
      s->last_ts[j] = t;
      s->has_ts[j] = 1;
    } else {
      const int K = s->K;
      const int rn = s->ring_n[j];
      for (int e = 0; e < rn; ++e) {
        const int64_t et = s->ring_ts[j * K + e], ec = s->ring_cents[j * K + e];
        for (int w = 0; w < 3; ++w)
          if (t - W[w] < et && et <= t) {
            c[w] += 1;
            sm[w] += ec;
          }
      }
      const int h = s->ring_head[j];
      s->ring_ts[j * K + h] = t;
      s->ring_cents[j * K + h] = cents[i];
      s->ring_head[j] = (h + 1) % K;
      if (rn < K) s->ring_n[j] = rn + 1;
    }
    r[9] = (double)c[0];
    r[10] = (double)c[1];
    r[11] = (double)c[2];
    r[12] = (double)sm[1] / 100.0;
    r[13] = (double)sm[2] / 100.0;
    r[14] = mult;
    r[15] = s->has_user[j] ? s->age[j] : 0;
    if (raw_out) memcpy(raw_out + i * ORC_RAW, r, sizeof(r));
    if (vec_out) orc_vector_from_raw(r, vec_out + i * ORC_VEC);
    if (vel5_out) vel5_out[i] = (double)sm[0] / 100.0;
  }
  return 0;
}

int orc_features_run(void* p, int64_t n, const uint64_t* key, const int64_t* ts, const int64_t* cents,
                     const int32_t* merchant, const uint64_t* dfp, const uint8_t* ipc, const uint8_t* hour_in,
                     const uint8_t* wk_in, double* raw_out, float* vec_out) {
  return orc_features_run_ex(p, n, key, ts, cents, merchant, dfp, ipc, hour_in, wk_in, raw_out, vec_out, NULL);
}
