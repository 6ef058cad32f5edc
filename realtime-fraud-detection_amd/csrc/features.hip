// features.hip — the feature half of the hot path on the device: HBM-resident keyed card state
// (replacing the Redis velocity hashes + profile lookups) and the per-transaction feature vector.
//
// Reference (fl/ = services/flink-jobs/src/main/java/com/frauddetection/):
//   FeatureExtractor.extractAllFeatures      fl/features/FeatureExtractor.java:50-87 (+ :92-363)
//   velocity read / write                    fl/services/RedisService.java:178-207,
//                                            fl/sinks/RedisTransactionSink.java:116-135 (TTL :47,188)
//   FeatureProcessor.process_features        ml/models/feature_processor.py:161-402
//   EnsemblePredictor._prepare_features      ml/models/ensemble_predictor.py:221-250
// Declared semantics (window modes, bridge, unknown user/merchant branches): DESIGN.md "Features".
//
// Micro-batch semantics = the reference's per-element semantics: transactions of one card are
// processed in arrival order, each reading the card's velocity before writing it. Two launches:
//   feat_assign  : per txn, find-or-insert the card slot (open addressing, atomicCAS on the key),
//                  then atomicExch the txn index into the slot's batch-list head (tagged with the
//                  batch epoch, so no per-batch reset of the 2^k-slot table is needed);
//   feat_process : the txn that holds the head owns the card for this batch: it walks the list in
//                  ascending arrival order (repeated min-selection: lists are short; a card seen L
//                  times costs O(L^2) index reads), keeps the card's state in registers, and emits
//                  each transaction's bridged raw features and 64-wide scoring vector.
// Velocity sums are integer cents (exact); amounts leave as cents/100.0 (f64, correctly rounded).
#include <cmath>
#include <cstring>

#include "fd_internal.h"

namespace fd {
namespace {

struct __attribute__((aligned(16))) CardHeader {  // 64 B: one card's header, AoS (random access per txn)
  unsigned long long key;   // 0 = empty slot
  unsigned long long head;  // batch list head: epoch << 32 | txn index
  long long last_ts;        // redis_compat: time of the last velocity write (ms)
  long long sum_cents;      // redis_compat: session amount
  int cnt;                  // redis_compat: session count
  int has_ts;
  int ring_n;               // sliding: events held (<= K)
  int ring_head;            // sliding: next write position
  double avg;               // profile: avg_transaction_amount (NaN = null)
  int age;                  // profile: account_age_days
  unsigned flags;           // bit 0: has a user profile; bits 8-15 seq events held; bits 16-23 seq write pos
};
static_assert(sizeof(CardHeader) == 64, "CardHeader must be 64 B");

struct __attribute__((aligned(16))) RingEvent {
  long long ts;
  long long cents;
};

struct Merchant {
  double fraud_rate;  // NaN = null
  double mult;
};

__device__ __forceinline__ unsigned long long mix64(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

__device__ long long find_or_insert(CardHeader* H, long long mask, unsigned long long key) {
  if (key == 0ull) key = 1ull;  // 0 marks an empty slot
  long long h = (long long)(mix64(key) & (unsigned long long)mask);
  for (long long p = 0; p <= mask; ++p) {
    const unsigned long long k = __hip_atomic_load(&H[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == key) return h;
    if (k == 0ull) {
      const unsigned long long old = atomicCAS(&H[h].key, 0ull, key);
      if (old == 0ull || old == key) return h;
    }
    h = (h + 1) & mask;
  }
  return -1;
}

__global__ void __launch_bounds__(256) users_load_kernel(CardHeader* H, unsigned long long* fps, long long mask,
                                                         int64_t n, const unsigned long long* key,
                                                         const double* avg, const int* age,
                                                         const unsigned long long* dfp, unsigned* err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long s = find_or_insert(H, mask, key[i]);
  if (s < 0) {
    atomicOr(err, 1u);
    return;
  }
  H[s].avg = avg[i];
  H[s].age = age[i];
  H[s].flags |= 1u;
  for (int f = 0; f < 3; ++f) fps[s * 4 + f] = dfp[i * 3 + f];
}

__global__ void __launch_bounds__(256) feat_assign_kernel(CardHeader* H, long long mask, int64_t n,
                                                          const unsigned long long* key, unsigned epoch,
                                                          unsigned* slot, int* next, unsigned* err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long s = find_or_insert(H, mask, key[i]);
  if (s < 0) {
    atomicOr(err, 1u);
    slot[i] = 0xffffffffu;
    return;
  }
  slot[i] = (unsigned)s;
  const unsigned long long prev =
      atomicExch(&H[s].head, ((unsigned long long)epoch << 32) | (unsigned long long)(unsigned)i);
  next[i] = ((unsigned)(prev >> 32) == epoch) ? (int)(unsigned)(prev & 0xffffffffull) : -1;
}

// Python max(x, lo) / min(x, hi) (feature_processor.py:231-234): NaN propagates like the reference
__device__ __forceinline__ double pmax(double x, double lo) { return (lo > x) ? lo : x; }
__device__ __forceinline__ double pmin(double x, double hi) { return (hi < x) ? hi : x; }
__device__ __forceinline__ float clip10(double x) {
  if (x < -10.0) x = -10.0;
  if (x > 10.0) x = 10.0;
  return (float)x;
}

// bridged raw features -> scoring vector: FeatureProcessor.process_features (41 definitions, derived
// features appended when present) + _prepare_features (pad to 64, clip +-10), then the f32 cast the
// models apply. Mirrors oracle/oracle_features.c orc_vector_from_raw.
__device__ void write_vector(const double* r, float* __restrict__ out) {
#pragma clang fp contract(off)
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
  if (amount > 0) alog = log1p(amount);
  // the 41 definitions in declaration order (feature_processor.py:66-147); built in registers
  // (compile-time indices only) and stored as 16 x 16 B
  float o[FD_VECTOR_WIDTH];
#pragma unroll
  for (int k = 0; k < FD_VECTOR_WIDTH; ++k) o[k] = 0.f;
  o[0] = clip10(amount);
  o[1] = clip10(alog);
  o[5] = clip10(hour);
  o[6] = clip10(dow);
  o[7] = r[4] > 0.5 ? 1.f : 0.f;
  o[12] = 0.5f;
  o[14] = clip10(c1);
  o[15] = clip10(c24);
  o[16] = clip10(s24);
  o[17] = clip10(uavg);
  o[19] = clip10(age);
  o[21] = clip10(mfr);
  o[23] = clip10(mrisk);
  o[24] = 0.5f;
  o[25] = 0.5f;
  o[26] = r[6] > 0.5 ? 1.f : 0.f;
  o[27] = clip10(ip);
  o[31] = clip10(s1);
  o[32] = clip10(c5);
  o[33] = 0.5f;
  o[34] = 0.5f;
  // derived, appended in order when present (feature_processor.py:330-363); merchant_avg_amount is 0 on
  // this path, so there is no amount_to_merchant_avg_ratio
  const bool pres[6] = {amount > 0, uavg > 0, c24 > 0, true, true, true};
  const float dv[6] = {clip10(sqrt(amount)), clip10(amount / uavg), clip10(c1 / (c24 / 24)), clip10((0.5 + ip) / 2),
                       (9 <= hour && hour <= 17) ? 1.f : 0.f, (hour < 6 || hour > 22) ? 1.f : 0.f};
  int k = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    if (pres[i]) {
#pragma unroll
      for (int m = 0; m < 6; ++m)
        if (m == k) o[41 + m] = dv[i];
      ++k;
    }
  }
  float4* o4 = reinterpret_cast<float4*>(out);
#pragma unroll
  for (int q = 0; q < FD_VECTOR_WIDTH / 4; ++q) o4[q] = make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
}

// per-event LSTM input: the bridged raw feature, NaN (null) -> 0, then sign(x) * log1p(|x|) in f64,
// stored f32 (DESIGN.md "LSTM head"). Mirrors oracle/lstm_ref.py event_inputs.
__device__ __forceinline__ float seq_input(double x) {
  if (isnan(x)) return 0.f;
  const double a = log1p(fabs(x));
  return (float)(x < 0 ? -a : a);
}

struct TxnArgs {
  const unsigned long long* key;
  const long long* ts;
  const long long* cents;
  const int* merchant;
  const unsigned long long* dfp;
  const unsigned char* ipc;
  const unsigned char* hour;
  const unsigned char* wk;
};

__global__ void __launch_bounds__(256) feat_process_kernel(CardHeader* H, const unsigned long long* fps,
                                                           RingEvent* ring, const Merchant* merchants, int nm,
                                                           int mode, int K, int64_t n, TxnArgs t,
                                                           const unsigned* slot, const int* next,
                                                           float* __restrict__ vec_out,
                                                           double* __restrict__ raw_out, float* seq_ring,
                                                           int S, float* __restrict__ seq_out,
                                                           double* __restrict__ vel5_out) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned s = slot[i];
  if (s == 0xffffffffu) return;
  CardHeader* h = &H[s];
  if ((unsigned)(h->head & 0xffffffffull) != (unsigned)i) return;  // not this card's owner
  // card state in registers for the whole list
  int cnt = h->cnt, has_ts = h->has_ts, ring_n = h->ring_n, ring_head = h->ring_head;
  long long last_ts = h->last_ts, sum_cents = h->sum_cents;
  unsigned flags = h->flags;
  const bool has_user = (flags & 1u) != 0u;
  int seq_n = (int)((flags >> 8) & 0xffu), seq_head = (int)((flags >> 16) & 0xffu);
  float* sr = S ? seq_ring + (size_t)s * S * kSeqInput : nullptr;
  const double uavg_raw = h->avg;
  const int uage = h->age;
  const unsigned long long fp0 = fps[(size_t)s * 4], fp1 = fps[(size_t)s * 4 + 1], fp2 = fps[(size_t)s * 4 + 2];
  RingEvent* rg = ring + (size_t)s * K;
  int last = -1;
  for (;;) {
    int j = (int)i, best = 0x7fffffff;  // next transaction of this card in arrival order
    while (j >= 0) {
      if (j > last && j < best) best = j;
      j = next[j];
    }
    if (best == 0x7fffffff) break;
    last = best;
    const long long ts = t.ts[best];
    const long long cents = t.cents[best];
    double r[FD_RAW_FEATURES];
    const double amount = (double)cents / 100.0;
    long long days = ts / 86400000LL;
    if (ts % 86400000LL < 0) days -= 1;
    int hour = (int)((ts - days * 86400000LL) / 3600000LL);
    long long dw = (days + 3) % 7;
    if (dw < 0) dw += 7;
    const int dow = (int)dw + 1;
    if (t.hour[best] != 255) hour = t.hour[best];
    const int weekend = (t.wk[best] == 255) ? (dow >= 6) : (t.wk[best] != 0);
    const int m = t.merchant[best];
    double mfr, mult;
    if (m >= 0 && m < nm) {
      const double f = merchants[m].fraud_rate;
      mfr = isnan(f) ? 0.05 : f;
      mult = merchants[m].mult;
    } else {
      mfr = 0.1;
      mult = 2.0;
    }
    const unsigned long long d = t.dfp[best];
    const bool known = has_user && d != 0ull && (d == fp0 || d == fp1 || d == fp2);
    const unsigned char ipc = t.ipc[best];
    r[0] = amount;
    r[1] = (amount + 1 > 0) ? log(amount + 1) : ((amount + 1 == 0) ? -INFINITY : NAN);
    r[2] = hour;
    r[3] = dow;
    r[4] = weekend ? 1.0 : 0.0;
    r[5] = mfr;
    r[6] = known ? 0.0 : 1.0;
    r[7] = ipc == 0 ? NAN : (ipc == 1 ? 0.1 : 0.3);
    r[8] = has_user ? (isnan(uavg_raw) ? 0.0 : uavg_raw) : NAN;
    long long c0 = 0, c1 = 0, c2 = 0, s0 = 0, s1 = 0, s2 = 0;
    if (mode == FD_WINDOW_REDIS_COMPAT) {
      const bool live = has_ts && (ts - last_ts <= 3600000LL);
      const long long cc = live ? cnt : 0, ss = live ? sum_cents : 0;
      c0 = c1 = c2 = cc;
      s0 = s1 = s2 = ss;
      cnt = (int)(cc + 1);
      sum_cents = ss + cents;
      last_ts = ts;
      has_ts = 1;
    } else {
      // 8 events per round trip: the loads of a group are independent (slots past ring_n are read
      // from the allocated ring and ignored)
      for (int e0 = 0; e0 < ring_n; e0 += 8) {
        RingEvent ev[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) ev[u] = rg[min(e0 + u, K - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (e0 + u < ring_n && ev[u].ts <= ts) {
            if (ts - 300000LL < ev[u].ts) {
              c0 += 1;
              s0 += ev[u].cents;
            }
            if (ts - 3600000LL < ev[u].ts) {
              c1 += 1;
              s1 += ev[u].cents;
            }
            if (ts - 86400000LL < ev[u].ts) {
              c2 += 1;
              s2 += ev[u].cents;
            }
          }
        }
      }
      rg[ring_head] = RingEvent{ts, cents};
      ring_head = (ring_head + 1 == K) ? 0 : ring_head + 1;
      if (ring_n < K) ++ring_n;
    }
    r[9] = (double)c0;
    r[10] = (double)c1;
    r[11] = (double)c2;
    r[12] = (double)s1 / 100.0;
    r[13] = (double)s2 / 100.0;
    r[14] = mult;
    r[15] = has_user ? (double)uage : 0.0;
    if (raw_out) {
      double2* ro = reinterpret_cast<double2*>(raw_out + (size_t)best * FD_RAW_FEATURES);
#pragma unroll
      for (int c = 0; c < FD_RAW_FEATURES / 2; ++c) ro[c] = make_double2(r[2 * c], r[2 * c + 1]);
    }
    write_vector(r, vec_out + (size_t)best * FD_VECTOR_WIDTH);
    if (vel5_out) vel5_out[best] = (double)s0 / 100.0;  // velocity_5min_amount (feature map only)
    if (S) {  // LSTM head input: this event appended to the card's history, last S events emitted
      float* slot_ev = sr + (size_t)seq_head * kSeqInput;
#pragma unroll
      for (int c = 0; c < kSeqInput; ++c) slot_ev[c] = seq_input(r[c]);
      seq_head = (seq_head + 1 == S) ? 0 : seq_head + 1;
      if (seq_n < S) ++seq_n;
      if (seq_out) {  // oldest -> newest, left-padded with zero events (Keras pad_sequences 'pre')
        float* so = seq_out + (size_t)best * S * kSeqInput;
        const int pad = S - seq_n;
        for (int q = 0; q < S; ++q) {
          float4* dst = reinterpret_cast<float4*>(so + (size_t)q * kSeqInput);
          if (q < pad) {
            for (int c = 0; c < kSeqInput / 4; ++c) dst[c] = make_float4(0.f, 0.f, 0.f, 0.f);
          } else {
            int src = seq_head - seq_n + (q - pad);
            if (src < 0) src += S;
            const float4* sp = reinterpret_cast<const float4*>(sr + (size_t)src * kSeqInput);
            for (int c = 0; c < kSeqInput / 4; ++c) dst[c] = sp[c];
          }
        }
      }
    }
  }
  h->flags = (flags & 0xffu) | ((unsigned)seq_n << 8) | ((unsigned)seq_head << 16);
  h->cnt = cnt;
  h->has_ts = has_ts;
  h->ring_n = ring_n;
  h->ring_head = ring_head;
  h->last_ts = last_ts;
  h->sum_cents = sum_cents;
}

__global__ void __launch_bounds__(256) count_cards_kernel(const CardHeader* H, int64_t cap,
                                                          unsigned long long* out) {
  unsigned long long c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x)
    c += (H[i].key != 0ull);
  atomicAdd(out, c);
}


// ------------------------------------------------------------------------------------------------
// Full FeatureExtractor map (a3) and the Flink rule scores ((f) rank 2), elementwise per transaction
// after feat_process (same batch: the card slots of feat_assign, the raw features of feat_process).
//   fmap[n][64] f64 in FeatureStore.getRegisteredFeatures order (fl/features/FeatureStore.java:325-365),
//     FeatureExtractor.extractAllFeatures semantics (fl/features/FeatureExtractor.java:50-493): NaN
//     where the Java map has no key; strings as the host's vocabulary codes, "unknown" = 254.
//   rules: FeatureEnrichmentProcessor.calculateFeatureBasedFraudScore + combine + updateRiskLevel
//     (fl/processors/FeatureEnrichmentProcessor.java:80-93,122-367) and TransactionProcessor
//     calculateBasicFeatures + applyFraudDetectionRules + makeFinalDecision (fl/processors/
//     TransactionProcessor.java:143-473, minimal profiles for unknown users/merchants :489-508).
// Declared semantics for the classes the reference is missing (UserProfile, MerchantProfile):
//   DESIGN.md "Feature map". Mirrors oracle/fmap_ref.py.
struct __attribute__((aligned(16))) UserExt {  // 48 B per card slot
  double risk;       // NaN = null
  double weekend;    // behavioral pattern weekend_activity, NaN = absent (-> 0.5)
  double online;     // behavioral pattern online_preference, NaN = absent (-> 0.7)
  double intl;       // international_transactions, NaN = null
  int freq;          // transaction_frequency, -1 = null
  signed char pstart, pend;  // preferred hours, -1 = null
  unsigned char kyc;         // kyc_status code, 255 = null
  unsigned char verified;    // isVerified()
  unsigned char has_patterns;
  unsigned char loaded;
  unsigned char pad[6];
};
static_assert(sizeof(UserExt) == 48, "UserExt must be 48 B");

struct __attribute__((aligned(8))) MerchExt {  // 16 B per merchant
  double avg;  // avg_transaction_amount, NaN = null
  unsigned char risk_level, blacklisted, category, high_risk, open, close, susp_name, loaded;
};
static_assert(sizeof(MerchExt) == 16, "MerchExt must be 16 B");

struct CtxArgs {
  const double* geo_lat;
  const double* geo_lon;
  const double* m_lat;
  const double* m_lon;
  const unsigned char* pay;
  const unsigned char* ttype;
  const unsigned char* ctype;
  const unsigned char* ua;
  const double* fraud_score;
};

constexpr double kUnknownCode = 254.0;

__device__ __forceinline__ double code_or_unknown(unsigned char c) { return c == 255 ? kUnknownCode : (double)c; }

// UTC day of month of a day count since 1970-01-01 (proleptic Gregorian, H. Hinnant's civil_from_days)
__host__ __device__ inline int day_of_month(long long z) {
  z += 719468;
  const long long era = (z >= 0 ? z : z - 146096) / 146097;
  const unsigned doe = (unsigned)(z - era * 146097);
  const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const unsigned mp = (5 * doy + 2) / 153;
  return (int)(doy - (153 * mp + 2) / 5 + 1);
}

// MerchantProfile.isOperatingAtHour (class absent): open <= h < close; unknown hours -> open
__device__ __forceinline__ bool operating_at(const MerchExt& me, int h) {
  if (!me.loaded || me.open == 255 || me.close == 255) return true;
  return h >= (int)me.open && h < (int)me.close;
}

__device__ __forceinline__ double to_rad(double d) { return d * 0.017453292519943295; }  // Math.toRadians

__global__ void __launch_bounds__(256) feat_ext_kernel(const CardHeader* __restrict__ H,
                                                       const unsigned long long* __restrict__ fps,
                                                       const UserExt* __restrict__ uext,
                                                       const Merchant* __restrict__ merchants,
                                                       const MerchExt* __restrict__ mext, int nm, int n_mext,
                                                       int64_t n,
                                                       TxnArgs t, CtxArgs c, const unsigned* __restrict__ slot,
                                                       const double* __restrict__ raw, const double* __restrict__ vel5,
                                                       const unsigned char* __restrict__ vocab, double tp_threshold,
                                                       double* __restrict__ fmap, fd_rule_scores* __restrict__ rules) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* r = raw + (size_t)i * FD_RAW_FEATURES;
  const unsigned s = slot[i];
  const bool has_slot = s != 0xffffffffu;
  const CardHeader h = has_slot ? H[s] : CardHeader{};
  const bool has_user = has_slot && (h.flags & 1u) != 0u;
  UserExt ue{};
  if (has_user && uext != nullptr) ue = uext[s];
  if (!ue.loaded) {
    ue.risk = ue.weekend = ue.online = ue.intl = __builtin_nan("");
    ue.freq = -1;
    ue.pstart = ue.pend = -1;
    ue.kyc = 255;
    ue.verified = 0;
    ue.has_patterns = 0;
  }
  const int m = t.merchant[i];
  const bool has_merch = m >= 0 && m < nm;
  MerchExt me{};
  if (has_merch && mext != nullptr && m < n_mext) me = mext[m];
  if (!me.loaded) {
    me.avg = __builtin_nan("");
    me.risk_level = me.blacklisted = me.category = me.susp_name = me.open = me.close = 255;
    me.high_risk = 0;
  }
  const double mfr_raw = has_merch ? merchants[m].fraud_rate : __builtin_nan("");  // NaN = null
  const long long cents = t.cents[i];
  const double amount = r[0];
  const int hour = (int)r[2];
  const unsigned char hour_field = t.hour[i];  // Transaction.hourOfDay (255 = null)
  const int age = h.age;                        // loaded profile: account_age_days (< 0 = null)
  const bool age_known = has_user && age >= 0;
  const double uavg = h.avg;                    // NaN = null
  const bool known_device = r[6] < 0.5;
  const double nan = __builtin_nan("");
  double f[FD_FEATURE_MAP_WIDTH];
#pragma unroll
  for (int k = 0; k < FD_FEATURE_MAP_WIDTH; ++k) f[k] = nan;

  // amount (12) FeatureExtractor.java:92-129
  f[0] = amount;
  f[1] = r[1];
  f[2] = sqrt(amount);
  f[3] = (cents % 100 == 0) ? 1.0 : 0.0;
  f[4] = (cents % 1000 == 0) ? 1.0 : 0.0;
  f[5] = (cents % 10000 == 0) ? 1.0 : 0.0;
  if (has_user && !isnan(uavg) && uavg > 0) {
    const double ratio = amount / uavg;
    f[6] = ratio;
    f[7] = (amount - uavg) / uavg;
    f[8] = ratio > 3.0 ? 1.0 : 0.0;
  }
  if (has_merch && !isnan(me.avg) && me.avg > 0) {
    f[9] = amount / me.avg;
    f[10] = amount > me.avg * 2.0 ? 1.0 : 0.0;
  }
  f[11] = amount < 10 ? 0.0 : amount < 100 ? 1.0 : amount < 1000 ? 2.0 : amount < 10000 ? 3.0 : 4.0;
  // temporal (8) :134-165
  f[12] = (double)hour;
  f[13] = r[3];
  long long days = t.ts[i] / 86400000LL;
  if (t.ts[i] % 86400000LL < 0) days -= 1;
  f[14] = (double)day_of_month(days);
  f[15] = r[4];
  f[16] = (hour >= 6 && hour < 12) ? 0.0 : (hour >= 12 && hour < 18) ? 1.0 : (hour >= 18 && hour < 22) ? 2.0 : 3.0;
  f[17] = (hour >= 9 && hour <= 17) ? 1.0 : 0.0;
  f[18] = (hour <= 6 || hour >= 22) ? 1.0 : 0.0;
  if (has_user && ue.pstart >= 0 && ue.pend >= 0) f[19] = (hour >= ue.pstart && hour <= ue.pend) ? 1.0 : 0.0;
  // geographic (8) :170-205
  const double glat = c.geo_lat ? c.geo_lat[i] : nan, glon = c.geo_lon ? c.geo_lon[i] : nan;
  const double mlat = c.m_lat ? c.m_lat[i] : nan, mlon = c.m_lon ? c.m_lon[i] : nan;
  f[20] = (!isnan(glat) || !isnan(glon)) ? 1.0 : 0.0;
  f[21] = (!isnan(mlat) || !isnan(mlon)) ? 1.0 : 0.0;
  if (!isnan(glat) && !isnan(glon)) {
    f[22] = glat;
    f[23] = glon;
    f[24] = (fabs(glat) > 60 || (fabs(glat) < 10 && fabs(glon) < 10)) ? 1.0 : 0.0;
    if (!isnan(mlat) && !isnan(mlon)) {
      const double dLat = to_rad(mlat - glat), dLon = to_rad(mlon - glon);
      const double a = sin(dLat / 2) * sin(dLat / 2) +
                       cos(to_rad(glat)) * cos(to_rad(mlat)) * sin(dLon / 2) * sin(dLon / 2);
      f[25] = 6371 * (2 * atan2(sqrt(a), sqrt(1 - a)));
    }
  }
  if (has_user && !isnan(ue.intl)) {
    f[26] = ue.intl;
    f[27] = ue.intl < 0.1 ? 1.0 : 0.0;
  }
  // user behaviour (10) :210-250
  if (has_user) {
    f[28] = age_known ? (double)age : 0.0;
    f[29] = (age_known && age < 30) ? 1.0 : 0.0;
    f[30] = (age_known && age < 7) ? 1.0 : 0.0;
    f[31] = isnan(ue.risk) ? 0.5 : ue.risk;
    f[32] = ue.verified ? 1.0 : 0.0;
    f[33] = code_or_unknown(ue.kyc);
    if (ue.has_patterns) {
      f[34] = isnan(ue.weekend) ? 0.5 : ue.weekend;
      f[35] = isnan(ue.online) ? 0.7 : ue.online;
    }
    f[36] = isnan(uavg) ? 0.0 : uavg;
    f[37] = ue.freq >= 0 ? (double)ue.freq : 0.0;
  } else {
    f[28] = 0.0;
    f[29] = 1.0;
    f[30] = 1.0;
    f[31] = 0.8;
    f[32] = 0.0;
    f[33] = kUnknownCode;
  }
  // merchant risk (8) :255-296
  if (has_merch) {
    f[38] = code_or_unknown(me.risk_level);
    f[39] = isnan(mfr_raw) ? 0.05 : mfr_raw;
    f[40] = me.blacklisted == 1 ? 1.0 : 0.0;
    f[41] = code_or_unknown(me.category);
    f[42] = me.high_risk ? 1.0 : 0.0;
    if (hour_field != 255) f[43] = operating_at(me, hour_field) ? 1.0 : 0.0;
    f[44] = r[14];
    if (me.susp_name != 255) f[45] = me.susp_name ? 1.0 : 0.0;
  } else {
    f[38] = kUnknownCode;
    f[39] = 0.1;
    f[40] = 0.0;
    f[41] = kUnknownCode;
    f[42] = 0.0;
    f[44] = 2.0;
  }
  // device / network (5) :301-324
  f[46] = known_device ? 1.0 : 0.0;
  f[47] = known_device ? 0.0 : 1.0;
  if (t.ipc[i] != 0) {
    f[48] = t.ipc[i] == 1 ? 1.0 : 0.0;
    f[49] = r[7];
  }
  const unsigned char ua = c.ua ? c.ua[i] : 255;
  if (ua != 255) f[50] = ua ? 1.0 : 0.0;
  // velocity (8) :329-363
  f[51] = r[9];
  f[52] = vel5[i];
  f[53] = r[10];
  f[54] = r[12];
  f[55] = r[11];
  f[56] = r[13];
  f[57] = r[9] > 5 ? 1.0 : 0.0;
  f[58] = r[10] > 20 ? 1.0 : 0.0;
  // contextual (5) :368-382
  const unsigned char pay = c.pay ? c.pay[i] : 255, tt = c.ttype ? c.ttype[i] : 255, ct = c.ctype ? c.ctype[i] : 255;
  f[59] = code_or_unknown(pay);
  f[60] = (pay != 255 && vocab[pay]) ? 1.0 : 0.0;
  f[61] = code_or_unknown(tt);
  f[62] = (tt != 255 && vocab[256 + tt]) ? 1.0 : 0.0;
  f[63] = code_or_unknown(ct);
  if (fmap) {
    double2* o = reinterpret_cast<double2*>(fmap + (size_t)i * FD_FEATURE_MAP_WIDTH);
#pragma unroll
    for (int k = 0; k < FD_FEATURE_MAP_WIDTH / 2; ++k) o[k] = make_double2(f[2 * k], f[2 * k + 1]);
  }
  if (!rules) return;

  // FeatureEnrichmentProcessor.calculateFeatureBasedFraudScore (:122-336), present() = key in the map
  auto is_true = [&](int k) { return !isnan(f[k]) && f[k] != 0.0; };
  auto is_false = [&](int k) { return !isnan(f[k]) && f[k] == 0.0; };
  double sa = 0.0;
  if (is_true(8)) sa += 0.3;
  if (is_true(5)) sa += 0.1;
  if (f[11] == 4.0) sa += 0.2;
  else if (f[11] == 0.0) sa += 0.1;
  double stt = 0.0;
  if (is_true(18)) stt += 0.2;
  if (is_false(19)) stt += 0.15;
  if (is_true(15) && !isnan(f[34]) && f[34] < 0.3) stt += 0.1;
  double su = 0.0;
  if (is_true(30)) su += 0.4;
  else if (is_true(29)) su += 0.2;
  if (is_false(32)) su += 0.3;
  if (!isnan(f[31])) su += f[31] * 0.5;
  double sm = 0.0;
  if (is_true(40)) sm += 0.8;
  if (is_true(42)) sm += 0.3;
  if (!isnan(f[39])) sm += f[39] * 2.0;
  if (is_true(45)) sm += 0.2;
  if (is_false(43)) sm += 0.15;
  double sv = 0.0;
  if (is_true(57)) sv += 0.6;
  if (is_true(58)) sv += 0.4;
  if (f[51] > 3) sv += 0.2;
  if (f[53] > 10) sv += 0.15;
  double sd = 0.0;
  if (is_true(47)) sd += 0.3;
  if (!isnan(f[49])) sd += f[49];
  if (is_true(50)) sd += 0.2;
  double fb = 0.0;
  fb += sa * 0.2;
  fb += stt * 0.1;
  fb += su * 0.25;
  fb += sm * 0.2;
  fb += sv * 0.15;
  fb += sd * 0.1;
  fb = fmax(0.0, fmin(1.0, fb));
  const double existing = c.fraud_score ? c.fraud_score[i] : nan;
  const double fe = isnan(existing) ? fb : fmax(0.0, fmin(1.0, (existing * 0.6) + (fb * 0.4)));
  fd_rule_scores out{};
  out.fe_score = fe;
  // updateRiskLevel (:341-367)
  out.fe_risk = fe >= 0.95 ? FD_CRITICAL : fe >= 0.8 ? FD_HIGH : fe >= 0.6 ? FD_MEDIUM : fe >= 0.3 ? FD_LOW : FD_VERY_LOW;
  out.fe_decision = fe >= 0.95 ? FD_DECLINE : fe >= 0.6 ? FD_REVIEW : FD_APPROVE;

  // TransactionProcessor (:143-473): unknown user / merchant get the minimal profiles (:489-508)
  const double urisk = has_user ? ue.risk : 0.5;
  const bool verified = has_user ? (ue.verified != 0) : false;  // minimal profile: kyc "pending"
  double pu = 0.0;
  if (!isnan(urisk)) pu += urisk * 0.2;
  if (age_known && age < 30) pu += 0.1;  // UserProfile.isNewAccount (class absent): age < 30 days
  if (!verified) pu += 0.15;
  const unsigned char rl = has_merch ? me.risk_level : 1;  // minimal merchant: "medium"
  const bool blacklisted = has_merch && me.blacklisted == 1;
  const double fr = has_merch ? mfr_raw : 0.05;
  double pm = 0.0;
  if (rl == 2) pm += 0.2;
  else if (rl == 1) pm += 0.1;
  if (blacklisted) pm += 0.4;
  if (!isnan(fr) && fr > 0.05) pm += fr * 2.0;
  if (has_merch && me.high_risk) pm += 0.15;
  double pf = 0.0;
  if (has_user && !isnan(uavg) && uavg > 0 && amount / uavg > 5.0) pf += 0.15;  // large_amount_flag
  if (has_user && t.dfp[i] != 0ull && !known_device) pf += 0.1;                   // new_device_flag
  if (hour_field != 255 && (hour_field <= 5 || hour_field >= 23)) pf += 0.05;     // unusual_hour_flag
  if (hour_field != 255 && !operating_at(me, hour_field)) pf += 0.1;              // within_operating_hours
  double tp = 0.0;
  if (!isnan(existing)) tp = existing * 0.5;
  tp += pu;
  tp += pm;
  tp += pf;
  tp = fmax(0.0, fmin(1.0, tp));
  out.tp_score = tp;
  unsigned char dec, risk;
  if (tp >= 0.9) {
    dec = FD_DECLINE;
    risk = FD_CRITICAL;
  } else if (tp >= tp_threshold) {
    dec = FD_REVIEW;
    risk = FD_HIGH;
  } else if (tp >= 0.5) {
    dec = FD_APPROVE;
    risk = FD_MEDIUM;
  } else {
    dec = FD_APPROVE;
    risk = FD_LOW;
  }
  if (blacklisted) {
    dec = FD_DECLINE;
    risk = FD_CRITICAL;
  }
  out.tp_decision = dec;
  out.tp_risk = risk;
  rules[i] = out;
}

__global__ void __launch_bounds__(256) users_ext_load_kernel(CardHeader* H, UserExt* U, long long mask, int64_t n,
                                                             const unsigned long long* key, const UserExt* src,
                                                             unsigned* err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long s = find_or_insert(H, mask, key[i]);
  if (s < 0) {
    atomicOr(err, 1u);
    return;
  }
  UserExt u = src[i];
  u.loaded = 1;
  U[s] = u;
}

unsigned grid_for(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

void state_init(Engine& e, const fd_state_params& p) {
  FD_REQUIRE(p.capacity > 0 && p.capacity <= (1ll << 31), FD_ERR_INVALID_ARG, "capacity must be in [1, 2^31]");
  FD_REQUIRE(p.window_mode == FD_WINDOW_REDIS_COMPAT || p.window_mode == FD_WINDOW_SLIDING, FD_ERR_INVALID_ARG,
             "unknown window_mode");
  FD_REQUIRE(p.ring_k >= 1 && p.ring_k <= 64, FD_ERR_INVALID_ARG, "ring_k must be in [1, 64]");
  FD_REQUIRE(p.seq_len >= 0 && p.seq_len <= FD_MAX_SEQ_LEN, FD_ERR_INVALID_ARG, "seq_len must be in [0, 16]");
  int64_t cap = 1;
  while (cap < p.capacity) cap <<= 1;
  CardStore& st = e.state;
  st.cap = cap;
  st.mode = p.window_mode;
  st.K = p.window_mode == FD_WINDOW_SLIDING ? p.ring_k : 1;
  st.headers.ensure((size_t)cap * sizeof(CardHeader));
  st.fps.ensure((size_t)cap * 4 * sizeof(unsigned long long));
  st.ring.ensure((size_t)cap * st.K * sizeof(RingEvent));
  st.S = p.seq_len;
  if (st.S) st.seq.ensure((size_t)cap * st.S * kSeqInput * sizeof(float));
  // extended user profiles are per slot: a re-initialised table starts without them (fd_state_load_users_ext
  // allocates for the new capacity)
  st.uext.release();
  st.err.ensure(16);
  st.ready = true;
  state_clear(e);
}

void state_clear(Engine& e) {
  CardStore& st = e.state;
  FD_REQUIRE(st.ready, FD_ERR_NOT_LOADED, "card state not initialised (fd_state_init)");
  FD_HIP(hipMemsetAsync(st.headers.ptr, 0, (size_t)st.cap * sizeof(CardHeader), e.stream));
  FD_HIP(hipMemsetAsync(st.fps.ptr, 0, (size_t)st.cap * 4 * sizeof(unsigned long long), e.stream));
  if (st.uext.ptr) FD_HIP(hipMemsetAsync(st.uext.ptr, 0, (size_t)st.cap * sizeof(UserExt), e.stream));
  FD_HIP(hipMemsetAsync(st.err.ptr, 0, 16, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  st.epoch = 0;
  // the window event logs hold card-table slots: clearing the table empties them too
  WindowState& w = e.windows;
  w.ucount = w.mcount = 0;
  w.wm = INT64_MIN;
  w.min_seen = INT64_MAX;
  w.max_seen = INT64_MIN;
}

int64_t state_count(Engine& e) {
  CardStore& st = e.state;
  FD_REQUIRE(st.ready, FD_ERR_NOT_LOADED, "card state not initialised (fd_state_init)");
  DeviceBuffer tmp;
  tmp.ensure(8);
  FD_HIP(hipMemsetAsync(tmp.ptr, 0, 8, e.stream));
  hipLaunchKernelGGL(count_cards_kernel, dim3(1024), dim3(256), 0, e.stream, st.headers.as<const CardHeader>(),
                     st.cap, tmp.as<unsigned long long>());
  FD_HIP(hipGetLastError());
  unsigned long long c = 0;
  FD_HIP(hipMemcpyAsync(&c, tmp.ptr, 8, hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  tmp.release();
  return (int64_t)c;
}

static void check_err(Engine& e) {
  unsigned v = 0;
  FD_HIP(hipMemcpyAsync(&v, e.state.err.ptr, 4, hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  if (v) {
    FD_HIP(hipMemsetAsync(e.state.err.ptr, 0, 4, e.stream));
    throw Error(FD_ERR_OOM, "card table full: raise fd_state_params.capacity");
  }
}

void load_users(Engine& e, const fd_users& u) {
  CardStore& st = e.state;
  FD_REQUIRE(st.ready, FD_ERR_NOT_LOADED, "card state not initialised (fd_state_init)");
  FD_REQUIRE(u.n >= 0 && (u.n == 0 || (u.key && u.avg_amount && u.account_age_days && u.device_fp)),
             FD_ERR_INVALID_ARG, "incomplete user arrays");
  if (u.n == 0) return;
  DeviceBuffer k, a, g, f;
  k.ensure(u.n * 8);
  a.ensure(u.n * 8);
  g.ensure(u.n * 4);
  f.ensure(u.n * 24);
  FD_HIP(hipMemcpyAsync(k.ptr, u.key, u.n * 8, hipMemcpyHostToDevice, e.stream));
  FD_HIP(hipMemcpyAsync(a.ptr, u.avg_amount, u.n * 8, hipMemcpyHostToDevice, e.stream));
  FD_HIP(hipMemcpyAsync(g.ptr, u.account_age_days, u.n * 4, hipMemcpyHostToDevice, e.stream));
  FD_HIP(hipMemcpyAsync(f.ptr, u.device_fp, u.n * 24, hipMemcpyHostToDevice, e.stream));
  hipLaunchKernelGGL(users_load_kernel, dim3(grid_for(u.n)), dim3(256), 0, e.stream, st.headers.as<CardHeader>(),
                     st.fps.as<unsigned long long>(), (long long)(st.cap - 1), u.n, k.as<const unsigned long long>(),
                     a.as<const double>(), g.as<const int>(), f.as<const unsigned long long>(), st.err.as<unsigned>());
  FD_HIP(hipGetLastError());
  check_err(e);  // synchronises before the staging buffers are freed
}

void load_merchants(Engine& e, const fd_merchants& m) {
  CardStore& st = e.state;
  FD_REQUIRE(m.n >= 0 && (m.n == 0 || (m.fraud_rate && m.risk_multiplier)), FD_ERR_INVALID_ARG,
             "incomplete merchant arrays");
  std::vector<Merchant> h((size_t)m.n);
  for (int64_t i = 0; i < m.n; ++i) h[i] = Merchant{m.fraud_rate[i], m.risk_multiplier[i]};
  st.merchants.ensure(std::max<size_t>(16, h.size() * sizeof(Merchant)));
  if (m.n) FD_HIP(hipMemcpy(st.merchants.ptr, h.data(), h.size() * sizeof(Merchant), hipMemcpyHostToDevice));
  st.n_merchants = m.n;
}

void launch_features(Engine& e, const fd_txn_batch& t, int64_t n, float* d_vec, double* d_raw, float* d_seq,
                     double* d_vel5) {
  CardStore& st = e.state;
  FD_REQUIRE(st.ready, FD_ERR_NOT_LOADED, "card state not initialised (fd_state_init)");
  FD_REQUIRE(d_vec != nullptr, FD_ERR_INVALID_ARG, "null vector output");
  FD_REQUIRE(d_seq == nullptr || st.S > 0, FD_ERR_INVALID_ARG, "sequence output needs fd_state_params.seq_len > 0");
  FD_REQUIRE(n >= 0 && n < (1ll << 31), FD_ERR_INVALID_ARG, "batch size out of range");
  if (n == 0) return;
  FD_REQUIRE(t.card_key && t.ts_ms && t.amount_cents && t.merchant && t.device_fp && t.ip_class && t.hour &&
                 t.weekend,
             FD_ERR_INVALID_ARG, "incomplete transaction batch");
  st.slot.ensure((size_t)n * 4);
  st.next.ensure((size_t)n * 4);
  if (st.merchants.ptr == nullptr) st.merchants.ensure(16);
  st.epoch = (st.epoch == 0xffffffffu) ? 1u : st.epoch + 1u;
  Engine::Timed* ev = e.timing ? e.next_event_pair(FD_TIMING_FEATURES) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, e.stream));
  hipLaunchKernelGGL(feat_assign_kernel, dim3(grid_for(n)), dim3(256), 0, e.stream, st.headers.as<CardHeader>(),
                     (long long)(st.cap - 1), n, reinterpret_cast<const unsigned long long*>(t.card_key), st.epoch,
                     st.slot.as<unsigned>(), st.next.as<int>(), st.err.as<unsigned>());
  FD_HIP(hipGetLastError());
  TxnArgs a{reinterpret_cast<const unsigned long long*>(t.card_key), reinterpret_cast<const long long*>(t.ts_ms),
            reinterpret_cast<const long long*>(t.amount_cents), reinterpret_cast<const int*>(t.merchant),
            reinterpret_cast<const unsigned long long*>(t.device_fp), t.ip_class, t.hour, t.weekend};
  hipLaunchKernelGGL(feat_process_kernel, dim3(grid_for(n)), dim3(256), 0, e.stream, st.headers.as<CardHeader>(),
                     st.fps.as<const unsigned long long>(), st.ring.as<RingEvent>(), st.merchants.as<const Merchant>(),
                     (int)st.n_merchants, st.mode, st.K, n, a, st.slot.as<const unsigned>(), st.next.as<const int>(),
                     d_vec, d_raw, st.S ? st.seq.as<float>() : nullptr, st.S, d_seq, d_vel5);
  FD_HIP(hipGetLastError());
  if (ev) FD_HIP(hipEventRecord(ev->b, e.stream));
}

void features_check(Engine& e) { check_err(e); }

void load_users_ext(Engine& e, const fd_users_ext& u) {
  CardStore& st = e.state;
  FD_REQUIRE(st.ready, FD_ERR_NOT_LOADED, "card state not initialised (fd_state_init)");
  FD_REQUIRE(u.n >= 0 && (u.n == 0 || u.key), FD_ERR_INVALID_ARG, "null user keys");
  if (!st.uext.ptr) {
    st.uext.ensure((size_t)st.cap * sizeof(UserExt));
    FD_HIP(hipMemsetAsync(st.uext.ptr, 0, (size_t)st.cap * sizeof(UserExt), e.stream));
  }
  if (u.n == 0) return;
  std::vector<UserExt> h((size_t)u.n);
  for (int64_t i = 0; i < u.n; ++i) {
    UserExt x{};
    x.risk = u.risk_score ? u.risk_score[i] : NAN;
    x.weekend = u.weekend_activity ? u.weekend_activity[i] : NAN;
    x.online = u.online_preference ? u.online_preference[i] : NAN;
    x.intl = u.intl_preference ? u.intl_preference[i] : NAN;
    x.freq = u.txn_frequency ? u.txn_frequency[i] : -1;
    x.pstart = u.pref_start ? u.pref_start[i] : (signed char)-1;
    x.pend = u.pref_end ? u.pref_end[i] : (signed char)-1;
    x.kyc = u.kyc_status ? u.kyc_status[i] : 255;
    x.verified = u.verified ? (u.verified[i] != 0) : 0;
    x.has_patterns = u.has_patterns ? (u.has_patterns[i] != 0) : 0;
    h[i] = x;
  }
  DeviceBuffer k, d;
  k.ensure(u.n * 8);
  d.ensure(h.size() * sizeof(UserExt));
  FD_HIP(hipMemcpyAsync(k.ptr, u.key, u.n * 8, hipMemcpyHostToDevice, e.stream));
  FD_HIP(hipMemcpyAsync(d.ptr, h.data(), h.size() * sizeof(UserExt), hipMemcpyHostToDevice, e.stream));
  hipLaunchKernelGGL(users_ext_load_kernel, dim3(grid_for(u.n)), dim3(256), 0, e.stream, st.headers.as<CardHeader>(),
                     st.uext.as<UserExt>(), (long long)(st.cap - 1), u.n, k.as<const unsigned long long>(),
                     d.as<const UserExt>(), st.err.as<unsigned>());
  FD_HIP(hipGetLastError());
  check_err(e);  // synchronises before the staging buffers are freed
}

void load_merchants_ext(Engine& e, const fd_merchants_ext& m) {
  CardStore& st = e.state;
  FD_REQUIRE(m.n >= 0, FD_ERR_INVALID_ARG, "bad merchant count");
  std::vector<MerchExt> h((size_t)std::max<int64_t>(m.n, 1));
  for (int64_t i = 0; i < m.n; ++i) {
    MerchExt x{};
    x.avg = m.avg_amount ? m.avg_amount[i] : NAN;
    x.risk_level = m.risk_level ? m.risk_level[i] : 255;
    x.blacklisted = m.blacklisted ? m.blacklisted[i] : 255;
    x.category = m.category ? m.category[i] : 255;
    x.high_risk = m.high_risk_category ? (m.high_risk_category[i] != 0) : 0;
    x.open = m.open_hour ? m.open_hour[i] : 255;
    x.close = m.close_hour ? m.close_hour[i] : 255;
    x.susp_name = m.suspicious_name ? m.suspicious_name[i] : 255;
    x.loaded = 1;
    h[i] = x;
  }
  st.mext.ensure(h.size() * sizeof(MerchExt));
  FD_HIP(hipMemcpy(st.mext.ptr, h.data(), h.size() * sizeof(MerchExt), hipMemcpyHostToDevice));
  st.n_mext = m.n;
}

void load_vocab(Engine& e, const uint8_t* pay_high_risk, const uint8_t* type_refund) {
  CardStore& st = e.state;
  uint8_t h[512] = {};
  for (int i = 0; i < 256; ++i) {
    h[i] = pay_high_risk ? (pay_high_risk[i] != 0) : 0;
    h[256 + i] = type_refund ? (type_refund[i] != 0) : 0;
  }
  st.vocab.ensure(512);
  FD_HIP(hipMemcpy(st.vocab.ptr, h, 512, hipMemcpyHostToDevice));
  st.vocab_loaded = true;
}

// features + vectors (launch_features) then the feature map / rule scores of the same batch
void launch_features_full(Engine& e, const fd_txn_batch& t, const fd_txn_context& c, int64_t n, float* d_vec,
                          double* d_raw, double* d_fmap, fd_rule_scores* d_rules) {
  CardStore& st = e.state;
  FD_REQUIRE(st.ready, FD_ERR_NOT_LOADED, "card state not initialised (fd_state_init)");
  FD_REQUIRE(d_vec != nullptr, FD_ERR_INVALID_ARG, "null vector output");
  if (n <= 0) return;
  const size_t rawb = d_raw ? 0 : (size_t)n * FD_RAW_FEATURES * 8;
  e.feat_ext.ensure(rawb + (size_t)n * 8);
  double* raw = d_raw ? d_raw : e.feat_ext.as<double>();
  double* vel5 = reinterpret_cast<double*>(e.feat_ext.as<char>() + rawb);
  launch_features(e, t, n, d_vec, raw, nullptr, vel5);
  if (!st.vocab_loaded) load_vocab(e, nullptr, nullptr);
  if (st.merchants.ptr == nullptr) st.merchants.ensure(16);
  TxnArgs a{reinterpret_cast<const unsigned long long*>(t.card_key), reinterpret_cast<const long long*>(t.ts_ms),
            reinterpret_cast<const long long*>(t.amount_cents), reinterpret_cast<const int*>(t.merchant),
            reinterpret_cast<const unsigned long long*>(t.device_fp), t.ip_class, t.hour, t.weekend};
  CtxArgs ca{c.geo_lat, c.geo_lon, c.merchant_lat, c.merchant_lon, c.payment_method, c.transaction_type,
             c.card_type, c.user_agent_flag, c.fraud_score};
  hipLaunchKernelGGL(feat_ext_kernel, dim3(grid_for(n)), dim3(256), 0, e.stream, st.headers.as<const CardHeader>(),
                     st.fps.as<const unsigned long long>(), st.uext.ptr ? st.uext.as<const UserExt>() : nullptr,
                     st.merchants.as<const Merchant>(), st.mext.ptr ? st.mext.as<const MerchExt>() : nullptr,
                     (int)st.n_merchants, (int)st.n_mext, n, a, ca,
                     st.slot.as<const unsigned>(), raw, vel5, st.vocab.as<const unsigned char>(), st.tp_threshold,
                     d_fmap, d_rules);
  FD_HIP(hipGetLastError());
}

}  // namespace fd
