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
                                                           int S, float* __restrict__ seq_out) {
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
    long long c0 = 0, c1 = 0, c2 = 0, s1 = 0, s2 = 0;
    if (mode == FD_WINDOW_REDIS_COMPAT) {
      const bool live = has_ts && (ts - last_ts <= 3600000LL);
      const long long cc = live ? cnt : 0, ss = live ? sum_cents : 0;
      c0 = c1 = c2 = cc;
      s1 = s2 = ss;
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
            if (ts - 300000LL < ev[u].ts) c0 += 1;
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
  st.err.ensure(16);
  st.ready = true;
  state_clear(e);
}

void state_clear(Engine& e) {
  CardStore& st = e.state;
  FD_REQUIRE(st.ready, FD_ERR_NOT_LOADED, "card state not initialised (fd_state_init)");
  FD_HIP(hipMemsetAsync(st.headers.ptr, 0, (size_t)st.cap * sizeof(CardHeader), e.stream));
  FD_HIP(hipMemsetAsync(st.fps.ptr, 0, (size_t)st.cap * 4 * sizeof(unsigned long long), e.stream));
  FD_HIP(hipMemsetAsync(st.err.ptr, 0, 16, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  st.epoch = 0;
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

void launch_features(Engine& e, const fd_txn_batch& t, int64_t n, float* d_vec, double* d_raw, float* d_seq) {
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
                     d_vec, d_raw, st.S ? st.seq.as<float>() : nullptr, st.S, d_seq);
  FD_HIP(hipGetLastError());
  if (ev) FD_HIP(hipEventRecord(ev->b, e.stream));
}

void features_check(Engine& e) { check_err(e); }

}  // namespace fd
