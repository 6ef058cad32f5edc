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
// processed in arrival order, each reading the card's velocity before writing it. The batch is
// sorted and segmented by card (two launches, no per-batch table reset):
//   feat_slot    : per txn, find-or-insert the card slot (open addressing, atomicCAS on the key), write its
//                  48-B prep record (fields + the merchant row already joined) and append its
//                  (slot << 32 | arrival index) key to its bucket's fixed-capacity region (bucket = slot mod
//                  NB, NB ~ n / 128; per block an LDS histogram and one global atomic per bucket; a bucket
//                  past its capacity spills to an overflow list its bucket kernel scans);
//   feat_bucket  : one workgroup per bucket: the bucket's keys sorted in LDS (rank counting up to 512 keys,
//                  bitonic beyond) -> segments = cards in arrival order. Segments of <= kSegLong transactions:
//                  one thread walks the card with its 128-B header in registers; longer ones (hot cards,
//                  card-testing bursts): the whole workgroup, 256 transactions per tile, each thread computing
//                  its transaction's windows from an LDS tile of the card's previous K events (positional
//                  form of the sequential definition) and the redis_compat session by a workgroup scan.
// Sliding windows are incremental: per window the header keeps how many of the ring's newest events are
// inside it, their cents sum and the oldest one's time, so a transaction reads ring events only to evict
// them (canonical state: the windows as of the card's last event). A ring that is not time-sorted (an
// out-of-order arrival) is scanned in full until the out-of-order event has left it (`unsorted` counts
// the appends left), then the windows are rebuilt. Both forms equal oracle/oracle_features.c exactly.
// Velocity sums are integer cents (exact); amounts leave as cents/100.0 (f64, correctly rounded).
#include <cmath>
#include <cstring>

#include "fd_internal.h"

namespace fd {
namespace {

constexpr long long kWin[3] = {300000LL, 3600000LL, 86400000LL};  // 5 min / 1 h / 24 h
constexpr long long kSessionTtl = 3600000LL;                      // RedisService TTL 3600 s (ms)
constexpr int kBT = 256;          // threads of the bucket kernel (and its scans)
constexpr int kST = 256;          // threads of the slot kernel (latency-bound probes: spread over every CU)
constexpr int kSegLong = 16;      // segments longer than this take the cooperative path
constexpr int kChunkCap = 4096;   // (slot, txn) keys sorted per pass in LDS
static_assert(kChunkCap == kGatherBatchMax, "the pipelined step picks the gather kernel by kGatherBatchMax");
constexpr int kMaxBuckets = 4096;
constexpr int kMaxBins = 4096;    // arrival-range bins of an oversized bucket
constexpr int kMaxK = 64;
constexpr size_t kBucketLds = (size_t)kChunkCap * 8 + (size_t)(kMaxBins + 1) * 4;  // keys | bin prefix sums

#ifdef FD_FOREST_PROFILE
// Phase stamps of the bucket kernel (profiling build only): per workgroup b < 4096 {start, keys loaded,
// sorted, short segments done (workgroup barrier), end} plus each wave's own end of the short loop.
__device__ unsigned long long g_fprof[4096 * 8];
__device__ unsigned long long g_fprof2[4096 * 4];  // thread 0's first card: header + prep in, ring done, emitted
#define FD_CSTAMP(k)                                                                                   \
  do {                                                                                                 \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_fprof2[blockIdx.x * 4 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
FD_TL_BUF(g_tl_feat);
#define FD_FSTAMP(k)                                                                              \
  do {                                                                                            \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_fprof[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define FD_FSTAMP(k)
#define FD_CSTAMP(k)
#endif

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


__global__ void __launch_bounds__(256) users_load_kernel(CardPages P, unsigned long long* K, long long mask, int64_t n,
                                                         const unsigned long long* key, const double* avg,
                                                         const int* age, const unsigned long long* dfp,
                                                         unsigned* err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long s = card_slot(K, P, mask, key[i]);
  if (s < 0) {
    atomicOr(err, 1u);
    return;
  }
  CardHeader* h = P.hdr(s);
  h->avg = avg[i];
  h->age = age[i];
  h->flags |= 1u;
  for (int f = 0; f < 3; ++f) h->fp[f] = dfp[i * 3 + f];
}

// ------------------------------------------------------------------------------------------------
// transaction sources: the SoA batch (fd_txn_batch) or received 48-B route records (route.hip)
struct Txn {
  long long ts, cents;
  unsigned long long dfp;
  int merchant;
  unsigned char ipc, hour, wk;
};

struct TxnSrc {
  const unsigned long long* key;
  const long long* ts;
  const long long* cents;
  const int* merchant;
  const unsigned long long* dfp;
  const unsigned char* ipc;
  const unsigned char* hour;
  const unsigned char* wk;
  const RouteRecord* rec;  // non-null: every field comes from the records
  __device__ __forceinline__ unsigned long long get_key(int64_t i) const { return rec ? rec[i].key : key[i]; }
  __device__ __forceinline__ Txn get(int64_t i) const {
    Txn t;
    if (rec) {
      const RouteRecord r = rec[i];
      t.ts = r.ts;
      t.cents = r.cents;
      t.dfp = r.dfp;
      t.merchant = r.merchant;
      t.ipc = r.ipc;
      t.hour = r.hour;
      t.wk = r.wk;
    } else {
      t.ts = ts[i];
      t.cents = cents[i];
      t.dfp = dfp[i];
      t.merchant = merchant[i];
      t.ipc = ipc[i];
      t.hour = hour[i];
      t.wk = wk[i];
    }
    return t;
  }
};

// Python max(x, lo) / min(x, hi) (feature_processor.py:231-234): NaN propagates like the reference
__device__ __forceinline__ double pmax(double x, double lo) { return (lo > x) ? lo : x; }
__device__ __forceinline__ double pmin(double x, double hi) { return (hi < x) ? hi : x; }
__device__ __forceinline__ float clip10(double x) {
  if (x < -10.0) x = -10.0;
  if (x > 10.0) x = 10.0;
  return (float)x;
}

// One transaction as the bucket kernel reads it, written by the slot kernel in arrival order: the fields the
// card-independent features need with the merchant row already looked up and the card-independent
// arithmetic done (log, log1p, sqrt, calendar fields), so the bucket kernel's random read of transaction i is
// ONE 64-B record (four 16-B loads in flight with the card header) whatever the source layout (eight SoA
// columns or a route record), no merchant-table round trip follows it and its dependent chain is shorter.
struct __attribute__((aligned(16))) Prep {
  long long ts, cents;
  unsigned long long dfp;
  double mfr;   // merchant fraud rate as the feature reads it (unknown merchant 0.1, null rate 0.05)
  double mult;  // merchant risk multiplier (unknown merchant 2.0)
  double r1;    // raw feature 1: log(amount + 1) (Java Math.log; the card-independent transcendental)
  float o1;     // vector slot 1: clip10(log1p(amount)) (FeatureProcessor amount_log)
  float dv0;    // derived amount_sqrt: clip10(sqrt(amount)) (used when amount > 0)
  int merchant;
  unsigned char ipc, hour, dow, weekend;  // hour / day of week / weekend as the features read them
};
static_assert(sizeof(Prep) == 64, "Prep must be 64 B");

// The card-independent part of a transaction's features, computed here where it hides under the slot
// probe's latency (base_raw / write_vector read the results; same operations, so the same bits).
__device__ __forceinline__ Prep make_prep(const Txn& t, const Merchant* __restrict__ merchants, int nm) {
#pragma clang fp contract(off)
  Prep p;
  p.ts = t.ts;
  p.cents = t.cents;
  p.dfp = t.dfp;
  if (t.merchant >= 0 && t.merchant < nm) {  // FeatureExtractor merchant lookup (see base_raw)
    const Merchant m = merchants[t.merchant];
    p.mfr = isnan(m.fraud_rate) ? 0.05 : m.fraud_rate;
    p.mult = m.mult;
  } else {
    p.mfr = 0.1;
    p.mult = 2.0;
  }
  const double r0 = (double)t.cents / 100.0;
  p.r1 = (r0 + 1 > 0) ? log(r0 + 1) : ((r0 + 1 == 0) ? -INFINITY : NAN);
  const double amount = pmax(r0, 0.0);  // write_vector's amount
  double alog = p.r1;
  if (isnan(alog) || isinf(alog)) alog = 0.0;
  if (amount > 0) alog = log1p(amount);
  p.o1 = clip10(alog);
  p.dv0 = clip10(sqrt(amount));
  long long days = t.ts / 86400000LL;  // event time -> hour / ISO day of week (1 = Monday) in UTC
  if (t.ts % 86400000LL < 0) days -= 1;
  int hour = (int)((t.ts - days * 86400000LL) / 3600000LL);
  long long dw = (days + 3) % 7;
  if (dw < 0) dw += 7;
  const int dow = (int)dw + 1;
  if (t.hour != 255) hour = t.hour;
  p.hour = (unsigned char)hour;
  p.dow = (unsigned char)dow;
  p.weekend = ((t.wk == 255) ? (dow >= 6) : (t.wk != 0)) ? 1 : 0;
  p.merchant = t.merchant;
  p.ipc = t.ipc;
  return p;
}

__device__ __forceinline__ void store_prep(Prep* dst, const Prep& p) {
  uint4* q = reinterpret_cast<uint4*>(dst);
  const unsigned long long a = (unsigned long long)p.ts, b = (unsigned long long)p.cents;
  const unsigned long long c = __double_as_longlong(p.mfr), d = __double_as_longlong(p.mult);
  const unsigned long long e = __double_as_longlong(p.r1);
  q[0] = make_uint4((unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32));
  q[1] = make_uint4((unsigned)p.dfp, (unsigned)(p.dfp >> 32), (unsigned)c, (unsigned)(c >> 32));
  q[2] = make_uint4((unsigned)d, (unsigned)(d >> 32), (unsigned)e, (unsigned)(e >> 32));
  q[3] = make_uint4(__float_as_uint(p.o1), __float_as_uint(p.dv0), (unsigned)p.merchant,
                    (unsigned)p.ipc | ((unsigned)p.hour << 8) | ((unsigned)p.dow << 16) | ((unsigned)p.weekend << 24));
}

__device__ __forceinline__ Prep load_prep(const Prep* __restrict__ src) {
  const uint4* q = reinterpret_cast<const uint4*>(src);
  const uint4 w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
  Prep p;
  p.ts = (long long)(((unsigned long long)w0.y << 32) | w0.x);
  p.cents = (long long)(((unsigned long long)w0.w << 32) | w0.z);
  p.dfp = ((unsigned long long)w1.y << 32) | w1.x;
  p.mfr = __longlong_as_double((long long)(((unsigned long long)w1.w << 32) | w1.z));
  p.mult = __longlong_as_double((long long)(((unsigned long long)w2.y << 32) | w2.x));
  p.r1 = __longlong_as_double((long long)(((unsigned long long)w2.w << 32) | w2.z));
  p.o1 = __uint_as_float(w3.x);
  p.dv0 = __uint_as_float(w3.y);
  p.merchant = (int)w3.z;
  p.ipc = (unsigned char)(w3.w & 0xffu);
  p.hour = (unsigned char)((w3.w >> 8) & 0xffu);
  p.dow = (unsigned char)((w3.w >> 16) & 0xffu);
  p.weekend = (unsigned char)((w3.w >> 24) & 0xffu);
  return p;
}

// Split rows (engine option compact_vectors 2, the pipelined stream's fused-kernel batches without LSTM history):
// the card-independent half of the scoring row is finished by the slot kernel, which has the transaction's columns
// in hand, and the bucket kernel reads back only what the card work needs. Per transaction (arrival order):
//   Prep32 (32 B, slot -> bucket kernel): ts, cents, device fingerprint — the bucket kernel's random read of
//           transaction i is one 32-B piece instead of the 64-B Prep;
//   RowA   (32 B, slot kernel -> fused kernel): the card-independent compact slots, final (features.hip
//           write_vector's arithmetic): amount, amount_log, amount_sqrt (derived), merchant fraud rate / risk
//           score, IP risk, the derived combined_device_ip_risk, and as bytes hour, day of week, weekend and the
//           flags {amount > 0, business hours, late night};
//   RowB   (32 B, bucket kernel -> fused kernel): the card-dependent slots: 24 h / 1 h amounts, user average,
//           amount / user average, hourly velocity ratio, and as bytes the 1 h / 24 h / 5 min counts, account age,
//           new device, {user average > 0}.
// The fused kernel (ensemble.hip load_split) assembles the 22 compact slots from the two rows, including the derived
// features' data-dependent positions; every value is the f32 write_vector stores, so the bins and outputs are the
// 64-wide path's bit for bit.
struct __attribute__((aligned(16))) Prep32 {
  long long ts, cents;
  unsigned long long dfp;
  unsigned long long pad;
};
static_assert(sizeof(Prep32) == 32, "Prep32 must be 32 B");
constexpr unsigned kRowAPos = 1u, kRowABus = 2u, kRowALate = 4u;  // RowA flags (byte 31)
constexpr unsigned kRowBUavg = 1u;                                 // RowB flags (byte 25)

__device__ __forceinline__ void store_prep32(Prep32* dst, const Txn& t) {
  uint4* q = reinterpret_cast<uint4*>(dst);
  const unsigned long long a = (unsigned long long)t.ts, b = (unsigned long long)t.cents;
  q[0] = make_uint4((unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32));
  q[1] = make_uint4((unsigned)t.dfp, (unsigned)(t.dfp >> 32), 0u, 0u);
}

// the fields the card work reads (base_raw / velocity_step in split mode: cents, ts, device fingerprint)
__device__ __forceinline__ Prep load_prep32(const Prep32* __restrict__ src) {
  const uint4* q = reinterpret_cast<const uint4*>(src);
  const uint4 w0 = q[0], w1 = q[1];
  Prep p{};
  p.ts = (long long)(((unsigned long long)w0.y << 32) | w0.x);
  p.cents = (long long)(((unsigned long long)w0.w << 32) | w0.z);
  p.dfp = ((unsigned long long)w1.y << 32) | w1.x;
  return p;
}

// RowA from the slot kernel's prep (the same operations as write_vector / base_raw on these fields)
__device__ __forceinline__ void store_row_a(uint4* dst, const Prep& p) {
#pragma clang fp contract(off)
  const double r0 = (double)p.cents / 100.0;
  const double amount = pmax(r0, 0.0);
  const double hour = pmin(pmax((double)p.hour, 0.0), 23.0);
  const double dow = pmin(pmax((double)p.dow, 0.0), 6.0);
  double mfr = pmin(pmax(p.mfr, 0.0), 1.0);
  if (isnan(mfr)) mfr = 0.0;
  const double r7 = p.ipc == 0 ? NAN : (p.ipc == 1 ? 0.1 : 0.3);
  const double ip = isnan(r7) ? 0.5 : pmin(pmax(r7, 0.0), 1.0);
  double mrisk = pmin(pmax(p.mult, 0.0), 1.0);
  if (isnan(mrisk)) mrisk = 0.5;
  unsigned b = 0u;
  b = __builtin_amdgcn_cvt_pk_u8_f32(clip10(hour), 0, b);
  b = __builtin_amdgcn_cvt_pk_u8_f32(clip10(dow), 1, b);
  b = __builtin_amdgcn_cvt_pk_u8_f32(p.weekend ? 1.f : 0.f, 2, b);
  const unsigned fl = (amount > 0 ? kRowAPos : 0u) | ((9 <= hour && hour <= 17) ? kRowABus : 0u) |
                      ((hour < 6 || hour > 22) ? kRowALate : 0u);
  b |= fl << 24;
  dst[0] = make_uint4(__float_as_uint(clip10(amount)), __float_as_uint(p.o1), __float_as_uint(p.dv0),
                      __float_as_uint(clip10(mfr)));
  dst[1] = make_uint4(__float_as_uint(clip10(mrisk)), __float_as_uint(clip10(ip)),
                      __float_as_uint(clip10((0.5 + ip) / 2)), b);
}

// RowB from the card work's raw features (write_vector's arithmetic for the card-dependent slots)
__device__ __forceinline__ void store_row_b(uint4* dst, const double* r) {
#pragma clang fp contract(off)
  const double amount = pmax(r[0], 0.0);
  const double uavg = isnan(r[8]) ? 0.0 : pmax(r[8], 0.0);
  const double c5 = pmax(r[9], 0.0), c1 = pmax(r[10], 0.0), c24 = pmax(r[11], 0.0);
  const double s1 = pmax(r[12], 0.0), s24 = pmax(r[13], 0.0);
  const double age = pmax(r[15], 0.0);
  unsigned b = 0u, b2 = 0u;
  b = __builtin_amdgcn_cvt_pk_u8_f32(clip10(c1), 0, b);
  b = __builtin_amdgcn_cvt_pk_u8_f32(clip10(c24), 1, b);
  b = __builtin_amdgcn_cvt_pk_u8_f32(clip10(age), 2, b);
  b = __builtin_amdgcn_cvt_pk_u8_f32(r[6] > 0.5 ? 1.f : 0.f, 3, b);
  b2 = __builtin_amdgcn_cvt_pk_u8_f32(clip10(c5), 0, b2);
  b2 |= (uavg > 0 ? kRowBUavg : 0u) << 8;
  dst[0] = make_uint4(__float_as_uint(clip10(s24)), __float_as_uint(clip10(uavg)), __float_as_uint(clip10(s1)),
                      __float_as_uint(clip10(amount / uavg)));
  dst[1] = make_uint4(__float_as_uint(clip10(c1 / (c24 / 24))), b, b2, 0u);
}

// ------------------------------------------------------------------------------------------------
// per-batch card grouping
// Per transaction: card slot (find-or-insert), prep record, and its (slot, arrival index) key appended to its
// bucket's fixed-capacity region (bucket = slot & nbm): per block an LDS histogram, one global atomic per
// (block, bucket) reserving the block's run, then each key at its rank in the run. A bucket that outgrows its
// capacity C spills the rest to an overflow list (bucket id + key) its bucket kernel scans. No count / scan /
// scatter passes: the bucket kernel's inputs are complete when this kernel ends.
__global__ void __launch_bounds__(kST) feat_slot_kernel(CardPages P, unsigned long long* K, long long mask, int64_t n, TxnSrc src,
                                                        const Merchant* __restrict__ merchants, int nm,
                                                        unsigned nbm, unsigned C, unsigned* __restrict__ slot,
                                                        Prep* __restrict__ prep, unsigned* __restrict__ fill,
                                                        unsigned long long* __restrict__ pairs,
                                                        unsigned* __restrict__ ovf_cnt,
                                                        unsigned long long* __restrict__ ovf_key,
                                                        unsigned* __restrict__ ovf_b, unsigned* err, int prio,
                                                        uint4* __restrict__ row_a) {
  extern __shared__ unsigned hist[];  // [nbm + 1] block counts | [nbm + 1] reserved run starts
  if (prio) __builtin_amdgcn_s_setprio(2);  // engine option slot_prio (pipelined stream)
  unsigned* run = hist + nbm + 1;
  FD_TL(g_tl_feat, 0, 0);
  for (unsigned b = threadIdx.x; b <= nbm; b += kST) hist[b] = 0u;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kST + threadIdx.x;
  unsigned local = 0, b = 0;
  unsigned long long key = 0;
  bool have = false;
  if (i < n) {
    const Txn t = src.get(i);  // in flight with the probe
    const long long s = card_slot(K, P, mask, src.get_key(i));
    if (row_a) {  // split rows: the 32-B prep the card work reads, the card-independent row finished here
      store_prep32(reinterpret_cast<Prep32*>(prep) + i, t);
      store_row_a(row_a + 2 * i, make_prep(t, merchants, nm));
    } else {
      store_prep(prep + i, make_prep(t, merchants, nm));
    }
    if (s < 0) {
      atomicOr(err, 1u);
      slot[i] = 0xffffffffu;
    } else {
      slot[i] = (unsigned)s;
      b = (unsigned)s & nbm;
      key = ((unsigned long long)s << 32) | (unsigned long long)i;
      local = atomicAdd(&hist[b], 1u);
      have = true;
    }
  }
  __syncthreads();
  for (unsigned q = threadIdx.x; q <= nbm; q += kST)
    if (hist[q]) run[q] = atomicAdd(&fill[q], hist[q]);
  __syncthreads();
  if (have) {
    const unsigned pos = run[b] + local;
    if (pos < C) {
      pairs[(size_t)b * C + pos] = key;
    } else {
      const unsigned j = atomicAdd(ovf_cnt, 1u);
      ovf_key[j] = key;
      ovf_b[j] = b;
    }
  }
  FD_TL(g_tl_feat, 0, 3);
}

// ------------------------------------------------------------------------------------------------
// per-transaction feature arithmetic (shared by the sequential and the cooperative path)

// bridged raw features -> scoring vector: FeatureProcessor.process_features (41 definitions, derived
// features appended when present) + _prepare_features (pad to 64, clip +-10), then the f32 cast the
// models apply. Mirrors oracle/oracle_features.c orc_vector_from_raw.
__device__ void write_vector(const double* r, float o1, float dv0, float* __restrict__ out, bool compact) {
#pragma clang fp contract(off)
  const double amount = pmax(r[0], 0.0);
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
  // the 41 definitions in declaration order (feature_processor.py:66-147); built in registers
  // (compile-time indices only) and stored as 16 x 16 B
  float o[FD_VECTOR_WIDTH];
#pragma unroll
  for (int k = 0; k < FD_VECTOR_WIDTH; ++k) o[k] = 0.f;
  o[0] = clip10(amount);
  o[1] = o1;  // clip10(log1p(amount)), or the sanitised log(amount + 1) when amount <= 0 (make_prep)
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
  const float dv[6] = {dv0, clip10(amount / uavg), clip10(c1 / (c24 / 24)), clip10((0.5 + ip) / 2),
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
  if (compact) {  // the 22 slots that vary (fd_internal.h kCompactSlot): 14 f32 words + 8 byte slots, 4 x 16 B
    float c[kCompactWidth];
    unsigned ib[2] = {0u, 0u};
#pragma unroll
    for (int ci = 0; ci < kCompactSlots; ++ci) {
      const float x = o[kCompactSlot[ci]];
      if (int_slot(ci) >= 0)  // an integer in 0..23 (see kIntCompact): exact as a byte (v_cvt_pk_u8_f32)
        ib[int_slot(ci) >> 2] = __builtin_amdgcn_cvt_pk_u8_f32(x, int_slot(ci) & 3, ib[int_slot(ci) >> 2]);
      else
        c[compact_word(ci)] = x;
    }
    c[14] = __uint_as_float(ib[0]);
    c[15] = __uint_as_float(ib[1]);
#pragma unroll
    for (int q = 0; q < kCompactWidth / 4; ++q) o4[q] = make_float4(c[4 * q], c[4 * q + 1], c[4 * q + 2], c[4 * q + 3]);
    return;
  }
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

// the card's profile as the sequential and cooperative paths read it
struct Profile {
  bool has_user;
  double avg;
  int age;
  unsigned long long fp[3];
};

// raw features 0-8, 14, 15 of one transaction (FeatureExtractor.java:92-325 for the bridged names)
__device__ __forceinline__ void base_raw(const Prep& t, const Profile& p, double* r) {
#pragma clang fp contract(off)
  const bool known = p.has_user && t.dfp != 0ull && (t.dfp == p.fp[0] || t.dfp == p.fp[1] || t.dfp == p.fp[2]);
  r[0] = (double)t.cents / 100.0;
  r[1] = t.r1;  // card-independent fields: make_prep (slot kernel)
  r[2] = t.hour;
  r[3] = t.dow;
  r[4] = t.weekend ? 1.0 : 0.0;
  r[5] = t.mfr;
  r[6] = known ? 0.0 : 1.0;
  r[7] = t.ipc == 0 ? NAN : (t.ipc == 1 ? 0.1 : 0.3);
  r[8] = p.has_user ? (isnan(p.avg) ? 0.0 : p.avg) : NAN;
  r[14] = t.mult;
  r[15] = p.has_user ? (double)p.age : 0.0;
}

__device__ __forceinline__ void velocity_raw(const long long (&c)[3], const long long (&s)[3], double* r) {
  r[9] = (double)c[0];
  r[10] = (double)c[1];
  r[11] = (double)c[2];
  r[12] = (double)s[1] / 100.0;
  r[13] = (double)s[2] / 100.0;
}

struct Outputs {
  float* vec;     // [n][64]
  double* raw;    // [n][16] or null
  double* vel5;   // [n] velocity_5min_amount (feature map) or null
  float* seq;     // [n][S][16] LSTM input sequences or null
  float* seq_ring;  // [cap][S][16] per-card LSTM history (S > 0)
  int S;
  // latency path (fd_score_batch_device, < 4 k transactions): per transaction where the LSTM kernel reads its
  // sequence — the card's ring (slot | head << 32 | count << 40; the card's last transaction of the batch, whose
  // sequence is the ring as this launch leaves it) or, kSeqMaterialized, row i of seq. Null: every row into seq.
  unsigned long long* seq_desc;
  // sliding mode: transactions whose 24 h window held the ring's whole capacity K of prior events (the count may
  // be truncated there: the reference's counters are unbounded, RedisTransactionSink.java:93-105); null otherwise
  unsigned long long* sat;
  int K;
  bool compact;  // vec rows are the compact form (64-B rows, fd_internal.h kCompactWidth: the fused pipeline's ensemble reads them)
};

template <bool SPLIT = false>
__device__ __forceinline__ void emit(const Outputs& o, int64_t i, const double* r, long long s5, float o1, float dv0) {
  if (o.sat && r[11] >= (double)o.K) atomicAdd(o.sat, 1ull);  // rare: the card's last K events all within 24 h
  if (o.raw) {
    double2* ro = reinterpret_cast<double2*>(o.raw + (size_t)i * FD_RAW_FEATURES);
#pragma unroll
    for (int c = 0; c < FD_RAW_FEATURES / 2; ++c) ro[c] = make_double2(r[2 * c], r[2 * c + 1]);
  }
  if (SPLIT)
    store_row_b(reinterpret_cast<uint4*>(o.vec) + 2 * i, r);
  else
    write_vector(r, o1, dv0, o.vec + (size_t)i * (o.compact ? kCompactWidth : FD_VECTOR_WIDTH), o.compact);
  if (o.vel5) o.vel5[i] = (double)s5 / 100.0;
}

// ------------------------------------------------------------------------------------------------
// the sequential path: one thread, one card, its header in registers

struct CardRegs {
  long long last_ts;
  unsigned flags;
  int rn, rh, us;
  int wc[3];
  long long ws[3], wo[3];
  long long rc_sum;
  int rc_cnt;
};

__device__ __forceinline__ long long ll2(unsigned lo, unsigned hi) {
  return (long long)(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ void load_card(const CardHeader* __restrict__ h, CardRegs& c, Profile& p) {
  const uint4* q = reinterpret_cast<const uint4*>(h);
  uint4 w[7];  // bytes 0-111 (the last 16 are padding)
#pragma unroll
  for (int k = 0; k < 7; ++k) w[k] = q[k];
  // field offsets: see CardHeader (fd_internal.h)
  c.last_ts = ll2(w[0].x, w[0].y);
  c.rn = (int)(w[0].z & 0xffu);
  c.rh = (int)((w[0].z >> 8) & 0xffu);
  c.us = (int)((w[0].z >> 16) & 0xffu);
  c.wc[0] = (int)(w[0].w & 0xffu);
  c.wc[1] = (int)((w[0].w >> 8) & 0xffu);
  c.wc[2] = (int)((w[0].w >> 16) & 0xffu);
  c.flags = w[1].x;
  c.rc_cnt = (int)w[1].y;
  c.ws[0] = ll2(w[1].z, w[1].w);
  c.rc_sum = c.ws[0];  // redis_compat keeps its session amount in ws[0]
  c.ws[1] = ll2(w[2].x, w[2].y);
  c.ws[2] = ll2(w[2].z, w[2].w);
  const unsigned wod[3] = {w[3].x, w[3].y, w[3].z};
#pragma unroll
  for (int k = 0; k < 3; ++k) c.wo[k] = c.wc[k] > 0 ? c.last_ts - (long long)wod[k] : 0;
  p.avg = __longlong_as_double(ll2(w[4].z, w[4].w));
  p.age = (int)w[5].x;
  p.fp[0] = (unsigned long long)ll2(w[5].z, w[5].w);
  p.fp[1] = (unsigned long long)ll2(w[6].x, w[6].y);
  p.fp[2] = (unsigned long long)ll2(w[6].z, w[6].w);
  p.has_user = (c.flags & 1u) != 0u;
}

// write back the mutable fields: bytes 0-63 of the header, as four 16-B stores (the key / profile half is never
// rewritten here). An in-window oldest time is at most a window (< 2^32 ms) below the last event: a 32-bit offset.
template <int MODE>
__device__ __forceinline__ void store_card(CardHeader* h, const CardRegs& c) {
  const unsigned long long cur = (unsigned long long)(unsigned)c.rn | ((unsigned long long)(unsigned)c.rh << 8) |
                                 ((unsigned long long)(unsigned)c.us << 16) |
                                 ((unsigned long long)(unsigned)c.wc[0] << 32) |
                                 ((unsigned long long)(unsigned)c.wc[1] << 40) |
                                 ((unsigned long long)(unsigned)c.wc[2] << 48);
  const unsigned long long lt = (unsigned long long)c.last_ts;
  const unsigned long long s0 = (unsigned long long)(MODE == FD_WINDOW_REDIS_COMPAT ? c.rc_sum : c.ws[0]);
  const unsigned long long s1 = (unsigned long long)c.ws[1], s2 = (unsigned long long)c.ws[2];
  unsigned wod[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) wod[k] = c.wc[k] > 0 ? (unsigned)(c.last_ts - c.wo[k]) : 0u;
  uint4* q = reinterpret_cast<uint4*>(h);
  q[0] = make_uint4((unsigned)lt, (unsigned)(lt >> 32), (unsigned)cur, (unsigned)(cur >> 32));
  q[1] = make_uint4(c.flags, (unsigned)c.rc_cnt, (unsigned)s0, (unsigned)(s0 >> 32));
  q[2] = make_uint4((unsigned)s1, (unsigned)(s1 >> 32), (unsigned)s2, (unsigned)(s2 >> 32));
  q[3] = make_uint4(wod[0], wod[1], wod[2], 0u);
}

// windows as of time t from the (time-sorted) ring: the newest events with ts > t - W
__device__ void rebuild_windows(CardRegs& c, const RingEvent* __restrict__ rg, int K, long long t) {
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    c.wc[w] = 0;
    c.ws[w] = 0;
    c.wo[w] = LLONG_MAX;
  }
  for (int e = 0; e < c.rn; ++e) {
    const RingEvent ev = rg[e];
#pragma unroll
    for (int w = 0; w < 3; ++w)
      if (ev.ts > t - kWin[w]) {
        c.wc[w] += 1;
        c.ws[w] += ev.cents;
        c.wo[w] = ev.ts < c.wo[w] ? ev.ts : c.wo[w];
      }
  }
#pragma unroll
  for (int w = 0; w < 3; ++w)
    if (c.wc[w] == 0) c.wo[w] = 0;
}

// one transaction of the card: velocity read (before write), then the write
template <int MODE>
__device__ __forceinline__ void velocity_step(CardRegs& c, RingEvent* __restrict__ rg, int K, long long ts,
                                              long long cents, long long (&cw)[3], long long (&sw)[3]) {
  if (MODE == FD_WINDOW_REDIS_COMPAT) {
    const bool live = (c.flags & 2u) && (ts - c.last_ts <= kSessionTtl);
    const long long cc = live ? c.rc_cnt : 0, ss = live ? c.rc_sum : 0;
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      cw[w] = cc;
      sw[w] = ss;
    }
    c.rc_cnt = (int)(cc + 1);
    c.rc_sum = ss + cents;
    c.last_ts = ts;
    c.flags |= 2u;
    return;
  }
  const bool descent = c.rn > 0 && ts < c.last_ts;
  const bool inc = c.us == 0 && !descent;
  if (inc) {  // time-sorted ring: evict each window's too-old events from its oldest end
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      while (c.wc[w] > 0 && c.wo[w] <= ts - kWin[w]) {
        int idx = c.rh - c.wc[w];
        if (idx < 0) idx += K;
        c.ws[w] -= rg[idx].cents;
        c.wc[w] -= 1;
        if (c.wc[w] > 0) c.wo[w] = rg[idx + 1 == K ? 0 : idx + 1].ts;
      }
      cw[w] = c.wc[w];
      sw[w] = c.ws[w];
    }
  } else {  // full scan (the definition): prior events e with t - W < e.ts <= t
#pragma unroll
    for (int w = 0; w < 3; ++w) cw[w] = sw[w] = 0;
    for (int e0 = 0; e0 < c.rn; e0 += 8) {
      RingEvent ev[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) ev[u] = rg[min(e0 + u, K - 1)];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (e0 + u < c.rn && ev[u].ts <= ts) {
#pragma unroll
          for (int w = 0; w < 3; ++w)
            if (ts - kWin[w] < ev[u].ts) {
              cw[w] += 1;
              sw[w] += ev[u].cents;
            }
        }
    }
  }
  // append: a full ring overwrites its oldest event, which leaves every window spanning the whole ring
  if (inc && c.rn == K && (c.wc[0] == K || c.wc[1] == K || c.wc[2] == K)) {
    const long long oc = rg[c.rh].cents;
    const long long nts = rg[c.rh + 1 == K ? 0 : c.rh + 1].ts;
#pragma unroll
    for (int w = 0; w < 3; ++w)
      if (c.wc[w] == K) {
        c.ws[w] -= oc;
        c.wc[w] -= 1;
        if (c.wc[w] > 0) c.wo[w] = nts;
      }
  }
  rg[c.rh] = RingEvent{ts, cents};
  c.rh = c.rh + 1 == K ? 0 : c.rh + 1;
  if (c.rn < K) ++c.rn;
  c.us = descent ? K : (c.us > 0 ? c.us - 1 : 0);
  c.last_ts = ts;
  if (c.us == 0) {
    if (inc) {
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        if (c.wc[w] == 0) c.wo[w] = ts;
        c.wc[w] += 1;
        c.ws[w] += cents;
      }
    } else {
      rebuild_windows(c, rg, K, ts);  // the ring just became time-sorted again
    }
  } else {
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      c.wc[w] = 0;
      c.ws[w] = 0;
      c.wo[w] = 0;
    }
  }
}

// LSTM head input: this event appended to the card's history, the last S events emitted (or, for the card's last
// transaction of the batch on the latency path, its place in the ring: the LSTM kernel reads them there)
__device__ __forceinline__ void seq_step(const Outputs& o, unsigned s, unsigned& flags, int64_t i, const double* r,
                                         bool last) {
  const int S = o.S;
  int seq_n = (int)((flags >> 8) & 0xffu), seq_head = (int)((flags >> 16) & 0xffu);
  float* sr = o.seq_ring + (size_t)s * S * kSeqInput;
  float* slot_ev = sr + (size_t)seq_head * kSeqInput;
#pragma unroll
  for (int c = 0; c < kSeqInput; ++c) slot_ev[c] = seq_input(r[c]);
  seq_head = (seq_head + 1 == S) ? 0 : seq_head + 1;
  if (seq_n < S) ++seq_n;
  if (o.seq_desc) {
    if (last) {
      o.seq_desc[i] = (unsigned long long)s | ((unsigned long long)seq_head << 32) | ((unsigned long long)seq_n << 40);
    } else {
      o.seq_desc[i] = kSeqMaterialized;
    }
  }
  if (o.seq && !(o.seq_desc && last)) {  // oldest -> newest, left-padded with zero events (Keras pad_sequences 'pre')
    float* so = o.seq + (size_t)i * S * kSeqInput;
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
  flags = (flags & 0xffu) | ((unsigned)seq_n << 8) | ((unsigned)seq_head << 16);
}

struct BucketArgs {
  CardPages P;  // header + ring per card slot
  int K;
  int64_t n;
  const Prep* prep;  // [n] in arrival order (feat_slot_kernel); split rows: Prep32 records
  Outputs out;
  unsigned* fill;                     // keys per bucket (this batch); reset here for the next batch
  const unsigned long long* pairs;    // [NB][C] bucket regions
  unsigned C;
  unsigned* ovf_cnt;                  // [2] overflow counts by batch parity
  int par;
  const unsigned long long* ovf_key;  // overflow list: key, bucket
  const unsigned* ovf_b;
  unsigned spec;                      // latency batches: region entries read before the fill count (<= kBT, <= C)
  bool spread;                        // card segments dealt round-robin over the 4 waves (engine option bucket_spread)
  bool prio;                          // issue priority 2 (engine option feature_prio, pipelined stream)
  int lean_group;                     // lean kernel grouping: 0 rank sort, 1 split rank sort, 2 hash (option lean_group)
};

// gather (latency batches, n <= kChunkCap, engine option slot_gather; feat_bucket_gather_kernel): no slot launch;
// bucket b takes the transactions whose key hashes to it (gather_bucket), finds / inserts their card slots, writes
// their prep records and slots, then runs the same sorted card pass. Its own argument block, so the other bucket
// kernels' arguments (and registers) do not grow.
struct GatherArgs {
  unsigned nbm;
  TxnSrc src;
  unsigned long long* keys;
  long long mask;
  const Merchant* merchants;
  int nm;
  Prep* prep_w;
  unsigned* slot;
  unsigned* err;
};

// transaction i's prep record as the card work reads it (split rows: the 32-B form)
template <bool SPLIT>
__device__ __forceinline__ Prep fetch_prep(const BucketArgs& a, int64_t i) {
  return SPLIT ? load_prep32(reinterpret_cast<const Prep32*>(a.prep) + i) : load_prep(a.prep + i);
}

// a card's bucket in gather mode: every transaction of a card in one bucket, buckets filled evenly
__device__ __forceinline__ unsigned gather_bucket(unsigned long long key, unsigned nbm) {
  return (unsigned)(mix64(key ^ 0x9E3779B97F4A7C15ull) >> 32) & nbm;
}

// The thread that takes bucket position pos (mod kBT): with `spread`, consecutive positions go to different waves, so
// a bucket's m < kBT cards are worked by all four SIMDs instead of the first m / 64 waves (the card loop is
// latency- and f64-issue-bound per wave)
static_assert(kBT == 256, "spread_pos deals positions over 4 waves of 64");
__device__ __forceinline__ int first_pos(bool spread) {
  const int t = (int)threadIdx.x;
  return spread ? (((t & 63) << 2) | (t >> 6)) : t;
}

template <int MODE, bool SPLIT, typename KeyT = unsigned long long>
__device__ void process_short(const BucketArgs& a, unsigned s, const KeyT* keys, int len) {
  CardHeader* h = a.P.hdr(s);
  CardRegs c;
  Profile p;
  Prep t = fetch_prep<SPLIT>(a, (unsigned)keys[0]);  // in flight with the header
  load_card(h, c, p);
  RingEvent* rg = a.P.ring(s);
  for (int q = 0; q < len; ++q) {
    const int64_t i = (int64_t)(unsigned)keys[q];
    if (q > 0) t = fetch_prep<SPLIT>(a, i);
    double r[FD_RAW_FEATURES];
    base_raw(t, p, r);
    if (q == 0) FD_CSTAMP(0);
    long long cw[3], sw[3];
    velocity_step<MODE>(c, rg, a.K, t.ts, t.cents, cw, sw);
    if (q == 0) FD_CSTAMP(1);
    velocity_raw(cw, sw, r);
    emit<SPLIT>(a.out, i, r, sw[0], t.o1, t.dv0);
    if (a.out.S) seq_step(a.out, s, c.flags, i, r, q == len - 1);
    if (q == 0) FD_CSTAMP(2);
  }
  store_card<MODE>(h, c);
}

// ------------------------------------------------------------------------------------------------
// the cooperative path: a long segment (hot card) processed by the whole workgroup, kBT per tile

struct LongLds {
  long long ev_ts[kMaxK + kBT];   // [0, K): the K events before the tile (hist_n valid at the top); [K, K+T): tile
  long long ev_c[kMaxK + kBT];
  long long pre[kBT];             // redis: inclusive prefix sum of the tile's cents
  int rst[kBT];                   // redis: last reset index <= j (-1 none); sliding: last descent index <= j
  float seqb[(FD_MAX_SEQ_LEN + kBT) * kSeqInput];  // LSTM inputs: [0, S) history, [S, S+T) tile
  CardHeader hdr;
  long long carry_c, carry_s;     // redis session after the previous tile
  int hist_n, us, seq_n, pad;
};

__device__ void block_scan_sum(long long* v) {  // inclusive, kBT entries
  for (int d = 1; d < kBT; d <<= 1) {
    const long long x = threadIdx.x >= (unsigned)d ? v[threadIdx.x - d] : 0;
    __syncthreads();
    v[threadIdx.x] += x;
    __syncthreads();
  }
}

__device__ void block_scan_max(int* v) {  // inclusive, kBT entries
  for (int d = 1; d < kBT; d <<= 1) {
    const int x = threadIdx.x >= (unsigned)d ? v[threadIdx.x - d] : -1;
    __syncthreads();
    v[threadIdx.x] = max(v[threadIdx.x], x);
    __syncthreads();
  }
}

template <int MODE, bool SPLIT>
__device__ void process_long(const BucketArgs& a, unsigned s, const unsigned long long* keys, int L, LongLds& sm) {
  const int tid = threadIdx.x, K = a.K, S = a.out.S;
  CardHeader* h = a.P.hdr(s);
  RingEvent* rg = a.P.ring(s);
  if (tid == 0) {
    sm.hdr = *h;
    sm.carry_c = sm.hdr.rc_cnt;
    sm.carry_s = sm.hdr.ws[0];  // redis_compat: the session amount
    sm.hist_n = MODE == FD_WINDOW_SLIDING ? sm.hdr.ring_n : 0;
    sm.us = sm.hdr.unsorted;
    sm.seq_n = (int)((sm.hdr.flags >> 8) & 0xffu);
  }
  __syncthreads();
  const int rn0 = sm.hdr.ring_n, rh0 = sm.hdr.ring_head;
  const long long ts0 = sm.hdr.last_ts;
  const bool has_ts0 = (sm.hdr.flags & 2u) != 0u;
  Profile p;
  p.has_user = (sm.hdr.flags & 1u) != 0u;
  p.avg = sm.hdr.avg;
  p.age = sm.hdr.age;
  for (int k = 0; k < 3; ++k) p.fp[k] = sm.hdr.fp[k];
  if (MODE == FD_WINDOW_SLIDING && tid < rn0) {  // the ring, oldest first, at the top of [0, K)
    int src = rh0 - rn0 + tid;
    if (src < 0) src += K;
    const RingEvent ev = rg[src];
    sm.ev_ts[K - rn0 + tid] = ev.ts;
    sm.ev_c[K - rn0 + tid] = ev.cents;
  }
  const int seq_n0 = sm.seq_n, seq_h0 = (int)((sm.hdr.flags >> 16) & 0xffu);
  const float* sr = S ? a.out.seq_ring + (size_t)s * S * kSeqInput : nullptr;
  if (S && tid < seq_n0 * kSeqInput) {  // the LSTM history, oldest first, at the top of [0, S)
    const int e = tid / kSeqInput, c = tid % kSeqInput;
    int src = seq_h0 - seq_n0 + e;
    if (src < 0) src += S;
    sm.seqb[(S - seq_n0 + e) * kSeqInput + c] = sr[(size_t)src * kSeqInput + c];
  }
  __syncthreads();
  for (int t0 = 0; t0 < L; t0 += kBT) {
    const int T = min(kBT, L - t0), j = tid;
    const bool act = j < T;
    const int64_t i = act ? (int64_t)(unsigned)keys[t0 + j] : 0;
    Prep t{};
    if (act) {
      t = fetch_prep<SPLIT>(a, i);
      sm.ev_ts[K + j] = t.ts;
      sm.ev_c[K + j] = t.cents;
    }
    __syncthreads();
    // the previous event's time in the card's order (ring / previous tile / this tile)
    const bool first = t0 == 0 && j == 0;
    const long long prev_ts = (j > 0 || t0 > 0) ? sm.ev_ts[K + j - 1] : ts0;
    const bool has_prev = !first || (MODE == FD_WINDOW_SLIDING ? rn0 > 0 : has_ts0);
    long long cw[3] = {0, 0, 0}, sw[3] = {0, 0, 0};
    if (MODE == FD_WINDOW_REDIS_COMPAT) {
      const bool live = act && has_prev && (t.ts - prev_ts <= kSessionTtl);
      sm.pre[j] = act ? t.cents : 0;
      sm.rst[j] = (act && !live) ? j : -1;
      __syncthreads();
      block_scan_sum(sm.pre);
      block_scan_max(sm.rst);
      if (act && live) {  // the session after the previous transaction
        long long cc, ss;
        if (j == 0) {
          cc = sm.carry_c;
          ss = sm.carry_s;
        } else {
          const int R = sm.rst[j - 1];
          cc = R < 0 ? sm.carry_c + j : j - R;
          ss = R < 0 ? sm.carry_s + sm.pre[j - 1] : sm.pre[j - 1] - (R > 0 ? sm.pre[R - 1] : 0);
        }
        for (int w = 0; w < 3; ++w) {
          cw[w] = cc;
          sw[w] = ss;
        }
      }
    } else {
      // positional windows: the card's previous K events are buffer slots [max(K - hist_n, j), K + j)
      if (act) {
        for (int e = max(K - sm.hist_n, j); e < K + j; ++e) {
          const long long et = sm.ev_ts[e];
          if (et <= t.ts)
            for (int w = 0; w < 3; ++w)
              if (t.ts - kWin[w] < et) {
                cw[w] += 1;
                sw[w] += sm.ev_c[e];
              }
        }
      }
      sm.rst[j] = (act && has_prev && t.ts < prev_ts) ? j : -1;  // descents (out-of-order arrivals)
      __syncthreads();
      block_scan_max(sm.rst);
    }
    double r[FD_RAW_FEATURES];
    if (act) {
      base_raw(t, p, r);
      velocity_raw(cw, sw, r);
      emit<SPLIT>(a.out, i, r, sw[0], t.o1, t.dv0);
      if (S)
        for (int c = 0; c < kSeqInput; ++c) sm.seqb[(S + j) * kSeqInput + c] = seq_input(r[c]);
    }
    __syncthreads();
    if (S && act && a.out.seq) {  // txn j's sequence: the last S events up to and including itself
      const int have = min(S, sm.seq_n + j + 1), pad = S - have;
      float* so = a.out.seq + (size_t)i * S * kSeqInput;
      for (int q = 0; q < S; ++q) {
        float4* dst = reinterpret_cast<float4*>(so + (size_t)q * kSeqInput);
        const float4* src = reinterpret_cast<const float4*>(&sm.seqb[(j + 1 + q) * kSeqInput]);
        for (int c = 0; c < kSeqInput / 4; ++c) dst[c] = q < pad ? make_float4(0.f, 0.f, 0.f, 0.f) : src[c];
      }
      if (a.out.seq_desc) a.out.seq_desc[i] = kSeqMaterialized;
    }
    // carries for the next tile (values read before the barrier, written after it)
    long long nts = 0, nc = 0;
    if (tid < K) {
      const int src = T + tid;  // the last K of [prior | tile]
      nts = sm.ev_ts[src];
      nc = sm.ev_c[src];
    }
    float sv[kSeqInput];
    const bool seq_mover = S && tid < S;
    if (seq_mover)
      for (int c = 0; c < kSeqInput; ++c) sv[c] = sm.seqb[(T + tid) * kSeqInput + c];
    long long ncc = 0, nss = 0;
    int nus = 0;
    if (tid == 0) {
      if (MODE == FD_WINDOW_REDIS_COMPAT) {
        const int R = sm.rst[T - 1];
        ncc = R < 0 ? sm.carry_c + T : T - R;
        nss = R < 0 ? sm.carry_s + sm.pre[T - 1] : sm.pre[T - 1] - (R > 0 ? sm.pre[R - 1] : 0);
      } else {
        const int d = sm.rst[T - 1];
        nus = d >= 0 ? max(0, K - (T - 1 - d)) : max(0, sm.us - T);
      }
    }
    __syncthreads();
    if (tid < K) {
      sm.ev_ts[tid] = nts;
      sm.ev_c[tid] = nc;
    }
    if (seq_mover)
      for (int c = 0; c < kSeqInput; ++c) sm.seqb[tid * kSeqInput + c] = sv[c];
    if (tid == 0) {
      sm.hist_n = min(K, sm.hist_n + T);
      sm.seq_n = min(S, sm.seq_n + T);
      sm.carry_c = ncc;
      sm.carry_s = nss;
      sm.us = nus;
    }
    __syncthreads();
  }
  // final state: ring = the card's last K events, header rebuilt as the sequential path leaves it
  const long long last = sm.ev_ts[K - 1];
  if (MODE == FD_WINDOW_SLIDING) {
    const int rn = min(K, rn0 + L), rh = (rh0 + L) % K;
    if (tid < rn) {
      int dst = rh - rn + tid;
      if (dst < 0) dst += K;
      rg[dst] = RingEvent{sm.ev_ts[K - rn + tid], sm.ev_c[K - rn + tid]};
    }
  }
  if (S && tid < sm.seq_n * kSeqInput) {
    const int e = tid / kSeqInput, c = tid % kSeqInput;
    const int sh = (seq_h0 + L) % S;
    int dst = sh - sm.seq_n + e;
    if (dst < 0) dst += S;
    a.out.seq_ring[((size_t)s * S + dst) * kSeqInput + c] = sm.seqb[(S - sm.seq_n + e) * kSeqInput + c];
  }
  if (tid == 0) {
    CardRegs c;
    c.last_ts = last;
    c.flags = sm.hdr.flags;
    if (S) c.flags = (c.flags & 0xffu) | ((unsigned)sm.seq_n << 8) | ((unsigned)((seq_h0 + L) % S) << 16);
    c.rn = sm.hdr.ring_n;
    c.rh = sm.hdr.ring_head;
    c.us = sm.hdr.unsorted;
    for (int w = 0; w < 3; ++w) {
      c.wc[w] = sm.hdr.wc[w];
      c.ws[w] = sm.hdr.ws[w];
      c.wo[w] = sm.hdr.wc[w] > 0 ? sm.hdr.last_ts - (long long)sm.hdr.wod[w] : 0;
    }
    c.rc_sum = sm.hdr.ws[0];
    c.rc_cnt = sm.hdr.rc_cnt;
    if (MODE == FD_WINDOW_REDIS_COMPAT) {
      c.rc_cnt = (int)sm.carry_c;
      c.rc_sum = sm.carry_s;
      c.flags |= 2u;
    } else {
      c.rn = min(K, rn0 + L);
      c.rh = (rh0 + L) % K;
      c.us = sm.us;
      for (int w = 0; w < 3; ++w) {
        c.wc[w] = 0;
        c.ws[w] = 0;
        c.wo[w] = 0;
      }
      if (c.us == 0) {  // windows as of the last event, from the newest events (time-sorted ring)
        for (int w = 0; w < 3; ++w) c.wo[w] = LLONG_MAX;
        for (int e = K - c.rn; e < K; ++e) {
          const long long et = sm.ev_ts[e];
          for (int w = 0; w < 3; ++w)
            if (et > last - kWin[w]) {
              c.wc[w] += 1;
              c.ws[w] += sm.ev_c[e];
              c.wo[w] = et < c.wo[w] ? et : c.wo[w];
            }
        }
        for (int w = 0; w < 3; ++w)
          if (c.wc[w] == 0) c.wo[w] = 0;
      }
    }
    store_card<MODE>(h, c);
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// the bucket kernel

// Ascending bitonic sort of N (a power of two) keys in LDS. Pair idx of a stage touches positions
// lo = 2*stride*(idx / stride) + idx % stride and lo + stride; the 64 pairs of one wave span 128 consecutive
// positions, so stages with stride <= 64 stay inside the wave (no workgroup barrier, only wave order).
__device__ void bitonic_sort(unsigned long long* k, int N) {
  for (int size = 2; size <= N; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const int sh = 31 - __clz(stride);
      if (stride >= 128) __syncthreads();  // other waves' positions: their previous stages must be done
      for (int idx = threadIdx.x; idx < (N >> 1); idx += kBT) {
        const int lo = ((idx >> sh) << (sh + 1)) + (idx & (stride - 1)), hi = lo + stride;
        const bool asc = (lo & size) == 0;
        const unsigned long long x = k[lo], y = k[hi];
        if ((x > y) == asc) {
          k[lo] = y;
          k[hi] = x;
        }
      }
      if (stride >= 128) __syncthreads();
      else __builtin_amdgcn_wave_barrier();
    }
  }
  __syncthreads();
}

// Ascending order of m <= kRankMax DISTINCT keys (the arrival index makes them distinct) by rank counting:
// each thread holds kRankMax / kBT keys in registers and counts the smaller keys of the whole list (every
// lane of a wave reads the same 16 B: a broadcast, no bank conflicts), then stores each key at its rank.
// O(m^2 / kBT) compares but no dependent LDS round trips per stage: at the usual bucket size (~128 keys)
// ~10x faster than the log^2 stages of the bitonic network, which remains for the larger chunks.
constexpr int kRankMax = 512;
__device__ void rank_sort(unsigned long long* k, int m) {
  constexpr int R = kRankMax / kBT;
  unsigned long long mine[R];
  int rank[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int q = threadIdx.x + r * kBT;
    mine[r] = q < m ? k[q] : 0ull;
    rank[r] = 0;
  }
  const int m2 = m & ~1;
  const ulonglong2* k2 = reinterpret_cast<const ulonglong2*>(k);
#pragma unroll 4
  for (int q = 0; q < m2; q += 2) {
    const ulonglong2 v = k2[q >> 1];
#pragma unroll
    for (int r = 0; r < R; ++r) rank[r] += (int)(v.x < mine[r]) + (int)(v.y < mine[r]);
  }
  if (m & 1) {
    const unsigned long long v = k[m - 1];
#pragma unroll
    for (int r = 0; r < R; ++r) rank[r] += (int)(v < mine[r]);
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (threadIdx.x + r * kBT < m) k[rank[r]] = mine[r];
  __syncthreads();
}

// The same ranks for m <= kBT keys with every thread working: key j's rank is summed over P = kBT / m' parts of the
// key list (m' = m rounded up to a power of two >= 64), each thread scanning one part for one key, the partial ranks
// added into rk[] (zeroed by the caller before the barrier that published the keys). The full form gives each of
// the first m threads all m compares and leaves the other waves idle — with m ~ 128 on the pipelined stream half its
// VALU issue, spent beside the fused ensemble kernel's waves on the same SIMDs.
__device__ void rank_sort_split(unsigned long long* k, int m, int* rk) {
  int mp = 64;
  while (mp < m) mp <<= 1;
  const int P = kBT / mp;
  const int j = (int)threadIdx.x & (mp - 1), p = (int)threadIdx.x / mp;
  const int L = (((m + P - 1) / P) + 1) & ~1;  // even: the part starts on a 16-B pair
  const int lo = min(m, p * L), hi = min(m, lo + L);
  const unsigned long long mine = j < m ? k[j] : 0ull;
  const unsigned long long own = (int)threadIdx.x < m ? k[threadIdx.x] : 0ull;
  const ulonglong2* k2 = reinterpret_cast<const ulonglong2*>(k);
  int r = 0;
#pragma unroll 4
  for (int q = lo; q + 1 < hi; q += 2) {
    const ulonglong2 v = k2[q >> 1];
    r += (int)(v.x < mine) + (int)(v.y < mine);
  }
  if ((hi - lo) & 1) r += (int)(k[hi - 1] < mine);
  if (j < m && r) atomicAdd(&rk[j], r);
  __syncthreads();
  if ((int)threadIdx.x < m) k[rk[threadIdx.x]] = own;
  __syncthreads();
}

// m keys (slot << 32 | arrival index) already in LDS skeys[0, m): sort, then process every segment
template <int MODE, bool SPLIT>
__device__ void process_sorted(const BucketArgs& a, unsigned long long* skeys, int m, LongLds& sm, int* long_list,
                               int* n_long) {
  if (threadIdx.x == 0) *n_long = 0;
  FD_FSTAMP(1);
  if (m <= kRankMax) {
    if (m > 1) rank_sort(skeys, m);  // its first barrier publishes *n_long
    else __syncthreads();
  } else {
    int N = 2;
    while (N < m) N <<= 1;
    for (int q = m + threadIdx.x; q < N; q += kBT) skeys[q] = ~0ull;
    __syncthreads();
    bitonic_sort(skeys, N);
  }
  FD_FSTAMP(2);
  for (int pos = first_pos(a.spread); pos < m; pos += kBT) {
    const unsigned s = (unsigned)(skeys[pos] >> 32);
    if (pos > 0 && (unsigned)(skeys[pos - 1] >> 32) == s) continue;  // not the first txn of its card
    int len = 1;
    while (pos + len < m && (unsigned)(skeys[pos + len] >> 32) == s && len <= kSegLong) ++len;
    if (len > kSegLong) {
      long_list[atomicAdd(n_long, 1)] = pos;
      continue;
    }
    process_short<MODE, SPLIT>(a, s, skeys + pos, len);
  }
#ifdef FD_FOREST_PROFILE
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096)
    g_fprof[blockIdx.x * 8 + 4 + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memtime();
#endif
  __syncthreads();
  FD_FSTAMP(3);
  const int nl = *n_long;
  for (int q = 0; q < nl; ++q) {
    const int pos = long_list[q];
    const unsigned s = (unsigned)(skeys[pos] >> 32);
    int len = 1;  // every thread finds the same length
    while (pos + len < m && (unsigned)(skeys[pos + len] >> 32) == s) ++len;
    process_long<MODE, SPLIT>(a, s, skeys + pos, len, sm);
  }
}

template <int MODE, bool GATHER = false, bool SPLIT = false>
__device__ void bucket_body(const BucketArgs& a, const int b, unsigned long long* skeys, LongLds& sm, int* long_list,
                            int& n_long, int& chunk_m, const GatherArgs* ga = nullptr) {
  unsigned* bins = reinterpret_cast<unsigned*>(skeys + kChunkCap);
  FD_FSTAMP(0);
  if (GATHER) {  // n <= kChunkCap: this bucket's keys always fit the LDS pass
    if (threadIdx.x == 0) chunk_m = 0;
    __syncthreads();
    const GatherArgs& g = *ga;
    // phase 1: every key of the batch in flight at once (kChunkCap / kBT per thread), this bucket's indices listed
    constexpr int kPer = kChunkCap / kBT;
    unsigned long long kk[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int64_t i = threadIdx.x + (int64_t)r * kBT;
      kk[r] = i < a.n ? g.src.get_key(i) : 0ull;
    }
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int64_t i = threadIdx.x + (int64_t)r * kBT;
      if (i < a.n && gather_bucket(kk[r], g.nbm) == (unsigned)b) skeys[atomicAdd(&chunk_m, 1)] = (unsigned long long)i;
    }
    if (threadIdx.x == 0) n_long = 0;  // phase 2's "a probe failed" flag (process_sorted resets it)
    __syncthreads();
    // phase 2: one listed transaction per thread: card slot (find-or-insert), prep record, its (slot, index) key in
    // the list position it came from
    const int m = chunk_m;
    for (int j = threadIdx.x; j < m; j += kBT) {
      const unsigned i = (unsigned)skeys[j];
      const Txn t = g.src.get(i);  // in flight with the probe
      const long long s = card_slot(g.keys, a.P, g.mask, g.src.get_key(i));
      store_prep(g.prep_w + i, make_prep(t, g.merchants, g.nm));
      if (s < 0) {  // table full: the batch fails (err), the key leaves the list below
        atomicOr(g.err, 1u);
        g.slot[i] = 0xffffffffu;
        // no card, so no ring: the LSTM (which runs before the error is reported) reads row i of the sequence
        // buffer instead of a stale descriptor's slot
        if (a.out.seq_desc) a.out.seq_desc[i] = kSeqMaterialized;
        skeys[j] = ~0ull;
        n_long = 1;
        continue;
      }
      g.slot[i] = (unsigned)s;
      skeys[j] = ((unsigned long long)s << 32) | (unsigned long long)i;
    }
    __threadfence_block();  // the prep records above are read back by other threads of this workgroup
    __syncthreads();
    if (n_long) {  // rare: compact the failed probes out (one thread; then every thread sees the new count)
      if (threadIdx.x == 0) {
        int w = 0;
        for (int j = 0; j < m; ++j)
          if (skeys[j] != ~0ull) skeys[w++] = skeys[j];
        chunk_m = w;
      }
      __syncthreads();
    }
    process_sorted<MODE, SPLIT>(a, skeys, chunk_m, sm, long_list, &n_long);
    __syncthreads();
    if (threadIdx.x == 0 && b == 0) a.ovf_cnt[a.par ^ 1] = 0u;  // as below: the next batch's overflow list
    return;
  }
  const unsigned long long* src = a.pairs + (size_t)b * a.C;
  // latency batches: the region's first `spec` entries are read in the same round trip as the fill count (stale
  // entries past it are dropped below), not after it
  const unsigned long long early = threadIdx.x < a.spec ? src[threadIdx.x] : 0ull;
  const unsigned m = a.fill[b];  // region (min(m, C)) + overflow entries (m - C) of this bucket
  const unsigned in_region = m < a.C ? m : a.C;
  const unsigned n_ovf = m > a.C ? a.ovf_cnt[a.par] : 0u;  // the whole list is scanned for this bucket's entries
  if (m <= (unsigned)kChunkCap) {
    if (threadIdx.x < a.spec && threadIdx.x < in_region) skeys[threadIdx.x] = early;
    for (unsigned q = threadIdx.x + a.spec; q < in_region; q += kBT) skeys[q] = src[q];
    if (n_ovf) {
      if (threadIdx.x == 0) chunk_m = (int)in_region;
      __syncthreads();
      for (unsigned q = threadIdx.x; q < n_ovf; q += kBT)
        if (a.ovf_b[q] == (unsigned)b) skeys[atomicAdd(&chunk_m, 1)] = a.ovf_key[q];
    }
    __syncthreads();
    process_sorted<MODE, SPLIT>(a, skeys, (int)m, sm, long_list, &n_long);
  } else {
    // Oversized bucket (a hot card): pass by arrival range so each pass's keys fit the LDS sort and every
    // card's transactions of pass c precede its transactions of pass c + 1 (state carried in HBM; the
    // workgroup barrier orders it: all passes run on this CU).
    const long long binw = (a.n + kMaxBins - 1) / kMaxBins;  // <= kChunkCap for n <= 16M (launch check)
    for (int q = threadIdx.x; q < kMaxBins; q += kBT) bins[q] = 0u;
    __syncthreads();
    for (unsigned q = threadIdx.x; q < in_region; q += kBT)
      atomicAdd(&bins[(unsigned)(src[q] & 0xffffffffull) / binw], 1u);
    for (unsigned q = threadIdx.x; q < n_ovf; q += kBT)
      if (a.ovf_b[q] == (unsigned)b) atomicAdd(&bins[(unsigned)(a.ovf_key[q] & 0xffffffffull) / binw], 1u);
    __syncthreads();
    {  // exclusive prefix over the bins, in place; bins[kMaxBins] = m
      constexpr int per = kMaxBins / kBT;
      unsigned v[per], sum = 0;
      for (int q = 0; q < per; ++q) {
        v[q] = bins[threadIdx.x * per + q];
        sum += v[q];
      }
      sm.rst[threadIdx.x] = (int)sum;
      __syncthreads();
      for (int d = 1; d < kBT; d <<= 1) {
        const int x = threadIdx.x >= (unsigned)d ? sm.rst[threadIdx.x - d] : 0;
        __syncthreads();
        sm.rst[threadIdx.x] += x;
        __syncthreads();
      }
      unsigned acc = threadIdx.x ? (unsigned)sm.rst[threadIdx.x - 1] : 0u;
      for (int q = 0; q < per; ++q) {
        bins[threadIdx.x * per + q] = acc;
        acc += v[q];
      }
      if (threadIdx.x == 0) bins[kMaxBins] = m;
      __syncthreads();
    }
    int lo = 0;
    while (lo < kMaxBins) {
      // the widest bin range [lo, hi) holding <= kChunkCap keys (a single bin always fits)
      int l = lo + 1, r = kMaxBins;
      while (l < r) {
        const int mid = (l + r + 1) >> 1;
        if (bins[mid] - bins[lo] <= (unsigned)kChunkCap) l = mid; else r = mid - 1;
      }
      const int hi = l;
      const unsigned i_lo = (unsigned)(lo * binw), i_hi = (unsigned)min((long long)hi * binw, a.n);
      if (threadIdx.x == 0) chunk_m = 0;
      __syncthreads();
      for (unsigned q = threadIdx.x; q < in_region; q += kBT) {
        const unsigned long long k = src[q];
        const unsigned i = (unsigned)(k & 0xffffffffull);
        if (i >= i_lo && i < i_hi) skeys[atomicAdd(&chunk_m, 1)] = k;
      }
      for (unsigned q = threadIdx.x; q < n_ovf; q += kBT) {
        if (a.ovf_b[q] != (unsigned)b) continue;
        const unsigned long long k = a.ovf_key[q];
        const unsigned i = (unsigned)(k & 0xffffffffull);
        if (i >= i_lo && i < i_hi) skeys[atomicAdd(&chunk_m, 1)] = k;
      }
      __syncthreads();
      process_sorted<MODE, SPLIT>(a, skeys, chunk_m, sm, long_list, &n_long);
      __syncthreads();
      lo = hi;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // the next batch's counters (it runs after this launch on the same stream)
    a.fill[b] = 0u;
    if (b == 0) a.ovf_cnt[a.par ^ 1] = 0u;  // the next batch's overflow list (this batch's is reset by the next)
  }
}

// One workgroup per bucket
template <int MODE>
__global__ void __launch_bounds__(kBT) feat_bucket_kernel(BucketArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long skeys[];  // kChunkCap keys | kMaxBins + 1 bins
  __shared__ LongLds sm;
  __shared__ int long_list[kChunkCap / (kSegLong + 1) + 1];
  __shared__ int n_long, chunk_m;
  FD_TL(g_tl_feat, 1, 0);
  bucket_body<MODE>(a, blockIdx.x, skeys, sm, long_list, n_long, chunk_m);
  FD_TL(g_tl_feat, 1, 3);
}

// The same with the slot pass folded in (BucketArgs::gather; a kernel of its own so the others keep their registers)
template <int MODE>
__global__ void __launch_bounds__(kBT) feat_bucket_gather_kernel(BucketArgs a, GatherArgs g) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long skeys[];
  __shared__ LongLds sm;
  __shared__ int long_list[kChunkCap / (kSegLong + 1) + 1];
  __shared__ int n_long, chunk_m;
  FD_TL(g_tl_feat, 1, 0);
  bucket_body<MODE, true>(a, blockIdx.x, skeys, sm, long_list, n_long, chunk_m, &g);
  FD_TL(g_tl_feat, 1, 3);
}

// The bucket kernel's LDS working set, in global memory (one per bucket) for the lean kernel's slow path
struct BucketScratch {
  unsigned long long keys[kChunkCap + (kMaxBins + 1 + 1) / 2];  // keys | bin prefix sums (kBucketLds)
  LongLds sm;
  int long_list[kChunkCap / (kSegLong + 1) + 1];
  int n_long, chunk_m;
};

// Lean form of the bucket kernel for the pipelined stream (fd_score_batch_pipelined): 4 KiB of LDS, so its
// workgroups fit beside a running ensemble_kernel workgroup (148 KiB of the CU's 160) and batch i+1's card work
// overlaps batch i's forests. The common bucket — at most kLeanCap keys, none in the overflow list, every card
// segment short — is sorted and walked in LDS; any other bucket (a hot card) takes the full bucket kernel's
// code with its working set in a per-bucket global scratch block (L1/L2-resident; same results, no launch
// that would have to wait for a whole CU).
constexpr int kLeanCap = 256;  // a bucket of ~128 keys on average; a larger one takes the slow path
// Lean grouping (engine option lean_group, default 2): the bucket's keys need only be grouped by card, each card's
// transactions in arrival order — not sorted. Each key's card slot goes into a 256-entry LDS hash table (atomic CAS
// insert, then an atomic count per card); a card of one transaction (nearly all at 64 k over 100 M cards) is
// processed at once, a card of several by the thread whose key inserted it, which gathers and orders that card's
// arrival indices. Two LDS atomics per key instead of the sort's ~m / 2 16-B LDS reads, which queue behind the
// fused ensemble kernel's LDS traffic on the same CU (lean phases, profiles/r05/lean_phases).
constexpr int kHashCap = 256;
constexpr unsigned kHashEmpty = 0xffffffffu;
constexpr int kLeadBit = 1 << 30;  // rk[pos]: the table entry of the key at pos, | kLeadBit where it inserted the card
static_assert(kHashCap == kBT, "one table entry per thread at initialisation");

template <int MODE, bool SPLIT>
__global__ void __launch_bounds__(kBT) feat_bucket_lean_kernel(BucketArgs a, BucketScratch* scratch) {
  // 6 KiB: beside a running ensemble_kernel workgroup (148 of the CU's 160 KiB) with room to spare
  __shared__ __attribute__((aligned(16))) unsigned long long skeys[kLeanCap];
  __shared__ int rk[kBT];  // split sort: partial ranks; hash grouping: each position's table entry (+ kLeadBit)
  __shared__ unsigned hslot[kHashCap], hcnt[kHashCap];
  __shared__ unsigned pool[kHashCap];  // the arrival indices of several-transaction cards, in order
  __shared__ int any_long, pool_n;
  if (a.prio) __builtin_amdgcn_s_setprio(2);
  FD_FSTAMP(0);
  const int b = blockIdx.x;
  const int t = (int)threadIdx.x;
  const unsigned m = a.fill[b];
  if (t == 0) any_long = 0, pool_n = 0;
  bool slow = m > (unsigned)kLeanCap || m > a.C;
  const bool hashed = a.lean_group == 2;
  if (!slow) {
    const unsigned long long* src = a.pairs + (size_t)b * a.C;
    for (unsigned q = threadIdx.x; q < m; q += kBT) skeys[q] = src[q];
    rk[t] = 0;
    if (hashed) {
      hslot[t] = kHashEmpty;
      hcnt[t] = 0u;
    }
    __syncthreads();
    FD_FSTAMP(1);
    if (hashed) {
      if (t < (int)m) {
        const unsigned s = (unsigned)(skeys[t] >> 32);
        unsigned h = (unsigned)(mix64(s) >> 32) & (kHashCap - 1);
        unsigned old;
        for (;;) {
          old = atomicCAS(&hslot[h], kHashEmpty, s);
          if (old == kHashEmpty || old == s) break;
          h = (h + 1) & (kHashCap - 1);
        }
        rk[t] = (int)h | (old == kHashEmpty ? kLeadBit : 0);
        if (atomicAdd(&hcnt[h], 1u) >= (unsigned)kSegLong) any_long = 1;  // a card past kSegLong transactions
      }
    } else {
      if (m > 1) {
        if (a.lean_group == 1) rank_sort_split(skeys, (int)m, rk);
        else rank_sort(skeys, (int)m);
      }
      for (int pos = t; pos < (int)m; pos += kBT) {
        const unsigned s = (unsigned)(skeys[pos] >> 32);
        if (pos > 0 && (unsigned)(skeys[pos - 1] >> 32) == s) continue;
        if (pos + kSegLong < (int)m && (unsigned)(skeys[pos + kSegLong] >> 32) == s) any_long = 1;
      }
    }
    __syncthreads();
    slow = any_long != 0;
    FD_FSTAMP(2);
  }
  if (slow) {
    BucketScratch& w = scratch[b];
    bucket_body<MODE, false, SPLIT>(a, b, w.keys, w.sm, w.long_list, w.n_long, w.chunk_m);
    return;
  }
  if (hashed) {
    for (int pos = first_pos(a.spread); pos < (int)m; pos += kBT) {
      const unsigned long long k = skeys[pos];
      const unsigned s = (unsigned)(k >> 32);
      const int e = rk[pos];
      const unsigned c = hcnt[e & (kHashCap - 1)];
      if (c == 1u) {
        process_short<MODE, SPLIT>(a, s, skeys + pos, 1);
        continue;
      }
      if (!(e & kLeadBit)) continue;  // the thread whose key inserted the card processes all of its transactions
      const int base = atomicAdd(&pool_n, (int)c);
      int w = 0;
      for (int q = 0; q < (int)m; ++q) {
        const unsigned long long x = skeys[q];
        if ((unsigned)(x >> 32) == s) pool[base + w++] = (unsigned)x;
      }
      for (int x = 1; x < w; ++x) {  // arrival order
        const unsigned v = pool[base + x];
        int y = x - 1;
        while (y >= 0 && pool[base + y] > v) {
          pool[base + y + 1] = pool[base + y];
          --y;
        }
        pool[base + y + 1] = v;
      }
      process_short<MODE, SPLIT>(a, s, pool + base, w);
    }
  } else {
    for (int pos = first_pos(a.spread); pos < (int)m; pos += kBT) {
      const unsigned s = (unsigned)(skeys[pos] >> 32);
      if (pos > 0 && (unsigned)(skeys[pos - 1] >> 32) == s) continue;
      int len = 1;
      while (pos + len < (int)m && (unsigned)(skeys[pos + len] >> 32) == s) ++len;
      process_short<MODE, SPLIT>(a, s, skeys + pos, len);
    }
  }
#ifdef FD_FOREST_PROFILE
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096)
    g_fprof[blockIdx.x * 8 + 4 + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memtime();
#endif
  FD_FSTAMP(3);
  if (t == 0) {  // the next batch's counters (it runs after this launch on the stream)
    a.fill[b] = 0u;
    if (b == 0) a.ovf_cnt[a.par ^ 1] = 0u;
  }
}

__global__ void __launch_bounds__(256) count_cards_kernel(CardPages P, int64_t cap, unsigned long long* out) {
  unsigned long long c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x)
    c += (P.hdr(i)->key != 0ull);
  atomicAdd(out, c);
}

// zero every slot's header (the rings need no clearing: a header with ring_n 0 holds no events); 16 B per thread
__global__ void __launch_bounds__(256) clear_headers_kernel(CardPages P, int64_t cap) {
  const int64_t words = cap * (kCardHeaderBytes / 16);
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < words; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = t / (kCardHeaderBytes / 16);
    reinterpret_cast<uint4*>(P.hdr(s))[t - s * (kCardHeaderBytes / 16)] = make_uint4(0u, 0u, 0u, 0u);
  }
}

// ------------------------------------------------------------------------------------------------
// Full FeatureExtractor map (a3) and the Flink rule scores ((f) rank 2), elementwise per transaction
// after feat_bucket (same batch: the card slots of feat_slot, the raw features of feat_bucket).
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

__global__ void __launch_bounds__(256) feat_ext_kernel(CardPages P,
                                                       const UserExt* __restrict__ uext,
                                                       const Merchant* __restrict__ merchants,
                                                       const MerchExt* __restrict__ mext, int nm, int n_mext,
                                                       int64_t n,
                                                       TxnSrc t, CtxArgs c, const unsigned* __restrict__ slot,
                                                       const double* __restrict__ raw, const double* __restrict__ vel5,
                                                       const unsigned char* __restrict__ vocab, double tp_threshold,
                                                       double* __restrict__ fmap, fd_rule_scores* __restrict__ rules) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* r = raw + (size_t)i * FD_RAW_FEATURES;
  const unsigned s = slot[i];
  const bool has_slot = s != 0xffffffffu;
  const CardHeader h = has_slot ? *P.hdr(s) : CardHeader{};
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

__global__ void __launch_bounds__(256) users_ext_load_kernel(CardPages P, unsigned long long* K, UserExt* U, long long mask, int64_t n,
                                                             const unsigned long long* key, const UserExt* src,
                                                             unsigned* err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long s = card_slot(K, P, mask, key[i]);
  if (s < 0) {
    atomicOr(err, 1u);
    return;
  }
  UserExt u = src[i];
  u.loaded = 1;
  U[s] = u;
}

unsigned grid_for(int64_t n) { return (unsigned)((n + 255) / 256); }

// buckets of a batch of n: NB = the power of two >= n / T, so a 256-thread bucket workgroup holds ~T cards: one
// segment per thread (a second round would double the dependent-load chain). T = 128 for throughput batches; a
// latency batch (< 8192 transactions) would leave most CUs idle with 128 (8 workgroups for 1 k), so it takes 16
// per bucket: 64 workgroups, each with a 16-key rank sort instead of 128 (engine option bucket_keys overrides)
unsigned buckets_for(int64_t n, int64_t cap, int keys) {
  // auto: 8 transactions per bucket up to 2048 (config 5, 1 k: 0.0591 -> 0.0582 ms), 16 below 8192, else 128
  const int64_t T = keys > 0 ? keys : (n <= 2048 ? 8 : n < 8192 ? 16 : 128);
  unsigned nb = 1;
  while ((int64_t)nb * T < n && nb < (unsigned)kMaxBuckets && (int64_t)nb < cap) nb <<= 1;
  return nb;
}

}  // namespace

void state_init(Engine& e, const fd_state_params& p) {
  FD_REQUIRE(p.capacity > 0 && p.capacity <= (1ll << 31), FD_ERR_INVALID_ARG, "capacity must be in [1, 2^31]");
  FD_REQUIRE(p.window_mode == FD_WINDOW_REDIS_COMPAT || p.window_mode == FD_WINDOW_SLIDING, FD_ERR_INVALID_ARG,
             "unknown window_mode");
  FD_REQUIRE(p.ring_k >= 1 && p.ring_k <= kMaxK, FD_ERR_INVALID_ARG, "ring_k must be in [1, 64]");
  FD_REQUIRE(p.seq_len >= 0 && p.seq_len <= FD_MAX_SEQ_LEN, FD_ERR_INVALID_ARG, "seq_len must be in [0, 16]");
  int64_t cap = 1;
  while (cap < p.capacity) cap <<= 1;
  CardStore& st = e.state;
  st.cap = cap;
  st.mode = p.window_mode;
  st.K = p.window_mode == FD_WINDOW_SLIDING ? p.ring_k : 1;
  st.page_bytes = kCardHeaderBytes + (st.mode == FD_WINDOW_SLIDING ? (long long)st.K * (long long)sizeof(RingEvent) : 0);
  if (st.pages.bytes < (size_t)cap * st.page_bytes) st.pages.release();  // free before the keys grow (peak HBM)
  st.keys.ensure((size_t)cap * sizeof(unsigned long long));
  st.pages.ensure((size_t)cap * st.page_bytes);
  st.S = p.seq_len;
  if (st.S) st.seq.ensure((size_t)cap * st.S * kSeqInput * sizeof(float));
  // extended user profiles are per slot: a re-initialised table starts without them (fd_state_load_users_ext
  // allocates for the new capacity)
  st.uext.release();
  st.err.ensure(16);
  st.sat.ensure(8);
  for (auto& g : st.gs) {
    g.bucket_fill.ensure(kMaxBuckets * sizeof(unsigned));
    g.ovf_cnt.ensure(2 * sizeof(unsigned));
  }
  st.ready = true;
  state_clear(e);
}

void state_clear(Engine& e) {
  CardStore& st = e.state;
  FD_REQUIRE(st.ready, FD_ERR_NOT_LOADED, "card state not initialised (fd_state_init)");
  hipLaunchKernelGGL(clear_headers_kernel, dim3(4096), dim3(256), 0, e.stream, st.view(), (int64_t)st.cap);
  FD_HIP(hipGetLastError());
  FD_HIP(hipMemsetAsync(st.keys.ptr, 0, (size_t)st.cap * sizeof(unsigned long long), e.stream));
  if (st.uext.ptr) FD_HIP(hipMemsetAsync(st.uext.ptr, 0, (size_t)st.cap * sizeof(UserExt), e.stream));
  FD_HIP(hipMemsetAsync(st.err.ptr, 0, 16, e.stream));
  FD_HIP(hipMemsetAsync(st.sat.ptr, 0, 8, e.stream));
  for (auto& g : st.gs) {
    FD_HIP(hipMemsetAsync(g.bucket_fill.ptr, 0, kMaxBuckets * sizeof(unsigned), e.stream));
    FD_HIP(hipMemsetAsync(g.ovf_cnt.ptr, 0, 2 * sizeof(unsigned), e.stream));
  }
  FD_HIP(hipStreamSynchronize(e.stream));
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
  hipLaunchKernelGGL(count_cards_kernel, dim3(1024), dim3(256), 0, e.stream, st.view(),
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
  hipLaunchKernelGGL(users_load_kernel, dim3(grid_for(u.n)), dim3(256), 0, e.stream, st.view(),
                     st.keys.as<unsigned long long>(),
                     (long long)(st.cap - 1), u.n, k.as<const unsigned long long>(), a.as<const double>(),
                     g.as<const int>(), f.as<const unsigned long long>(), st.err.as<unsigned>());
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

namespace {

// The grouping launch (feat_slot) + the bucket kernel over any transaction source.
// lean: the pipelined stream's bucket pass (feat_bucket_lean_kernel: fits beside the ensemble kernel)
// set: the scratch set (CardStore::gs); before_buckets: an event the bucket pass waits for (the previous batch's
// card updates, pipelined stream) while the slot pass runs ahead
void launch_grouped(Engine& e, const TxnSrc& src, int64_t n, float* d_vec, double* d_raw, float* d_seq,
                    double* d_vel5, hipStream_t stream = nullptr, bool lean = false, int set = 0,
                    hipEvent_t before_buckets = nullptr, int compact = 0,
                    unsigned long long* d_seq_desc = nullptr) {
  CardStore& st = e.state;
  CardStore::GroupScratch& g = st.gs[set];
  const hipStream_t s = stream ? stream : e.stream;
  // split rows (compact 2): RowA at d_vec, RowB after the batch's n RowAs (32 B each); the pipelined stream's lean
  // bucket pass only, and no LSTM history (seq_step reads the raw features the split card work does not form)
  const bool split = compact == 2;
  FD_REQUIRE(!split || (lean && st.S == 0 && !d_raw && !d_seq && !d_vel5), FD_ERR_INVALID_ARG,
             "internal: split rows need the lean bucket pass and no raw / sequence outputs");
  uint4* row_a = split ? reinterpret_cast<uint4*>(d_vec) : nullptr;
  float* vec_out = split ? d_vec + (size_t)n * 8 : d_vec;
  FD_REQUIRE(n <= (int64_t)kMaxBins * kChunkCap, FD_ERR_INVALID_ARG, "micro-batch larger than 16M transactions");
  g.slot.ensure((size_t)n * 4);
  g.prep.ensure((size_t)n * sizeof(Prep));
  if (st.merchants.ptr == nullptr) st.merchants.ensure(16);
  const unsigned nb = buckets_for(n, st.cap, st.bucket_keys);
  // bucket capacity: 4x the mean (Poisson tail beyond it is negligible for hashed cards; skewed batches spill
  // to the overflow list), a multiple of 64
  const unsigned C = (unsigned)std::max<int64_t>(512, ((4 * ((n + nb - 1) / nb)) + 63) / 64 * 64);
  g.pairs.ensure((size_t)nb * C * 8);
  g.ovf_key.ensure((size_t)n * 8);
  g.ovf_b.ensure((size_t)n * 4);
  const int par = g.batch_parity;
  g.batch_parity ^= 1;
  // the slot pass on the engine's slot stream when the pipelined step set one (option slot_stream), else on s
  const hipStream_t ss = e.slot_pass_stream ? e.slot_pass_stream : s;
  // latency batches: the slot pass inside the bucket kernel (no slot launch; its probes in the card loop's launch)
  const bool gather = st.slot_gather && !lean && n <= (int64_t)kChunkCap && ss == s;  // (never with split: lean)
  Engine::Timed* ev = e.timing ? e.next_event_pair(FD_TIMING_FEATURES) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, ss));
  if (!gather) hipLaunchKernelGGL(feat_slot_kernel, dim3((unsigned)((n + kST - 1) / kST)), dim3(kST), 2 * nb * sizeof(unsigned),
                     ss, st.view(), st.keys.as<unsigned long long>(), (long long)(st.cap - 1), n, src,
                     st.merchants.as<const Merchant>(), (int)st.n_merchants, nb - 1, C, g.slot.as<unsigned>(),
                     g.prep.as<Prep>(), g.bucket_fill.as<unsigned>(), g.pairs.as<unsigned long long>(),
                     g.ovf_cnt.as<unsigned>() + par, g.ovf_key.as<unsigned long long>(), g.ovf_b.as<unsigned>(),
                     st.err.as<unsigned>(), lean && st.slot_prio ? 1 : 0, row_a);
  FD_HIP(hipGetLastError());
  if (ss != s) {
    FD_HIP(hipEventRecord(e.slot_pass_ev, ss));
    FD_HIP(hipStreamWaitEvent(s, e.slot_pass_ev, 0));
  }
  if (before_buckets) FD_HIP(hipStreamWaitEvent(s, before_buckets, 0));
  if (ev && ss != s) {  // timed in two parts: the slot pass on ss, the bucket pass from here on s
    if (!ev->c) {
      FD_HIP(hipEventCreateWithFlags(&ev->c, hipEventDisableSystemFence));
      FD_HIP(hipEventCreateWithFlags(&ev->d, hipEventDisableSystemFence));
    }
    FD_HIP(hipEventRecord(ev->b, ss));
    FD_HIP(hipEventRecord(ev->c, s));
    ev->split = true;
  }
  static bool attrs = false;
  if (!attrs) {  // > 48 KiB of dynamic LDS
    FD_HIP(hipFuncSetAttribute((const void*)feat_bucket_kernel<FD_WINDOW_SLIDING>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBucketLds));
    FD_HIP(hipFuncSetAttribute((const void*)feat_bucket_kernel<FD_WINDOW_REDIS_COMPAT>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBucketLds));
    FD_HIP(hipFuncSetAttribute((const void*)feat_bucket_gather_kernel<FD_WINDOW_SLIDING>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBucketLds));
    FD_HIP(hipFuncSetAttribute((const void*)feat_bucket_gather_kernel<FD_WINDOW_REDIS_COMPAT>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBucketLds));
    attrs = true;
  }
  BucketArgs a{};
  a.P = st.view();
  a.K = st.K;
  a.n = n;
  a.prep = g.prep.as<const Prep>();
  a.out = Outputs{vec_out, d_raw, d_vel5, d_seq, st.S ? st.seq.as<float>() : nullptr, st.S, d_seq_desc,
                  st.mode == FD_WINDOW_SLIDING ? st.sat.as<unsigned long long>() : nullptr, st.K, compact != 0};
  a.fill = g.bucket_fill.as<unsigned>();
  a.pairs = g.pairs.as<const unsigned long long>();
  a.C = C;
  a.ovf_cnt = g.ovf_cnt.as<unsigned>();
  a.par = par;
  a.ovf_key = g.ovf_key.as<const unsigned long long>();
  a.ovf_b = g.ovf_b.as<const unsigned>();
  // early region reads (latency batches): 4x the mean bucket fill covers the Poisson tail, at most one per thread
  // spread measured: config 4 (64 k, ~128 keys per bucket: 2 full waves -> 4 half waves) 0.0967 -> 0.0942 ms per
  // step; config 5 (1 k, 16 keys: 1 wave -> 4 waves of 4 lanes) the card loop 2x slower (profiles/r04/config5)
  a.spread = st.bucket_spread && n >= 8192;
  a.prio = lean && st.feat_prio;
  a.lean_group = st.lean_group;
  a.spec = n < 8192 ? (unsigned)std::min<int64_t>({(int64_t)kBT, (int64_t)C, 4 * ((n + nb - 1) / nb)}) : 0u;
  GatherArgs ga{};
  if (gather) {
    ga.nbm = nb - 1;
    ga.src = src;
    ga.keys = st.keys.as<unsigned long long>();
    ga.mask = (long long)(st.cap - 1);
    ga.merchants = st.merchants.as<const Merchant>();
    ga.nm = (int)st.n_merchants;
    ga.prep_w = g.prep.as<Prep>();
    ga.slot = g.slot.as<unsigned>();
    ga.err = st.err.as<unsigned>();
  }
  const size_t lds = kBucketLds;
  if (lean) {
    st.bucket_scr.ensure((size_t)nb * sizeof(BucketScratch));
    BucketScratch* scr = st.bucket_scr.as<BucketScratch>();
    if (split) {
      if (st.mode == FD_WINDOW_SLIDING)
        hipLaunchKernelGGL((feat_bucket_lean_kernel<FD_WINDOW_SLIDING, true>), dim3(nb), dim3(kBT), 0, s, a, scr);
      else
        hipLaunchKernelGGL((feat_bucket_lean_kernel<FD_WINDOW_REDIS_COMPAT, true>), dim3(nb), dim3(kBT), 0, s, a, scr);
    } else if (st.mode == FD_WINDOW_SLIDING) {
      hipLaunchKernelGGL((feat_bucket_lean_kernel<FD_WINDOW_SLIDING, false>), dim3(nb), dim3(kBT), 0, s, a, scr);
    } else {
      hipLaunchKernelGGL((feat_bucket_lean_kernel<FD_WINDOW_REDIS_COMPAT, false>), dim3(nb), dim3(kBT), 0, s, a, scr);
    }
  } else if (gather) {
    if (st.mode == FD_WINDOW_SLIDING)
      hipLaunchKernelGGL(feat_bucket_gather_kernel<FD_WINDOW_SLIDING>, dim3(nb), dim3(kBT), lds, s, a, ga);
    else
      hipLaunchKernelGGL(feat_bucket_gather_kernel<FD_WINDOW_REDIS_COMPAT>, dim3(nb), dim3(kBT), lds, s, a, ga);
  } else if (st.mode == FD_WINDOW_SLIDING) {
    hipLaunchKernelGGL(feat_bucket_kernel<FD_WINDOW_SLIDING>, dim3(nb), dim3(kBT), lds, s, a);
  } else {
    hipLaunchKernelGGL(feat_bucket_kernel<FD_WINDOW_REDIS_COMPAT>, dim3(nb), dim3(kBT), lds, s, a);
  }
  FD_HIP(hipGetLastError());
  if (ev) FD_HIP(hipEventRecord(ev->split ? ev->d : ev->b, s));
}

}  // namespace

void launch_features(Engine& e, const fd_txn_batch& t, int64_t n, float* d_vec, double* d_raw, float* d_seq,
                     double* d_vel5, hipStream_t stream, bool lean, int set, hipEvent_t before_buckets, int compact,
                     unsigned long long* d_seq_desc) {
  CardStore& st = e.state;
  FD_REQUIRE(st.ready, FD_ERR_NOT_LOADED, "card state not initialised (fd_state_init)");
  FD_REQUIRE(d_vec != nullptr, FD_ERR_INVALID_ARG, "null vector output");
  FD_REQUIRE(d_seq == nullptr || st.S > 0, FD_ERR_INVALID_ARG, "sequence output needs fd_state_params.seq_len > 0");
  FD_REQUIRE(n >= 0 && n < (1ll << 31), FD_ERR_INVALID_ARG, "batch size out of range");
  if (n == 0) return;
  FD_REQUIRE(t.card_key && t.ts_ms && t.amount_cents && t.merchant && t.device_fp && t.ip_class && t.hour &&
                 t.weekend,
             FD_ERR_INVALID_ARG, "incomplete transaction batch");
  TxnSrc src{reinterpret_cast<const unsigned long long*>(t.card_key), reinterpret_cast<const long long*>(t.ts_ms),
             reinterpret_cast<const long long*>(t.amount_cents), reinterpret_cast<const int*>(t.merchant),
             reinterpret_cast<const unsigned long long*>(t.device_fp), t.ip_class, t.hour, t.weekend, nullptr};
  FD_REQUIRE(d_seq_desc == nullptr || d_seq != nullptr, FD_ERR_INVALID_ARG, "sequence descriptors need the buffer");
  launch_grouped(e, src, n, d_vec, d_raw, d_seq, d_vel5, stream, lean, set, before_buckets, compact, d_seq_desc);
}

void launch_features_records(Engine& e, const void* d_records, int64_t n, float* d_vec, float* d_seq,
                             hipStream_t stream, bool lean, int set, hipEvent_t before_buckets, int compact) {
  CardStore& st = e.state;
  FD_REQUIRE(st.ready, FD_ERR_NOT_LOADED, "card state not initialised (fd_state_init)");
  FD_REQUIRE(d_vec != nullptr && (n == 0 || d_records != nullptr), FD_ERR_INVALID_ARG, "null records / output");
  FD_REQUIRE(d_seq == nullptr || st.S > 0, FD_ERR_INVALID_ARG, "sequence output needs fd_state_params.seq_len > 0");
  FD_REQUIRE(n >= 0 && n < (1ll << 31), FD_ERR_INVALID_ARG, "batch size out of range");
  if (n == 0) return;
  TxnSrc src{};
  src.rec = static_cast<const RouteRecord*>(d_records);
  launch_grouped(e, src, n, d_vec, nullptr, d_seq, nullptr, stream, lean, set, before_buckets, compact);
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
  hipLaunchKernelGGL(users_ext_load_kernel, dim3(grid_for(u.n)), dim3(256), 0, e.stream, st.view(),
                     st.keys.as<unsigned long long>(),
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
  TxnSrc a{reinterpret_cast<const unsigned long long*>(t.card_key), reinterpret_cast<const long long*>(t.ts_ms),
           reinterpret_cast<const long long*>(t.amount_cents), reinterpret_cast<const int*>(t.merchant),
           reinterpret_cast<const unsigned long long*>(t.device_fp), t.ip_class, t.hour, t.weekend, nullptr};
  CtxArgs ca{c.geo_lat, c.geo_lon, c.merchant_lat, c.merchant_lon, c.payment_method, c.transaction_type,
             c.card_type, c.user_agent_flag, c.fraud_score};
  hipLaunchKernelGGL(feat_ext_kernel, dim3(grid_for(n)), dim3(256), 0, e.stream, st.view(),
                     st.uext.ptr ? st.uext.as<const UserExt>() : nullptr,
                     st.merchants.as<const Merchant>(), st.mext.ptr ? st.mext.as<const MerchExt>() : nullptr,
                     (int)st.n_merchants, (int)st.n_mext, n, a, ca,
                     st.gs[0].slot.as<const unsigned>(), raw, vel5, st.vocab.as<const unsigned char>(), st.tp_threshold,
                     d_fmap, d_rules);
  FD_HIP(hipGetLastError());
}

#ifdef FD_FOREST_PROFILE
extern "C" __attribute__((visibility("default"))) int fd_debug_feat_profile2(unsigned long long* out, int n) {
#ifdef FD_FOREST_PROFILE
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fprof2), sizeof(unsigned long long) * (size_t)n);
#else
  (void)out, (void)n;
  return -1;
#endif
}
extern "C" __attribute__((visibility("default"))) int fd_debug_feat_profile(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fprof), sizeof(unsigned long long) * (size_t)n);
}
extern "C" __attribute__((visibility("default"))) int fd_debug_tl_feat(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tl_feat), sizeof(g_tl_feat));
}
#endif

}  // namespace fd
