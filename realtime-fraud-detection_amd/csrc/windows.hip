// windows.hip — the Flink window aggregates of the feature half on the device.
//
// Reference: fl/windows/WindowProcessor.java (fl/ = services/flink-jobs/src/main/java/com/frauddetection/)
//   processUserVelocity      keyBy(userId), SlidingEventTimeWindows(5 min, 1 min)      :36-48
//   processMerchantPatterns  keyBy(merchantId), TumblingEventTimeWindows(1 h)         :54-66
//   watermarks               forBoundedOutOfOrderness(10 s)                              :40-43, 58-61
//   UserVelocityAggregateFunction (count, total, fraud, high-risk, distinct merchants and payment
//     methods, first/last event time, avg, fraud rate, velocity score)                  :248-352
//   MerchantAggregateFunction (+ fraud amount, distinct users, population stddev, risk score) :357-484
// (The session / geographic / fraud-pattern / high-frequency / amount-cluster aggregate functions the
// job file names are not implemented in the reference source, so they are not here either.)
//
// Micro-batch semantics (declared, DESIGN.md "Windows"): the watermark W = max event time seen - 10 s - 1
// (Flink's BoundedOutOfOrderness) advances once per micro-batch, after the batch's events are added;
// a window fires when W passes its last millisecond (EventTimeTrigger), with every event of its range
// that arrived before it fired (an event arriving after its window fired is late and dropped for that
// window, as Flink does with allowed lateness 0). Amount sums are exact integer cents; the merchant
// stddev is the exact integer-moment formula sqrt((n S2 - S1^2) / n^2) / 100.
//
// Per micro-batch (fd_windows_step_device):
//   win_append   : every transaction -> a 40-B event in the user log and in the merchant log (HBM);
//                  batch max event time (atomic max)
//   win_select_* : events -> (window key, event) pairs for the windows firing now
//                  (user key: slot | minute | merchant+1, merchant key: merchant | hour | user slot)
//   radix sort   : rocPRIM radix_sort_pairs on the 64-bit keys
//   win_reduce_* : one thread per window segment (contiguous after the sort): counts, cents, distinct
//                  merchants / users (key changes), payment-method bitmask, min / max event time -> result
//   win_compact  : drop events no open window can still contain
#include <algorithm>
#include <cstring>
#include <numeric>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "fd_internal.h"

namespace fd {
namespace {

struct __attribute__((aligned(8))) WinEvent {  // 40 B
  long long ts;
  long long cents;
  unsigned long long key;  // card key (result identity)
  unsigned slot;           // card-table slot (sort identity)
  int merchant;            // -1 = unknown (Java: null merchantId, a distinct value)
  unsigned char pm;        // payment-method code, 255 = null
  unsigned char fraud;     // Transaction.isFraud
  unsigned char high;      // Transaction.fraudScore > 0.7
  unsigned char pad[5];
};
static_assert(sizeof(WinEvent) == 40, "WinEvent must be 40 B");

constexpr long long kUserSize = 300000, kUserSlide = 60000, kMerchSize = 3600000;


// the card table's slot of a key (insert when absent, as feat_assign does)

__device__ __forceinline__ long long floor_div(long long a, long long b) {
  long long q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}

__global__ void __launch_bounds__(256) win_append_kernel(unsigned long long* card_keys, CardPages pages,
                                                         long long mask, int64_t n, const unsigned long long* key,
                                                         const long long* ts, const long long* cents,
                                                         const int* merchant, const unsigned char* pm,
                                                         const unsigned char* fraud, const double* fscore,
                                                         WinEvent* ulog, WinEvent* mlog, unsigned long long* max_ts,
                                                         unsigned long long* min_ts, unsigned* err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long s = card_slot(card_keys, pages, mask, key[i]);
  if (s < 0) {
    atomicOr(err, 1u);
    return;
  }
  WinEvent e;
  e.ts = ts[i];
  e.cents = cents[i];
  e.key = key[i];
  e.slot = (unsigned)s;
  e.merchant = merchant[i];
  e.pm = pm ? pm[i] : 255;
  e.fraud = fraud ? (fraud[i] != 0) : 0;
  const double fs = fscore ? fscore[i] : __builtin_nan("");
  e.high = (!isnan(fs) && fs > 0.7) ? 1 : 0;
  for (int q = 0; q < 5; ++q) e.pad[q] = 0;
  ulog[i] = e;
  mlog[i] = e;
  const unsigned long long biased = (unsigned long long)e.ts ^ 0x8000000000000000ull;  // order-preserving
  atomicMax(max_ts, biased);
  atomicMin(min_ts, biased);
}

// user windows [start, start + 5 min), start = k * 1 min; an event is in the 5 windows with
// start in (ts - 5 min, ts]; fires when W_prev < end - 1 <= W_new
__global__ void __launch_bounds__(256) win_select_user_kernel(const WinEvent* __restrict__ log, int64_t n,
                                                              long long w_prev, long long w_new, long long base_min,
                                                              unsigned long long* keys, unsigned* vals,
                                                              unsigned* count, unsigned cap, unsigned* err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const WinEvent e = log[i];
  const long long last = floor_div(e.ts, kUserSlide);
  for (int j = 0; j < (int)(kUserSize / kUserSlide); ++j) {
    const long long m = last - j;
    const long long end = m * kUserSlide + kUserSize;
    if (end - 1 > w_prev && end - 1 <= w_new) {
      const long long rel = m - base_min;
      if (rel < 0 || rel >= (1ll << 16) || e.merchant + 1 >= (1 << 17)) {
        atomicOr(err, 4u);
        continue;
      }
      const unsigned p = atomicAdd(count, 1u);
      if (p >= cap) {
        atomicOr(err, 2u);
        continue;
      }
      keys[p] = ((unsigned long long)e.slot << 33) | ((unsigned long long)rel << 17) |
                (unsigned long long)(unsigned)(e.merchant + 1);
      vals[p] = (unsigned)i;
    }
  }
}

__global__ void __launch_bounds__(256) win_select_merchant_kernel(const WinEvent* __restrict__ log, int64_t n,
                                                                  long long w_prev, long long w_new,
                                                                  long long base_hour, unsigned long long* keys,
                                                                  unsigned* vals, unsigned* count, unsigned cap,
                                                                  unsigned* err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const WinEvent e = log[i];
  if (e.merchant < 0) return;  // keyBy(merchantId) on a null id: not aggregated (declared)
  const long long hr = floor_div(e.ts, kMerchSize);
  const long long end = hr * kMerchSize + kMerchSize;
  if (!(end - 1 > w_prev && end - 1 <= w_new)) return;
  const long long rel = hr - base_hour;
  if (rel < 0 || rel >= (1ll << 16) || e.merchant >= (1 << 17)) {
    atomicOr(err, 4u);
    return;
  }
  const unsigned p = atomicAdd(count, 1u);
  if (p >= cap) {
    atomicOr(err, 2u);
    return;
  }
  keys[p] = ((unsigned long long)e.merchant << 47) | ((unsigned long long)rel << 31) | (unsigned long long)e.slot;
  vals[p] = (unsigned)i;
}

__global__ void __launch_bounds__(256) win_reduce_user_kernel(const WinEvent* __restrict__ log,
                                                              const unsigned long long* __restrict__ keys,
                                                              const unsigned* __restrict__ vals, unsigned n,
                                                              long long base_min, fd_user_window* out,
                                                              unsigned* out_count, unsigned cap, unsigned* err) {
#pragma clang fp contract(off)
  const unsigned p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const unsigned long long seg = keys[p] >> 17;
  if (p > 0 && (keys[p - 1] >> 17) == seg) return;  // not a segment head
  long long cents = 0, first = 0, last = 0;
  int cnt = 0, fraud = 0, high = 0, uniq_m = 0;
  unsigned long long pm[4] = {0, 0, 0, 0};
  unsigned long long prev_m = ~0ull;
  unsigned long long ukey = 0;
  for (unsigned q = p; q < n && (keys[q] >> 17) == seg; ++q) {
    const WinEvent e = log[vals[q]];
    ukey = e.key;
    cnt += 1;
    cents += e.cents;
    fraud += e.fraud;
    high += e.high;
    const unsigned long long mk = keys[q] & 0x1FFFFull;
    if (mk != prev_m) {
      uniq_m += 1;
      prev_m = mk;
    }
    if (e.pm != 255) pm[e.pm >> 6] |= 1ull << (e.pm & 63);
    if (first == 0 || e.ts < first) first = e.ts;  // accumulator.windowStart (0 = unset)
    if (e.ts > last) last = e.ts;                  // accumulator.windowEnd
  }
  const long long m = (long long)((seg) & 0xFFFFull) + base_min;
  fd_user_window r{};
  r.user_key = ukey;
  r.window_start = m * kUserSlide;
  r.window_end = m * kUserSlide + kUserSize;
  r.first_ts = first;
  r.last_ts = last;
  r.count = cnt;
  r.fraud_count = fraud;
  r.high_risk_count = high;
  r.unique_merchants = uniq_m;
  r.unique_payment_methods = __popcll(pm[0]) + __popcll(pm[1]) + __popcll(pm[2]) + __popcll(pm[3]);
  r.total_amount = (double)cents / 100.0;
  r.avg_amount = cnt > 0 ? r.total_amount / cnt : 0.0;
  r.fraud_rate = cnt > 0 ? (double)fraud / cnt : 0.0;
  // calculateVelocityScore (WindowProcessor.java:327-351); amount thresholds on exact cents
  double score = 0.0;
  if (cnt > 20) score += 0.4;
  else if (cnt > 10) score += 0.2;
  else if (cnt > 5) score += 0.1;
  if (cents > 1000000) score += 0.3;
  else if (cents > 500000) score += 0.2;
  else if (cents > 100000) score += 0.1;
  score += r.fraud_rate * 0.4;
  const double diversity = cnt > 0 ? (double)uniq_m / cnt : 0.0;
  if (diversity < 0.2) score += 0.2;
  r.velocity_score = fmin(1.0, score);
  const unsigned o = atomicAdd(out_count, 1u);
  if (o >= cap) {
    atomicOr(err, 8u);
    return;
  }
  out[o] = r;
}

// MerchantAggregateFunction.getResult (:403-424) from the exact moments: avg, fraud rate, population
// stddev (calculateStandardDeviation :447-457 as the integer-moment formula) and calculateMerchantRiskScore
// (:459-483). Shared by the reduce kernel and the host merge of shard partials (fd_merchant_windows_merge),
// so a merged window is bit-identical to one reduced whole.
__host__ __device__ inline void merchant_window_finalize(fd_merchant_window& r) {
#pragma clang fp contract(off)
  const int cnt = r.count;
  r.unique_payment_methods = __builtin_popcountll(r.pm_mask[0]) + __builtin_popcountll(r.pm_mask[1]) +
                             __builtin_popcountll(r.pm_mask[2]) + __builtin_popcountll(r.pm_mask[3]);
  r.total_amount = (double)r.cents / 100.0;
  r.fraud_amount = (double)r.fraud_cents / 100.0;
  r.avg_amount = cnt > 0 ? r.total_amount / cnt : 0.0;
  r.fraud_rate = cnt > 0 ? (double)r.fraud_count / cnt : 0.0;
  // population stddev, exact moments: (n S2 - S1^2) / n^2 cents^2
  double sd = 0.0;
  if (cnt >= 2) {
    const unsigned __int128 s2 = ((unsigned __int128)r.sq_hi << 64) | (unsigned __int128)r.sq_lo;
    const __int128 num = (__int128)cnt * (__int128)s2 - (__int128)r.cents * (__int128)r.cents;
    const double var = (double)num / ((double)cnt * (double)cnt);
    sd = sqrt(var) / 100.0;
  }
  r.amount_stddev = sd;
  double score = 0.0;
  score += r.fraud_rate * 0.5;
  if (cnt > 1000) score += 0.2;
  else if (cnt > 500) score += 0.1;
  if (r.avg_amount > 0 && sd / r.avg_amount > 2.0) score += 0.2;
  const double diversity = cnt > 0 ? (double)r.unique_users / cnt : 0.0;
  if (diversity < 0.1) score += 0.3;
  r.risk_score = fmin(1.0, score);
}

__global__ void __launch_bounds__(256) win_reduce_merchant_kernel(const WinEvent* __restrict__ log,
                                                                  const unsigned long long* __restrict__ keys,
                                                                  const unsigned* __restrict__ vals, unsigned n,
                                                                  long long base_hour, fd_merchant_window* out,
                                                                  unsigned* out_count, unsigned cap, unsigned* err) {
#pragma clang fp contract(off)
  const unsigned p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const unsigned long long seg = keys[p] >> 31;
  if (p > 0 && (keys[p - 1] >> 31) == seg) return;
  long long cents = 0, fcents = 0, first = 0, last = 0;
  unsigned __int128 s2 = 0;
  int cnt = 0, fraud = 0, high = 0, uniq_u = 0;
  unsigned long long pm[4] = {0, 0, 0, 0};
  unsigned long long prev_u = ~0ull;
  for (unsigned q = p; q < n && (keys[q] >> 31) == seg; ++q) {
    const WinEvent e = log[vals[q]];
    cnt += 1;
    cents += e.cents;
    s2 += (unsigned __int128)((unsigned long long)(e.cents * e.cents));
    if (e.fraud) {
      fraud += 1;
      fcents += e.cents;
    }
    high += e.high;
    const unsigned long long uk = keys[q] & 0x7FFFFFFFull;
    if (uk != prev_u) {
      uniq_u += 1;
      prev_u = uk;
    }
    if (e.pm != 255) pm[e.pm >> 6] |= 1ull << (e.pm & 63);
    if (first == 0 || e.ts < first) first = e.ts;
    if (e.ts > last) last = e.ts;
  }
  const long long hr = (long long)(seg & 0xFFFFull) + base_hour;
  fd_merchant_window r{};
  r.merchant = (int)(seg >> 16);
  r.count = cnt;
  r.window_start = hr * kMerchSize;
  r.window_end = hr * kMerchSize + kMerchSize;
  r.first_ts = first;
  r.last_ts = last;
  r.fraud_count = fraud;
  r.high_risk_count = high;
  r.unique_users = uniq_u;
  r.cents = cents;
  r.fraud_cents = fcents;
  r.sq_lo = (unsigned long long)s2;
  r.sq_hi = (unsigned long long)(s2 >> 64);
  for (int q = 0; q < 4; ++q) r.pm_mask[q] = pm[q];
  merchant_window_finalize(r);
  const unsigned o = atomicAdd(out_count, 1u);
  if (o >= cap) {
    atomicOr(err, 8u);
    return;
  }
  out[o] = r;
}

// keep events a still-open window may contain: ts > W + 1 - size (merchant log: known merchants only)
__global__ void __launch_bounds__(256) win_compact_kernel(const WinEvent* __restrict__ in, int64_t n, long long keep_from,
                                                          int merchants_only, WinEvent* out, unsigned* count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const WinEvent e = in[i];
  if (e.ts < keep_from || (merchants_only && e.merchant < 0)) return;
  out[atomicAdd(count, 1u)] = e;
}

unsigned g256(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

void windows_init(Engine& e, const fd_window_params& p) {
  FD_REQUIRE(p.log_capacity > 0 && p.log_capacity <= (1ll << 28), FD_ERR_INVALID_ARG,
             "log_capacity must be in (0, 2^28]");
  FD_REQUIRE(p.max_out_of_orderness_ms >= 0, FD_ERR_INVALID_ARG, "negative out-of-orderness");
  WindowState& w = e.windows;
  w.cap = p.log_capacity;
  w.ooo = p.max_out_of_orderness_ms;
  for (int b = 0; b < 2; ++b) {
    w.ulog[b].ensure((size_t)w.cap * sizeof(WinEvent));
    w.mlog[b].ensure((size_t)w.cap * sizeof(WinEvent));
  }
  w.ucur = w.mcur = 0;
  w.ucount = w.mcount = 0;
  w.wm = INT64_MIN;
  w.min_seen = INT64_MAX;
  w.max_seen = INT64_MIN;
  w.cand_cap = (kUserSize / kUserSlide) * w.cap;  // each user event is in 5 windows
  w.keys.ensure((size_t)w.cand_cap * 8 * 2);
  w.vals.ensure((size_t)w.cand_cap * 4 * 2);
  w.scalars.ensure(64);
  w.ready = true;
}

namespace {

// scalars: [0] batch max ts (biased u64), [8] batch min ts (biased u64), [16] candidate count,
// [20] error bits, [24] result count
constexpr size_t kScMax = 0, kScMin = 8, kScCnt = 16, kScErr = 20, kScOut = 24;

void windows_check(Engine& e, const char* what) {
  WindowState& w = e.windows;
  unsigned v = 0;
  FD_HIP(hipMemcpyAsync(&v, w.scalars.as<char>() + kScErr, 4, hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  if (v) {
    FD_HIP(hipMemsetAsync(w.scalars.as<char>() + kScErr, 0, 4, e.stream));
    std::string m = std::string(what) + ": ";
    if (v & 1u) m += "card table full; ";
    if (v & 2u) m += "candidate buffer full; ";
    if (v & 4u) m += "firing windows span more than 65535 slides, or merchant index >= 131072; ";
    if (v & 8u) m += "more windows fired than the result capacity; ";
    throw Error(FD_ERR_OOM, m);
  }
}

unsigned read_u32(Engine& e, size_t off) {
  unsigned v = 0;
  FD_HIP(hipMemcpyAsync(&v, e.windows.scalars.as<char>() + off, 4, hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  return v;
}

// sort (keys, vals)[0, n) with rocPRIM (LSD radix over the 64 key bits); returns the sorted arrays
void windows_sort(Engine& e, unsigned n, unsigned long long** k_out, unsigned** v_out) {
  WindowState& w = e.windows;
  unsigned long long* k0 = w.keys.as<unsigned long long>();
  unsigned long long* k1 = k0 + w.cand_cap;
  unsigned* v0 = w.vals.as<unsigned>();
  unsigned* v1 = v0 + w.cand_cap;
  size_t tb = 0;
  FD_HIP(rocprim::radix_sort_pairs(nullptr, tb, k0, k1, v0, v1, (size_t)n, 0, 64, e.stream));
  w.sort_tmp.ensure(std::max<size_t>(tb, 16));
  FD_HIP(rocprim::radix_sort_pairs(w.sort_tmp.ptr, tb, k0, k1, v0, v1, (size_t)n, 0, 64, e.stream));
  *k_out = k1;
  *v_out = v1;
}

}  // namespace

void windows_step(Engine& e, const fd_txn_batch& t, const fd_window_inputs& in, int64_t n, bool flush,
                  fd_user_window* u_out, int64_t u_cap, int64_t* n_user, fd_merchant_window* m_out, int64_t m_cap,
                  int64_t* n_merch) {
  WindowState& w = e.windows;
  CardStore& st = e.state;
  FD_REQUIRE(w.ready, FD_ERR_NOT_LOADED, "windows not initialised (fd_windows_init)");
  FD_REQUIRE(st.ready, FD_ERR_NOT_LOADED, "card state not initialised (fd_state_init)");
  FD_REQUIRE(n >= 0, FD_ERR_INVALID_ARG, "negative batch size");
  FD_REQUIRE(u_cap >= 0 && m_cap >= 0 && u_cap < (1ll << 31) && m_cap < (1ll << 31), FD_ERR_INVALID_ARG,
             "bad result capacity");
  FD_REQUIRE(w.ucount + n <= w.cap && w.mcount + n <= w.cap, FD_ERR_OOM,
             "window event log full: raise fd_window_params.log_capacity");
  *n_user = *n_merch = 0;
  char* sc = w.scalars.as<char>();
  unsigned* d_cnt = reinterpret_cast<unsigned*>(sc + kScCnt);
  unsigned* d_err = reinterpret_cast<unsigned*>(sc + kScErr);
  unsigned* d_out = reinterpret_cast<unsigned*>(sc + kScOut);
  FD_HIP(hipMemsetAsync(sc, 0, 64, e.stream));
  FD_HIP(hipMemsetAsync(sc + kScMin, 0xFF, 8, e.stream));
  if (n > 0) {
    FD_REQUIRE(t.card_key && t.ts_ms && t.amount_cents && t.merchant, FD_ERR_INVALID_ARG,
               "batch needs card_key, ts_ms, amount_cents and merchant");
    WinEvent* ul = w.ulog[w.ucur].as<WinEvent>() + w.ucount;
    WinEvent* ml = w.mlog[w.mcur].as<WinEvent>() + w.mcount;
    hipLaunchKernelGGL(win_append_kernel, dim3(g256(n)), dim3(256), 0, e.stream,
                       st.keys.as<unsigned long long>(), st.view(), (long long)(st.cap - 1), n,
                       reinterpret_cast<const unsigned long long*>(t.card_key),
                       reinterpret_cast<const long long*>(t.ts_ms), reinterpret_cast<const long long*>(t.amount_cents),
                       reinterpret_cast<const int*>(t.merchant), in.payment_method, in.is_fraud, in.fraud_score, ul,
                       ml, reinterpret_cast<unsigned long long*>(sc + kScMax),
                       reinterpret_cast<unsigned long long*>(sc + kScMin), d_err);
    FD_HIP(hipGetLastError());
    w.ucount += n;
    w.mcount += n;
    unsigned long long mm[2] = {0, 0};
    FD_HIP(hipMemcpyAsync(mm, sc + kScMax, 16, hipMemcpyDeviceToHost, e.stream));
    windows_check(e, "window append");
    const long long bmax = (long long)(mm[0] ^ 0x8000000000000000ull);
    const long long bmin = (long long)(mm[1] ^ 0x8000000000000000ull);
    w.max_seen = std::max<int64_t>(w.max_seen, bmax);
    w.min_seen = std::min<int64_t>(w.min_seen, bmin);
  }
  const long long w_prev = w.wm;
  long long w_new = w_prev;
  // BoundedOutOfOrdernessWatermarks; a sharded step also advances on the node-wide max (fd_windows_observe)
  if ((n > 0 || w.observed) && w.max_seen - w.ooo - 1 > w_new) w_new = w.max_seen - w.ooo - 1;
  w.observed = false;
  if (flush && w.max_seen != INT64_MIN && w.max_seen + kMerchSize > w_new) w_new = w.max_seen + kMerchSize;
  if (w_new == w_prev) return;  // no window can fire
  w.wm = w_new;
  // smallest window index that can fire now: its end - 1 > w_prev (first firing: the oldest event's)
  const long long base_min = (w_prev == INT64_MIN) ? floor_div_host(w.min_seen, kUserSlide) - (kUserSize / kUserSlide - 1)
                                                  : floor_div_host(w_prev + 1 - kUserSize, kUserSlide);
  const long long base_hour = (w_prev == INT64_MIN) ? floor_div_host(w.min_seen, kMerchSize)
                                                   : floor_div_host(w_prev + 1 - kMerchSize, kMerchSize);

  for (int which = 0; which < 2; ++which) {
    const bool user = which == 0;
    const int64_t count = user ? w.ucount : w.mcount;
    const WinEvent* log = user ? w.ulog[w.ucur].as<const WinEvent>() : w.mlog[w.mcur].as<const WinEvent>();
    if (count == 0) continue;
    FD_HIP(hipMemsetAsync(d_cnt, 0, 4, e.stream));
    if (user)
      hipLaunchKernelGGL(win_select_user_kernel, dim3(g256(count)), dim3(256), 0, e.stream, log, count, w_prev, w_new,
                         base_min, w.keys.as<unsigned long long>(), w.vals.as<unsigned>(), d_cnt,
                         (unsigned)w.cand_cap, d_err);
    else
      hipLaunchKernelGGL(win_select_merchant_kernel, dim3(g256(count)), dim3(256), 0, e.stream, log, count, w_prev,
                         w_new, base_hour, w.keys.as<unsigned long long>(), w.vals.as<unsigned>(), d_cnt,
                         (unsigned)w.cand_cap, d_err);
    FD_HIP(hipGetLastError());
    windows_check(e, user ? "user window select" : "merchant window select");
    const unsigned nc = read_u32(e, kScCnt);
    if (nc == 0) continue;
    unsigned long long* ks;
    unsigned* vs;
    windows_sort(e, nc, &ks, &vs);
    FD_HIP(hipMemsetAsync(d_out, 0, 4, e.stream));
    const int64_t cap = user ? u_cap : m_cap;
    if (user) {
      w.uout.ensure((size_t)std::max<int64_t>(cap, 1) * sizeof(fd_user_window));
      hipLaunchKernelGGL(win_reduce_user_kernel, dim3(g256(nc)), dim3(256), 0, e.stream, log, ks, vs, nc, base_min,
                         w.uout.as<fd_user_window>(), d_out, (unsigned)cap, d_err);
    } else {
      w.mout.ensure((size_t)std::max<int64_t>(cap, 1) * sizeof(fd_merchant_window));
      hipLaunchKernelGGL(win_reduce_merchant_kernel, dim3(g256(nc)), dim3(256), 0, e.stream, log, ks, vs, nc,
                         base_hour, w.mout.as<fd_merchant_window>(), d_out, (unsigned)cap, d_err);
    }
    FD_HIP(hipGetLastError());
    windows_check(e, user ? "user window reduce" : "merchant window reduce");
    const unsigned no = read_u32(e, kScOut);
    if (user) {
      if (no) FD_REQUIRE(u_out, FD_ERR_INVALID_ARG, "null user_out");
      if (no) FD_HIP(hipMemcpyAsync(u_out, w.uout.ptr, (size_t)no * sizeof(fd_user_window), hipMemcpyDeviceToHost,
                                    e.stream));
      *n_user = no;
    } else {
      if (no) FD_REQUIRE(m_out, FD_ERR_INVALID_ARG, "null merchant_out");
      if (no) FD_HIP(hipMemcpyAsync(m_out, w.mout.ptr, (size_t)no * sizeof(fd_merchant_window),
                                    hipMemcpyDeviceToHost, e.stream));
      *n_merch = no;
    }
  }
  // compaction: drop events no window still open can contain (ts <= w_new + 1 - size)
  for (int which = 0; which < 2; ++which) {
    const bool user = which == 0;
    const long long size = user ? kUserSize : kMerchSize;
    int64_t& count = user ? w.ucount : w.mcount;
    int& cur = user ? w.ucur : w.mcur;
    DeviceBuffer* logs = user ? w.ulog : w.mlog;
    if (count == 0) continue;
    FD_HIP(hipMemsetAsync(d_cnt, 0, 4, e.stream));
    hipLaunchKernelGGL(win_compact_kernel, dim3(g256(count)), dim3(256), 0, e.stream, logs[cur].as<const WinEvent>(),
                       count, w_new + 2 - size, user ? 0 : 1, logs[cur ^ 1].as<WinEvent>(), d_cnt);
    FD_HIP(hipGetLastError());
    count = read_u32(e, kScCnt);
    cur ^= 1;
  }
  FD_HIP(hipStreamSynchronize(e.stream));
}

void windows_observe(Engine& e, int64_t max_event_ts) {
  WindowState& w = e.windows;
  FD_REQUIRE(w.ready, FD_ERR_NOT_LOADED, "windows not initialised (fd_windows_init)");
  w.max_seen = std::max<int64_t>(w.max_seen, max_event_ts);
  w.observed = true;
}

void merchant_windows_merge(const fd_merchant_window* p, int64_t n, fd_merchant_window* out, int64_t* n_out) {
  FD_REQUIRE(n >= 0 && (n == 0 || (p && out)) && n_out, FD_ERR_INVALID_ARG, "bad arguments");
  std::vector<int64_t> idx((size_t)n);
  std::iota(idx.begin(), idx.end(), (int64_t)0);
  std::stable_sort(idx.begin(), idx.end(), [p](int64_t a, int64_t b) {
    return p[a].window_start != p[b].window_start ? p[a].window_start < p[b].window_start
                                                  : p[a].merchant < p[b].merchant;
  });
  int64_t m = 0;
  for (int64_t k : idx) {
    const fd_merchant_window& b = p[k];
    if (m > 0 && out[m - 1].window_start == b.window_start && out[m - 1].merchant == b.merchant) {
      fd_merchant_window& a = out[m - 1];
      a.count += b.count;
      a.fraud_count += b.fraud_count;
      a.high_risk_count += b.high_risk_count;
      a.unique_users += b.unique_users;  // a card (user) lives on one shard: the sets are disjoint
      a.cents += b.cents;
      a.fraud_cents += b.fraud_cents;
      const unsigned __int128 s2 = (((unsigned __int128)a.sq_hi << 64) | a.sq_lo) +
                                   (((unsigned __int128)b.sq_hi << 64) | b.sq_lo);
      a.sq_lo = (uint64_t)s2;
      a.sq_hi = (uint64_t)(s2 >> 64);
      for (int q = 0; q < 4; ++q) a.pm_mask[q] |= b.pm_mask[q];
      if (a.first_ts == 0 || (b.first_ts != 0 && b.first_ts < a.first_ts)) a.first_ts = b.first_ts;  // add() rule
      if (b.last_ts > a.last_ts) a.last_ts = b.last_ts;
    } else {
      out[m++] = b;
    }
  }
  for (int64_t i = 0; i < m; ++i) merchant_window_finalize(out[i]);
  *n_out = m;
}

void windows_release(Engine& e) {
  WindowState& w = e.windows;
  for (auto* b : {&w.ulog[0], &w.ulog[1], &w.mlog[0], &w.mlog[1], &w.keys, &w.vals, &w.sort_tmp, &w.uout, &w.mout,
                  &w.scalars, &w.stage})
    b->release();
  w.ready = false;
}

}  // namespace fd
