// sink.hip — RedisTransactionSink's bucket aggregates on the device.
//
// Reference (fl/ = services/flink-jobs/src/main/java/com/frauddetection/):
//   updateAggregations          fl/sinks/RedisTransactionSink.java:140-160  hour = ts / 3 600 000, day = ts / 86 400 000
//   updateHourlyAggregations    :165-194  hourly:{hour}  count, amount, fraud, high-risk (fraudScore > 0.7), rate, avg
//   updateDailyAggregations     :199-222  daily:{day}    count, amount, fraud, rate, avg
//   updateMerchantAggregations  :227-262  merchant:{id}:{hour}  count, amount, fraud, distinct users, rate, avg
//   storage                     fl/services/RedisService.java:246-276 (JSON under "agg:" keys, TTL 1800 s)
// Declared semantics: the aggregates of a key after a micro-batch are the reference's after
// the same transactions (counts exact; amounts exact integer cents, reported as cents / 100 — the reference's
// sequential double sum differs by rounding only); the reference's 30-minute TTL is processing (wall-clock)
// time, so retention here is explicit by event-time bucket (fd_sink_evict_before).
//
// HBM state: one open-addressed table of 48-B aggregate entries keyed by kind | bucket | merchant, and a set of
// (merchant, hour, card) 16-B entries for the exact distinct-user counts. Per micro-batch one thread per
// transaction: three find-or-insert + atomic adds, one set insert (a newly inserted member adds one user).
// Integer atomics make the result independent of the order the batch's transactions are applied in.
#include "fd_internal.h"

namespace fd {
namespace {

struct __attribute__((aligned(16))) AggEntry {  // 48 B
  unsigned long long key;  // 0 = empty
  unsigned long long count;
  long long cents;
  unsigned long long fraud;
  unsigned long long high_risk;
  unsigned long long unique_users;
};
static_assert(sizeof(AggEntry) == 48, "AggEntry must be 48 B");

struct __attribute__((aligned(16))) UserEntry {  // 16 B
  unsigned long long tag;  // fmix64 of (merchant, hour, card); 0 = empty
  long long hour;
};

constexpr long long kHourMs = 3600000ll, kDayMs = 86400000ll;

__device__ __forceinline__ unsigned long long smix(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

// kind (2 bits) | merchant + 1 (30 bits) | bucket (32 bits); never 0
__device__ __host__ __forceinline__ unsigned long long agg_key(int kind, long long merchant, long long bucket) {
  return ((unsigned long long)kind << 62) | ((unsigned long long)(merchant + 1) & 0x3FFFFFFFull) << 32 |
         ((unsigned long long)bucket & 0xFFFFFFFFull);
}

__device__ long long agg_slot(AggEntry* T, unsigned long long mask, unsigned long long key, bool insert) {
  unsigned long long h = smix(key) & mask;
  for (unsigned long long p = 0; p <= mask; ++p) {
    const unsigned long long k = __hip_atomic_load(&T[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == key) return (long long)h;
    if (k == 0ull) {
      if (!insert) return -1;
      const unsigned long long old = atomicCAS(&T[h].key, 0ull, key);
      if (old == 0ull || old == key) return (long long)h;
    }
    h = (h + 1) & mask;
  }
  return -2;  // full
}

// true when (tag) was newly inserted
__device__ int user_insert(UserEntry* U, unsigned long long mask, unsigned long long tag, long long hour) {
  unsigned long long h = smix(tag ^ 0x5851F42D4C957F2Dull) & mask;
  for (unsigned long long p = 0; p <= mask; ++p) {
    const unsigned long long k = __hip_atomic_load(&U[h].tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == tag) return 0;
    if (k == 0ull) {
      const unsigned long long old = atomicCAS(&U[h].tag, 0ull, tag);
      if (old == 0ull) {
        U[h].hour = hour;
        return 1;
      }
      if (old == tag) return 0;
    }
    h = (h + 1) & mask;
  }
  return -1;  // full
}

__device__ __forceinline__ long long java_div(long long a, long long b) { return a / b; }  // truncation (Java)

__global__ void __launch_bounds__(256) sink_update_kernel(AggEntry* T, unsigned long long tmask, UserEntry* U,
                                                          unsigned long long umask, int64_t n,
                                                          const unsigned long long* __restrict__ key,
                                                          const long long* __restrict__ ts,
                                                          const long long* __restrict__ cents,
                                                          const int* __restrict__ merchant,
                                                          const unsigned char* __restrict__ is_fraud,
                                                          const double* __restrict__ fscore, unsigned* err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long t = ts[i];
  const long long hour = java_div(t, kHourMs), day = java_div(t, kDayMs);
  const long long c = cents[i];
  const unsigned long long fr = (is_fraud && is_fraud[i]) ? 1ull : 0ull;
  const double fs = fscore ? fscore[i] : __builtin_nan("");
  const unsigned long long hr = (!isnan(fs) && fs > 0.7) ? 1ull : 0ull;
  const int m = merchant[i];
  for (int kind = 1; kind <= 3; ++kind) {
    if (kind == 3 && m < 0) break;  // merchantId == null: no merchant aggregation (:229)
    const unsigned long long k = agg_key(kind, kind == 3 ? m : -1, kind == 2 ? day : hour);
    const long long s = agg_slot(T, tmask, k, true);
    if (s < 0) {
      atomicOr(err, 1u);
      return;
    }
    AggEntry& e = T[s];
    atomicAdd(&e.count, 1ull);
    atomicAdd(reinterpret_cast<unsigned long long*>(&e.cents), (unsigned long long)c);
    if (fr) atomicAdd(&e.fraud, 1ull);
    if (kind == 1 && hr) atomicAdd(&e.high_risk, 1ull);  // only the hourly summary tracks it (:180-183)
    if (kind == 3) {
      unsigned long long kk = key[i];
      if (kk == 0ull) kk = 1ull;  // the card table's key normalisation
      const unsigned long long tag = smix(smix(kk) ^ ((unsigned long long)(m + 1) << 32 | (unsigned long long)hour)) | 1ull;
      const int r = user_insert(U, umask, tag, hour);
      if (r < 0) {
        atomicOr(err, 2u);
        return;
      }
      if (r) atomicAdd(&e.unique_users, 1ull);
    }
  }
}

__global__ void __launch_bounds__(256) sink_query_kernel(const AggEntry* T, unsigned long long tmask, int64_t n,
                                                         const unsigned long long* __restrict__ keys,
                                                         fd_aggregate* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long s = agg_slot(const_cast<AggEntry*>(T), tmask, keys[i], false);
  fd_aggregate a{};
  if (s >= 0) {
    const AggEntry e = T[s];
    a.found = 1;
    a.total_count = (int64_t)e.count;
    a.fraud_count = (int64_t)e.fraud;
    a.high_risk_count = (int64_t)e.high_risk;
    a.unique_user_count = (int64_t)e.unique_users;
    a.total_amount = (double)e.cents / 100.0;
    a.fraud_rate = (double)e.fraud / (double)e.count;        // (double) fraudCount / totalCount
    a.avg_amount = a.total_amount / (double)e.count;         // totalAmount / totalCount
  }
  out[i] = a;
}

// retention: re-insert the entries whose bucket is still kept into a fresh table
__global__ void __launch_bounds__(256) sink_rehash_kernel(const AggEntry* __restrict__ src, unsigned long long cap,
                                                          AggEntry* dst, unsigned long long dmask, long long keep_hour,
                                                          unsigned long long* kept, unsigned* err) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)cap) return;
  const AggEntry e = src[i];
  if (e.key == 0ull) return;
  const int kind = (int)(e.key >> 62);
  const long long bucket = (long long)(int)(unsigned)(e.key & 0xFFFFFFFFull);
  const long long hour = kind == 2 ? bucket * 24 + 23 : bucket;  // a day is kept while any of its hours is
  if (hour < keep_hour) return;
  const long long s = agg_slot(dst, dmask, e.key, true);
  if (s < 0) {
    atomicOr(err, 1u);
    return;
  }
  dst[s] = e;
  atomicAdd(kept, 1ull);
}

__global__ void __launch_bounds__(256) sink_user_rehash_kernel(const UserEntry* __restrict__ src,
                                                               unsigned long long cap, UserEntry* dst,
                                                               unsigned long long dmask, long long keep_hour,
                                                               unsigned long long* kept, unsigned* err) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)cap) return;
  const UserEntry e = src[i];
  if (e.tag == 0ull || e.hour < keep_hour) return;
  if (user_insert(dst, dmask, e.tag, e.hour) < 0) atomicOr(err, 2u);
  else atomicAdd(kept, 1ull);
}

unsigned blocks_of(long long n) { return (unsigned)((n + 255) / 256); }

unsigned long long pow2_at_least(long long n) {
  unsigned long long c = 16;
  while ((long long)c < n) c <<= 1;
  return c;
}

void sink_check(Engine& e) {
  SinkState& k = e.sink;
  unsigned v = 0;
  FD_HIP(hipMemcpyAsync(&v, k.err.ptr, 4, hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  if (v) {
    FD_HIP(hipMemsetAsync(k.err.ptr, 0, 4, e.stream));
    throw Error(FD_ERR_OOM, (v & 1u) ? "aggregate table full: raise fd_sink_params.capacity (or evict)"
                                     : "distinct-user set full: raise fd_sink_params.user_capacity (or evict)");
  }
}

}  // namespace

void sink_init(Engine& e, const fd_sink_params& p) {
  FD_REQUIRE(p.capacity > 0 && p.capacity <= (1ll << 32), FD_ERR_INVALID_ARG, "capacity must be in [1, 2^32]");
  FD_REQUIRE(p.user_capacity > 0 && p.user_capacity <= (1ll << 34), FD_ERR_INVALID_ARG,
             "user_capacity must be in [1, 2^34]");
  SinkState& k = e.sink;
  k.cap = pow2_at_least(p.capacity);
  k.ucap = pow2_at_least(p.user_capacity);
  k.table.ensure(k.cap * sizeof(AggEntry));
  k.users.ensure(k.ucap * sizeof(UserEntry));
  k.err.ensure(16);
  FD_HIP(hipMemsetAsync(k.table.ptr, 0, k.cap * sizeof(AggEntry), e.stream));
  FD_HIP(hipMemsetAsync(k.users.ptr, 0, k.ucap * sizeof(UserEntry), e.stream));
  FD_HIP(hipMemsetAsync(k.err.ptr, 0, 16, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  k.ready = true;
}

void sink_update(Engine& e, const fd_txn_batch& t, const fd_window_inputs& in, int64_t n) {
  SinkState& k = e.sink;
  FD_REQUIRE(k.ready, FD_ERR_NOT_LOADED, "sink not initialised (fd_sink_init)");
  FD_REQUIRE(n >= 0 && n < (1ll << 31), FD_ERR_INVALID_ARG, "batch size out of range");
  if (n == 0) return;
  FD_REQUIRE(t.card_key && t.ts_ms && t.amount_cents && t.merchant, FD_ERR_INVALID_ARG,
             "batch needs card_key, ts_ms, amount_cents and merchant");
  hipLaunchKernelGGL(sink_update_kernel, dim3(blocks_of(n)), dim3(256), 0, e.stream, k.table.as<AggEntry>(),
                     (unsigned long long)(k.cap - 1), k.users.as<UserEntry>(), (unsigned long long)(k.ucap - 1), n,
                     reinterpret_cast<const unsigned long long*>(t.card_key), reinterpret_cast<const long long*>(t.ts_ms),
                     reinterpret_cast<const long long*>(t.amount_cents), reinterpret_cast<const int*>(t.merchant),
                     in.is_fraud, in.fraud_score, k.err.as<unsigned>());
  FD_HIP(hipGetLastError());
  sink_check(e);
}

void sink_query(Engine& e, int kind, const int64_t* bucket, const int32_t* merchant, int64_t n, fd_aggregate* out) {
  SinkState& k = e.sink;
  FD_REQUIRE(k.ready, FD_ERR_NOT_LOADED, "sink not initialised (fd_sink_init)");
  FD_REQUIRE(kind >= FD_AGG_HOURLY && kind <= FD_AGG_MERCHANT, FD_ERR_INVALID_ARG, "unknown aggregate kind");
  FD_REQUIRE(n >= 0 && (n == 0 || (bucket && out && (kind != FD_AGG_MERCHANT || merchant))), FD_ERR_INVALID_ARG,
             "bad query arrays");
  if (n == 0) return;
  std::vector<unsigned long long> keys((size_t)n);
  for (int64_t i = 0; i < n; ++i)
    keys[i] = agg_key(kind, kind == FD_AGG_MERCHANT ? merchant[i] : -1, bucket[i]);
  DeviceBuffer dk, dout;
  dk.ensure((size_t)n * 8);
  dout.ensure((size_t)n * sizeof(fd_aggregate));
  FD_HIP(hipMemcpyAsync(dk.ptr, keys.data(), (size_t)n * 8, hipMemcpyHostToDevice, e.stream));
  hipLaunchKernelGGL(sink_query_kernel, dim3(blocks_of(n)), dim3(256), 0, e.stream, k.table.as<const AggEntry>(),
                     (unsigned long long)(k.cap - 1), n, dk.as<const unsigned long long>(), dout.as<fd_aggregate>());
  FD_HIP(hipGetLastError());
  FD_HIP(hipMemcpyAsync(out, dout.ptr, (size_t)n * sizeof(fd_aggregate), hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  dk.release();
  dout.release();
}

void sink_evict_before(Engine& e, int64_t hour, int64_t* kept_entries, int64_t* kept_users) {
  SinkState& k = e.sink;
  FD_REQUIRE(k.ready, FD_ERR_NOT_LOADED, "sink not initialised (fd_sink_init)");
  DeviceBuffer nt, nu, cnt;
  nt.ensure(k.cap * sizeof(AggEntry));
  nu.ensure(k.ucap * sizeof(UserEntry));
  cnt.ensure(16);
  FD_HIP(hipMemsetAsync(nt.ptr, 0, k.cap * sizeof(AggEntry), e.stream));
  FD_HIP(hipMemsetAsync(nu.ptr, 0, k.ucap * sizeof(UserEntry), e.stream));
  FD_HIP(hipMemsetAsync(cnt.ptr, 0, 16, e.stream));
  hipLaunchKernelGGL(sink_rehash_kernel, dim3(blocks_of((long long)k.cap)), dim3(256), 0, e.stream,
                     k.table.as<const AggEntry>(), (unsigned long long)k.cap, nt.as<AggEntry>(),
                     (unsigned long long)(k.cap - 1), (long long)hour, cnt.as<unsigned long long>(), k.err.as<unsigned>());
  FD_HIP(hipGetLastError());
  hipLaunchKernelGGL(sink_user_rehash_kernel, dim3(blocks_of((long long)k.ucap)), dim3(256), 0, e.stream,
                     k.users.as<const UserEntry>(), (unsigned long long)k.ucap, nu.as<UserEntry>(),
                     (unsigned long long)(k.ucap - 1), (long long)hour, cnt.as<unsigned long long>() + 1,
                     k.err.as<unsigned>());
  FD_HIP(hipGetLastError());
  unsigned long long c[2] = {0, 0};
  FD_HIP(hipMemcpyAsync(c, cnt.ptr, 16, hipMemcpyDeviceToHost, e.stream));
  sink_check(e);
  std::swap(k.table.ptr, nt.ptr);
  std::swap(k.users.ptr, nu.ptr);
  nt.release();
  nu.release();
  cnt.release();
  if (kept_entries) *kept_entries = (int64_t)c[0];
  if (kept_users) *kept_users = (int64_t)c[1];
}

void sink_release(Engine& e) {
  SinkState& k = e.sink;
  k.table.release();
  k.users.release();
  k.err.release();
  k.ready = false;
}

}  // namespace fd
