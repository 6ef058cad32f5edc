// route.hip — card-hash sharding of the keyed state across GPUs.
//
// The reference partitions per-card work by Kafka key / Flink keyBy(userId)
// (fl/FraudDetectionJob.java keyBy, fl/windows/WindowProcessor.java:45-64) and keeps the per-card
// velocity state in one Redis (fl/services/RedisService.java:178-207). Here every GPU owns the cards
// with shard_of(card_key) == rank and keeps their state resident in its HBM; a micro-batch ingested
// on any GPU is routed to the owners with one RCCL all-to-all of fixed-size transaction records
// (done by the host shim, fdengine/sharding.py), scored there, and the results come back with a
// second all-to-all of result records.
//
// Kernels (all stable: the records for one owner keep the ingest order, so each card sees its
// transactions in (step, ingest rank, ingest index) order — the global arrival order the oracle uses):
//   route_count   : per 256-txn block, per-shard counts (wave ballots)        -> blk[s * nblk + b]
//   route_scan    : one workgroup, exclusive scan of blk in shard-major order -> offsets, counts[s]
//   route_scatter : per txn, pos = offset[s][b] + rank among same-shard txns before it in the block;
//                   writes the 48-B transaction record at pos (seq = ingest index)
//   (owner side: the feature kernels read the received records in place, features.hip TxnSrc)
//   result_pack   : owner side, per scored txn a 24-B result record {fp, conf, seq, decision, risk}
//   result_scatter: ingest side, out[seq] = record (inverse permutation)
#include "fd_internal.h"

namespace fd {
namespace {

static_assert(sizeof(RouteRecord) == FD_ROUTE_RECORD_BYTES, "route record size");
static_assert(sizeof(ResultRecord) == FD_RESULT_RECORD_BYTES, "result record size");

constexpr int kRouteBlock = 256;  // txns per block (4 waves)

__device__ __forceinline__ unsigned long long rmix64(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

// owner GPU of a card: high 32 bits of the mix (the card table's home slot uses the low bits, so the
// owned keys still spread over every slot of the owner's table), multiply-shift range reduction.
__device__ __forceinline__ unsigned shard_of_dev(unsigned long long key, unsigned G) {
  if (key == 0ull) key = 1ull;  // the card table's key normalisation (features.hip find_or_insert)
  return (unsigned)(((rmix64(key) >> 32) * (unsigned long long)G) >> 32);
}

__device__ __forceinline__ unsigned long long lanemask_lt() {
  const unsigned lane = __lane_id();
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// totals (optional, zero on entry): per-shard counts added up across blocks, so the count exchange can start
// before the scan (the sharded step's forward half)
__global__ void __launch_bounds__(kRouteBlock) route_count_kernel(const unsigned long long* __restrict__ key,
                                                                  int64_t n, unsigned G, int nblk,
                                                                  int* __restrict__ blk,
                                                                  unsigned long long* __restrict__ totals) {
  __shared__ int cnt[64];
  const int64_t i = (int64_t)blockIdx.x * kRouteBlock + threadIdx.x;
  if (threadIdx.x < G) cnt[threadIdx.x] = 0;
  __syncthreads();
  const unsigned s = i < n ? shard_of_dev(key[i], G) : 0xffffffffu;
  for (unsigned t = 0; t < G; ++t) {
    const unsigned long long m = __ballot(s == t);
    if (__lane_id() == 0 && m) atomicAdd(&cnt[t], __popcll(m));
  }
  __syncthreads();
  if (threadIdx.x < G) {
    blk[(size_t)threadIdx.x * nblk + blockIdx.x] = cnt[threadIdx.x];
    if (totals && cnt[threadIdx.x]) atomicAdd(&totals[threadIdx.x], (unsigned long long)cnt[threadIdx.x]);
  }
}

// exclusive scan of the shard-major block counts: each of the 1024 threads scans a contiguous segment
__global__ void __launch_bounds__(1024) route_scan_kernel(int* __restrict__ blk, int64_t total, unsigned G,
                                                          int nblk, long long* __restrict__ counts, CountPublish pub) {
  __shared__ long long part[1024];
  const int t = threadIdx.x;
  if (pub.cnt) {  // the sharded step's split sizes first (the host is waiting for them), then the scan
    if (t < 2 * pub.G) {
      const int64_t v = (t >= pub.G && pub.gather_rank >= 0) ? pub.cnt[pub.G + (t - pub.G) * pub.G + pub.gather_rank]
                                                             : pub.cnt[t];
      __hip_atomic_store(pub.h + t, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __threadfence_system();
      if (t < pub.G) pub.cnt[t] = 0;
    }
    __syncthreads();
    if (t == 0) __hip_atomic_store(pub.h_seq, pub.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const int64_t seg = (total + 1023) / 1024;
  const int64_t a = t * seg, b = (a + seg < total) ? a + seg : total;
  long long s = 0;
  for (int64_t j = a; j < b; ++j) s += blk[j];
  part[t] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan
    const long long v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  long long run = t ? part[t - 1] : 0;
  for (int64_t j = a; j < b; ++j) {
    const int c = blk[j];
    blk[j] = (int)run;
    run += c;
  }
  __syncthreads();
  if (counts && t < (int)G) {  // per-shard totals = offset of the next shard's first block - this one's
    const long long lo = blk[(size_t)t * nblk];
    const long long hi = (t + 1 < (int)G) ? (long long)blk[(size_t)(t + 1) * nblk] : part[1023];
    counts[t] = hi - lo;
  }
}

__global__ void __launch_bounds__(kRouteBlock) route_scatter_kernel(
    const unsigned long long* __restrict__ key, const long long* __restrict__ ts, const long long* __restrict__ cents,
    const int* __restrict__ merchant, const unsigned long long* __restrict__ dfp, const unsigned char* __restrict__ ipc,
    const unsigned char* __restrict__ hour, const unsigned char* __restrict__ wk,
    const unsigned char* __restrict__ pm, const unsigned char* __restrict__ fraud, int64_t n, unsigned G, int nblk,
    const int* __restrict__ blk, RouteRecord* __restrict__ out) {
  __shared__ int wcnt[kRouteBlock / 64][64];
  const int64_t i = (int64_t)blockIdx.x * kRouteBlock + threadIdx.x;
  const int w = threadIdx.x >> 6;
  const unsigned s = i < n ? shard_of_dev(key[i], G) : 0xffffffffu;
  int rank = 0;
  for (unsigned t = 0; t < G; ++t) {
    const unsigned long long m = __ballot(s == t);
    if (s == t) rank = __popcll(m & lanemask_lt());
    if (__lane_id() == 0) wcnt[w][t] = __popcll(m);
  }
  __syncthreads();
  if (i >= n) return;
  int before = 0;
  for (int v = 0; v < w; ++v) before += wcnt[v][s];
  const int64_t pos = (int64_t)blk[(size_t)s * nblk + blockIdx.x] + before + rank;
  RouteRecord r;
  r.key = key[i];
  r.ts = ts[i];
  r.cents = cents[i];
  r.dfp = dfp[i];
  r.merchant = merchant[i];
  r.seq = (unsigned)i;
  r.ipc = ipc[i];
  r.hour = hour[i];
  r.wk = wk[i];
  r.pm = pm ? pm[i] : (unsigned char)255;
  r.flags = (fraud && fraud[i]) ? 1u : 0u;
  out[pos] = r;
}

// owner side: records (+ their result records) back to columns for the window / sink kernels
__global__ void __launch_bounds__(256) route_unpack_kernel(const RouteRecord* __restrict__ rec,
                                                           const ResultRecord* __restrict__ res, int64_t n,
                                                           unsigned long long* key, long long* ts, long long* cents,
                                                           int* merchant, unsigned long long* dfp, unsigned char* ipc,
                                                           unsigned char* hour, unsigned char* wk, unsigned char* pm,
                                                           unsigned char* fraud, double* score) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const RouteRecord r = rec[i];
  if (key) key[i] = r.key;
  if (ts) ts[i] = r.ts;
  if (cents) cents[i] = r.cents;
  if (merchant) merchant[i] = r.merchant;
  if (dfp) dfp[i] = r.dfp;
  if (ipc) ipc[i] = r.ipc;
  if (hour) hour[i] = r.hour;
  if (wk) wk[i] = r.wk;
  if (pm) pm[i] = r.pm;
  if (fraud) fraud[i] = (unsigned char)(r.flags & 1u);
  if (score) score[i] = res ? res[i].fraud_prob : __builtin_nan("");
}

__global__ void __launch_bounds__(256) result_pack_kernel(const double* __restrict__ fp,
                                                          const double* __restrict__ conf,
                                                          const unsigned char* __restrict__ dec,
                                                          const unsigned char* __restrict__ risk,
                                                          const RouteRecord* __restrict__ rec, int64_t n,
                                                          ResultRecord* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ResultRecord r;
  r.fraud_prob = fp[i];
  r.confidence = conf[i];
  r.seq = rec[i].seq;
  r.decision = dec[i];
  r.risk = risk[i];
  r.pad = 0;
  out[i] = r;
}

__global__ void __launch_bounds__(256) result_scatter_kernel(const ResultRecord* __restrict__ in, int64_t n,
                                                             double* fp, double* conf, unsigned char* dec,
                                                             unsigned char* risk, unsigned* err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ResultRecord r = in[i];
  if ((int64_t)r.seq >= n) {  // a record from another batch: never write out of bounds
    atomicOr(err, 2u);
    return;
  }
  fp[r.seq] = r.fraud_prob;
  if (conf) conf[r.seq] = r.confidence;
  if (dec) dec[r.seq] = r.decision;
  if (risk) risk[r.seq] = r.risk;
}

unsigned grid256(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

unsigned shard_of_host(unsigned long long key, unsigned G) {
  if (key == 0ull) key = 1ull;
  key ^= key >> 33;
  key *= 0xff51afd7ed558ccdULL;
  key ^= key >> 33;
  key *= 0xc4ceb9fe1a85ec53ULL;
  key ^= key >> 33;
  return (unsigned)(((key >> 32) * (unsigned long long)G) >> 32);
}

void launch_route_partition(Engine& e, const fd_txn_batch& t, const fd_window_inputs* extra, int64_t n, int G,
                            void* d_records, int64_t* d_counts, hipStream_t stream, DeviceBuffer* scratch,
                            bool timed) {
  const hipStream_t st = stream ? stream : e.stream;
  DeviceBuffer& blk = scratch ? *scratch : e.route_blk;
  FD_REQUIRE(G >= 1 && G <= FD_MAX_SHARDS, FD_ERR_INVALID_ARG, "n_shards must be in [1, 64]");
  FD_REQUIRE(n >= 0 && n < (1ll << 31), FD_ERR_INVALID_ARG, "batch size out of range");
  FD_REQUIRE(d_counts != nullptr, FD_ERR_INVALID_ARG, "null counts");
  if (n == 0) {
    FD_HIP(hipMemsetAsync(d_counts, 0, (size_t)G * sizeof(int64_t), st));
    return;
  }
  FD_REQUIRE(d_records != nullptr, FD_ERR_INVALID_ARG, "null records");
  FD_REQUIRE(t.card_key && t.ts_ms && t.amount_cents && t.merchant && t.device_fp && t.ip_class && t.hour &&
                 t.weekend,
             FD_ERR_INVALID_ARG, "incomplete transaction batch");
  const int nblk = (int)((n + kRouteBlock - 1) / kRouteBlock);
  blk.ensure((size_t)G * nblk * sizeof(int));
  Engine::Timed* ev = e.timing && timed ? e.next_event_pair(FD_TIMING_ROUTE) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, st));
  const auto* key = reinterpret_cast<const unsigned long long*>(t.card_key);
  hipLaunchKernelGGL(route_count_kernel, dim3(nblk), dim3(kRouteBlock), 0, st, key, n, (unsigned)G, nblk,
                     blk.as<int>(), nullptr);
  FD_HIP(hipGetLastError());
  hipLaunchKernelGGL(route_scan_kernel, dim3(1), dim3(1024), 0, st, blk.as<int>(),
                     (int64_t)G * nblk, (unsigned)G, nblk, reinterpret_cast<long long*>(d_counts), CountPublish{});
  FD_HIP(hipGetLastError());
  hipLaunchKernelGGL(route_scatter_kernel, dim3(nblk), dim3(kRouteBlock), 0, st, key,
                     reinterpret_cast<const long long*>(t.ts_ms), reinterpret_cast<const long long*>(t.amount_cents),
                     reinterpret_cast<const int*>(t.merchant), reinterpret_cast<const unsigned long long*>(t.device_fp),
                     t.ip_class, t.hour, t.weekend, extra ? extra->payment_method : nullptr,
                     extra ? extra->is_fraud : nullptr, n, (unsigned)G, nblk, blk.as<const int>(),
                     static_cast<RouteRecord*>(d_records));
  FD_HIP(hipGetLastError());
  if (ev) FD_HIP(hipEventRecord(ev->b, st));
}

void launch_route_count(const fd_txn_batch& t, int64_t n, int G, int64_t* totals, hipStream_t st,
                        DeviceBuffer& blk) {
  FD_REQUIRE(G >= 1 && G <= FD_MAX_SHARDS, FD_ERR_INVALID_ARG, "n_shards must be in [1, 64]");
  FD_REQUIRE(n >= 0 && n < (1ll << 31), FD_ERR_INVALID_ARG, "batch size out of range");
  if (n == 0) return;  // the totals stay zero
  FD_REQUIRE(t.card_key, FD_ERR_INVALID_ARG, "incomplete transaction batch");
  const int nblk = (int)((n + kRouteBlock - 1) / kRouteBlock);
  blk.ensure((size_t)G * nblk * sizeof(int));
  hipLaunchKernelGGL(route_count_kernel, dim3(nblk), dim3(kRouteBlock), 0, st,
                     reinterpret_cast<const unsigned long long*>(t.card_key), n, (unsigned)G, nblk, blk.as<int>(),
                     reinterpret_cast<unsigned long long*>(totals));
  FD_HIP(hipGetLastError());
}

void launch_route_place(const fd_txn_batch& t, int64_t n, int G, void* d_records, hipStream_t st, DeviceBuffer& blk,
                        const CountPublish* pub) {
  const CountPublish P = pub ? *pub : CountPublish{};
  if (n == 0) {  // nothing to place; the publish alone
    if (pub) {
      hipLaunchKernelGGL(route_scan_kernel, dim3(1), dim3(1024), 0, st, nullptr, (int64_t)0, (unsigned)G, 0, nullptr, P);
      FD_HIP(hipGetLastError());
    }
    return;
  }
  FD_REQUIRE(d_records != nullptr, FD_ERR_INVALID_ARG, "null records");
  FD_REQUIRE(t.card_key && t.ts_ms && t.amount_cents && t.merchant && t.device_fp && t.ip_class && t.hour &&
                 t.weekend,
             FD_ERR_INVALID_ARG, "incomplete transaction batch");
  const int nblk = (int)((n + kRouteBlock - 1) / kRouteBlock);
  FD_REQUIRE(blk.bytes >= (size_t)G * nblk * sizeof(int), FD_ERR_INVALID_ARG, "route_place before route_count");
  hipLaunchKernelGGL(route_scan_kernel, dim3(1), dim3(1024), 0, st, blk.as<int>(), (int64_t)G * nblk, (unsigned)G,
                     nblk, nullptr, P);
  FD_HIP(hipGetLastError());
  hipLaunchKernelGGL(route_scatter_kernel, dim3(nblk), dim3(kRouteBlock), 0, st,
                     reinterpret_cast<const unsigned long long*>(t.card_key),
                     reinterpret_cast<const long long*>(t.ts_ms), reinterpret_cast<const long long*>(t.amount_cents),
                     reinterpret_cast<const int*>(t.merchant), reinterpret_cast<const unsigned long long*>(t.device_fp),
                     t.ip_class, t.hour, t.weekend, nullptr, nullptr, n, (unsigned)G, nblk, blk.as<const int>(),
                     static_cast<RouteRecord*>(d_records));
  FD_HIP(hipGetLastError());
}

void launch_route_unpack(Engine& e, const void* d_records, const void* d_results, int64_t n, const fd_txn_batch& out,
                         uint8_t* pm, uint8_t* fraud, double* score) {
  FD_REQUIRE(n >= 0 && n < (1ll << 31), FD_ERR_INVALID_ARG, "batch size out of range");
  if (n == 0) return;
  FD_REQUIRE(d_records != nullptr, FD_ERR_INVALID_ARG, "null records");
  hipLaunchKernelGGL(route_unpack_kernel, dim3(grid256(n)), dim3(256), 0, e.stream,
                     static_cast<const RouteRecord*>(d_records), static_cast<const ResultRecord*>(d_results), n,
                     reinterpret_cast<unsigned long long*>(const_cast<uint64_t*>(out.card_key)),
                     reinterpret_cast<long long*>(const_cast<int64_t*>(out.ts_ms)),
                     reinterpret_cast<long long*>(const_cast<int64_t*>(out.amount_cents)),
                     const_cast<int32_t*>(out.merchant),
                     reinterpret_cast<unsigned long long*>(const_cast<uint64_t*>(out.device_fp)),
                     const_cast<uint8_t*>(out.ip_class), const_cast<uint8_t*>(out.hour),
                     const_cast<uint8_t*>(out.weekend), pm, fraud, score);
  FD_HIP(hipGetLastError());
}

void launch_result_pack(Engine& e, const double* fp, const double* conf, const uint8_t* dec, const uint8_t* risk,
                        const RouteRecord* records, int64_t n, void* d_results) {
  if (n == 0) return;
  FD_REQUIRE(d_results != nullptr, FD_ERR_INVALID_ARG, "null result records");
  hipLaunchKernelGGL(result_pack_kernel, dim3(grid256(n)), dim3(256), 0, e.stream, fp, conf, dec, risk, records, n,
                     static_cast<ResultRecord*>(d_results));
  FD_HIP(hipGetLastError());
}

void launch_result_scatter(Engine& e, const void* d_results, int64_t n, double* fp, double* conf, uint8_t* dec,
                           uint8_t* risk) {
  FD_REQUIRE(n >= 0 && n < (1ll << 31), FD_ERR_INVALID_ARG, "batch size out of range");
  if (n == 0) return;
  FD_REQUIRE(d_results && fp, FD_ERR_INVALID_ARG, "null result records / output");
  if (!e.route_err_live) {
    e.route_err.ensure(16);
    FD_HIP(hipMemsetAsync(e.route_err.ptr, 0, 16, e.stream));
    e.route_err_live = true;
  }
  hipLaunchKernelGGL(result_scatter_kernel, dim3(grid256(n)), dim3(256), 0, e.stream,
                     static_cast<const ResultRecord*>(d_results), n, fp, conf, dec, risk, e.route_err.as<unsigned>());
  FD_HIP(hipGetLastError());
}

// Synchronises; raises if a result record carried a seq outside its batch (records from another batch).
void route_check(Engine& e) {
  if (!e.route_err_live) return;
  unsigned v = 0;
  FD_HIP(hipMemcpyAsync(&v, e.route_err.ptr, 4, hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  if (v) {
    FD_HIP(hipMemsetAsync(e.route_err.ptr, 0, 4, e.stream));
    throw Error(FD_ERR_INVALID_ARG, "result record with seq outside its micro-batch (mismatched all-to-all)");
  }
}

}  // namespace fd
