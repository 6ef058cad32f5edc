// Card-hash sharding over RCCL, driven by the engine itself (fd_comm_* / fd_sharded_step, engine.hip).
//
// The reference partitions per-card work by key across Kafka partitions and Flink's keyBy(userId)
// (fl/FraudDetectionJob.java, WindowProcessor.java:44,63). Here each GPU owns the cards of its hash range and a
// micro-batch's transactions travel to their owners as 48-B records and come back as 24-B results, point to point
// over xGMI: grouped ncclSend / ncclRecv with per-peer counts (uneven all-to-all), on the engine's own streams, so a
// step is one C-ABI call and no Python collective sits between the kernels.
//
// RCCL is the one the host process already loaded (torch's librccl.so, passed by path): dlopen on the same file
// returns that instance, so the process keeps one RCCL and one HIP runtime. Any library exporting the same ten
// symbols can stand in (the tests' in-process loopback, tests/native/rccl_loopback.cpp, runs several ranks on one
// GPU); each communicator remembers the library it came from. Two communicators per engine: `fwd` (count and
// record exchanges, on the engine's forward stream) and `back` (results, on the engine stream). The calling
// thread issues all of a step's operations, in the same order on every rank (fd_internal.h, ShardComm).
#include <dlfcn.h>
#include <time.h>

#include <rccl/rccl.h>

#include <cstring>
#include <map>
#include <mutex>
#include <string>

#include "fd_internal.h"

namespace fd {

struct RcclApi {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclCommAbort) comm_abort = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

namespace {
std::mutex g_rccl_mu;
std::map<std::string, RcclApi>* g_rccl = nullptr;  // by library path; entries live for the process

template <class F>
void sym(void* h, const char* name, F& out) {
  out = reinterpret_cast<F>(dlsym(h, name));
  FD_REQUIRE(out != nullptr, FD_ERR_UNSUPPORTED, std::string("RCCL symbol missing: ") + name);
}

const RcclApi& rccl(const char* path) {
  FD_REQUIRE(path && *path, FD_ERR_INVALID_ARG, "RCCL library path required");
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (!g_rccl) g_rccl = new std::map<std::string, RcclApi>();
  auto it = g_rccl->find(path);
  if (it != g_rccl->end()) return it->second;
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  FD_REQUIRE(h != nullptr, FD_ERR_UNSUPPORTED, std::string("dlopen RCCL failed: ") + dlerror());
  RcclApi a;
  sym(h, "ncclGetUniqueId", a.get_unique_id);
  sym(h, "ncclCommInitRank", a.comm_init_rank);
  sym(h, "ncclCommDestroy", a.comm_destroy);
  sym(h, "ncclCommAbort", a.comm_abort);
  sym(h, "ncclGroupStart", a.group_start);
  sym(h, "ncclGroupEnd", a.group_end);
  sym(h, "ncclSend", a.send);
  sym(h, "ncclRecv", a.recv);
  sym(h, "ncclAllGather", a.all_gather);
  sym(h, "ncclGetErrorString", a.error_string);
  return g_rccl->emplace(path, a).first->second;
}

const RcclApi& api(const ShardComm& c) { return *static_cast<const RcclApi*>(c.api); }

void check(const RcclApi& R, ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw Error(FD_ERR_HIP, std::string(what) + ": " + R.error_string(r));
}

constexpr size_t kCntSeqOff = 2 * FD_MAX_SHARDS * sizeof(int64_t);  // the sequence word after the counts
constexpr size_t kCntBytes = kCntSeqOff + 64;
}  // namespace

void comm_unique_id(const char* rccl_path, uint8_t* out) {
  const RcclApi& R = rccl(rccl_path);
  ncclUniqueId id;
  check(R, R.get_unique_id(&id), "ncclGetUniqueId");
  std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
}

void comm_init(Engine& e, const char* rccl_path, int rank, int world, const uint8_t* id_fwd, const uint8_t* id_back) {
  FD_REQUIRE(world >= 1 && world <= FD_MAX_SHARDS && rank >= 0 && rank < world, FD_ERR_INVALID_ARG,
             "bad rank / world");
  FD_REQUIRE(id_fwd && id_back, FD_ERR_INVALID_ARG, "null unique ids");
  const RcclApi& R = rccl(rccl_path);
  ShardComm& c = e.comm;
  FD_REQUIRE(!c.ready, FD_ERR_INVALID_ARG, "communicators already initialised (fd_comm_destroy first)");
  ncclUniqueId a, b;
  std::memcpy(a.internal, id_fwd, NCCL_UNIQUE_ID_BYTES);
  std::memcpy(b.internal, id_back, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t f = nullptr, k = nullptr;
  check(R, R.comm_init_rank(&f, world, a, rank), "ncclCommInitRank (forward)");
  check(R, R.comm_init_rank(&k, world, b, rank), "ncclCommInitRank (back)");
  c.api = &R;
  c.fwd = f;
  c.back = k;
  c.rank = rank;
  c.world = world;
  c.count_gather = c.count_mode == 1 || (c.count_mode < 0 && world >= 4);
  if (!c.x_fwd) c.x_fwd = make_stream(e.stream_prio == 2 ? -1 : e.stream_prio == 3 ? 1 : 0);
  for (int s = 0; s < 2; ++s) {
    if (!c.h_cnt[s]) {
      FD_HIP(hipHostMalloc(reinterpret_cast<void**>(&c.h_cnt[s]), kCntBytes, hipHostMallocMapped | hipHostMallocCoherent));
      std::memset(c.h_cnt[s], 0, kCntBytes);
      c.cnt_seq[s] = 0;
      FD_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&c.d_hcnt[s]), c.h_cnt[s], 0));
    }
    // send [G], then the receive half: [G] (point-to-point counts) or the G x G all-gathered matrix
    const size_t cb = (size_t)(FD_MAX_SHARDS + FD_MAX_SHARDS * FD_MAX_SHARDS) * sizeof(int64_t);
    c.cnt[s].ensure(cb);
    FD_HIP(hipMemset(c.cnt[s].ptr, 0, cb));
  }
  for (int q = 0; q < ShardComm::kInbox; ++q) {
    if (!c.in_ev[q]) FD_HIP(hipEventCreateWithFlags(&c.in_ev[q], hipEventDisableTiming | hipEventDisableSystemFence));
    if (!c.inbox_ev[q])
      FD_HIP(hipEventCreateWithFlags(&c.inbox_ev[q], hipEventDisableTiming | hipEventDisableSystemFence));
    c.inbox_live[q] = false;
  }
  c.inbox_next = 0;
  c.pending = false;
  c.pending_id = 0;
  c.next_slot = 0;  // (the count buffers keep their sequence numbers across communicators)
  FD_HIP(hipGetDevice(&c.device));
  c.ready = true;
}

void comm_abort(Engine& e, const std::string& reason) {
  ShardComm& c = e.comm;
  if (!c.ready || c.aborted) return;
  const RcclApi& R = api(c);
  // RCCL kernels still queued or running on x_fwd / the engine stream wait for peers that will not come: abort
  // exits them, so the streams drain instead of the hang moving into the next sync or the teardown
  if (c.fwd) (void)R.comm_abort(static_cast<ncclComm_t>(c.fwd));
  if (c.back) (void)R.comm_abort(static_cast<ncclComm_t>(c.back));
  c.fwd = c.back = nullptr;
  c.aborted = true;
  c.abort_reason = reason;
  c.pending = false;
}

bool comm_sync_stream(Engine& e, hipStream_t st) {
  if (!st) return true;
  if (!e.comm.aborted) {
    FD_HIP(hipStreamSynchronize(st));
    return true;
  }
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(e.comm.timeout_ms);
  for (;;) {
    const hipError_t q = hipStreamQuery(st);
    if (q != hipErrorNotReady) return true;  // done, or an error the stream already reported
    if (std::chrono::steady_clock::now() >= deadline) return false;
    const timespec ts{0, 200000};
    nanosleep(&ts, nullptr);
  }
}

void comm_destroy(Engine& e) {
  ShardComm& c = e.comm;
  // after an abort the forward and engine streams are waited for at most comm_timeout_ms each; when either never
  // drains, every buffer an operation on them may still touch is leaked (route blocks of the count / place kernels
  // on x_fwd, the back exchange's results on the engine stream) rather than freed under a live operation
  const bool fwd_drained = comm_sync_stream(e, c.x_fwd);
  const bool eng_drained = comm_sync_stream(e, e.stream);
  const bool drained = fwd_drained && eng_drained;
  if (c.ready && !c.aborted) {
    const RcclApi& R = api(c);
    if (c.fwd) (void)R.comm_destroy(static_cast<ncclComm_t>(c.fwd));
    if (c.back) (void)R.comm_destroy(static_cast<ncclComm_t>(c.back));
  }
  c.fwd = c.back = nullptr;
  if (!drained) {
    if (!fwd_drained) c.x_fwd = nullptr;  // a stream still running work is not destroyed either
    for (int s = 0; s < 2; ++s) c.rec[s].ptr = c.cnt[s].ptr = nullptr, c.h_cnt[s] = nullptr;
    for (int q = 0; q < ShardComm::kInbox; ++q) c.inbox[q].ptr = c.res[q].ptr = nullptr;
    c.back_buf.ptr = nullptr;
    c.route_blk.ptr = nullptr;
  }
  for (int s = 0; s < 2; ++s) {
    for (auto* b : {&c.rec[s], &c.cnt[s]}) b->release();
    if (c.h_cnt[s]) (void)hipHostFree(c.h_cnt[s]);
    c.h_cnt[s] = c.d_hcnt[s] = nullptr;
  }
  for (int q = 0; q < ShardComm::kInbox; ++q) {
    c.inbox[q].release();
    c.res[q].release();
    if (c.in_ev[q]) (void)hipEventDestroy(c.in_ev[q]);
    if (c.inbox_ev[q]) (void)hipEventDestroy(c.inbox_ev[q]);
    c.in_ev[q] = c.inbox_ev[q] = nullptr;
    c.inbox_live[q] = false;
  }
  c.back_buf.release();
  c.route_blk.release();
  if (c.x_fwd) (void)hipStreamDestroy(c.x_fwd);
  c.x_fwd = nullptr;
  c.ready = false;
  c.aborted = false;
  c.abort_reason.clear();
  c.pending = false;
  c.api = nullptr;
}

// On the forward stream: the per-owner counts of `t` (send[p] to peer p, recv[p] from it: one int64 each way per
// peer), published to the slot's coherent host buffer by the first thing the places' scan kernel does (one lane per
// count, each store visible system-wide before the barrier, the sequence word last: the host polls it instead of an
// event — a D2H copy + event wait measured ~70 us from the exchange to the host), then the records' places (scan +
// scatter into rec[s]). Three parts, so the count exchange can also ride
// in the records exchange's group (comm_forward_group): the count kernel, the exchange's sends / receives (inside a
// group the caller opened), the publish + places.
namespace {
void counts_pre(Engine& e, const fd_txn_batch& t, int64_t n, hipEvent_t ready, int s) {
  ShardComm& c = e.comm;
  hipStream_t st = c.x_fwd;
  if (ready) FD_HIP(hipStreamWaitEvent(st, ready, 0));
  launch_route_count(t, n, c.world, c.cnt[s].as<int64_t>(), st, c.route_blk);  // send half zero (comm_init)
}

// the point-to-point form (option count_exchange 0): inside the caller's group
void counts_ops(Engine& e, int s) {
  ShardComm& c = e.comm;
  const RcclApi& R = api(c);
  const int G = c.world;
  int64_t* cnt = c.cnt[s].as<int64_t>();
  const ncclComm_t f = static_cast<ncclComm_t>(c.fwd);
  for (int p = 0; p < G; ++p) {
    check(R, R.send(cnt + p, 1, ncclInt64, p, f, c.x_fwd), "ncclSend (counts)");
    check(R, R.recv(cnt + G + p, 1, ncclInt64, p, f, c.x_fwd), "ncclRecv (counts)");
  }
  c.ops.fetch_add(2 * (unsigned long long)G, std::memory_order_relaxed);
}

// the all-gather form (default): every rank's send vector to every rank, one collective outside any group (the same
// place in the call sequence on every rank: after the records group, or alone)
void counts_gather(Engine& e, int s) {
  ShardComm& c = e.comm;
  const RcclApi& R = api(c);
  int64_t* cnt = c.cnt[s].as<int64_t>();
  check(R, R.all_gather(cnt, cnt + c.world, (size_t)c.world, ncclInt64, static_cast<ncclComm_t>(c.fwd), c.x_fwd),
        "ncclAllGather (counts)");
  c.ops.fetch_add(1, std::memory_order_relaxed);
}

void counts_post(Engine& e, const fd_txn_batch& t, int64_t n, int s) {
  ShardComm& c = e.comm;
  hipStream_t st = c.x_fwd;
  const unsigned long long seq = ++c.cnt_seq[s];
  auto* dseq = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(c.d_hcnt[s]) + kCntSeqOff);
  c.rec[s].ensure_headroom((size_t)std::max<int64_t>(n, 1) * sizeof(RouteRecord));
  const CountPublish pub{c.cnt[s].as<int64_t>(), c.world, c.count_gather ? c.rank : -1, c.d_hcnt[s], dseq, seq};
  launch_route_place(t, n, c.world, c.rec[s].ptr, st, c.route_blk, &pub);  // its scan kernel publishes first
}
}  // namespace

void comm_launch_counts(Engine& e, const fd_txn_batch& t, int64_t n, hipEvent_t ready, int s, HostLaps& L) {
  const RcclApi& R = api(e.comm);
  counts_pre(e, t, n, ready, s);
  L(1);
  if (e.comm.count_gather) {
    counts_gather(e, s);
  } else {
    check(R, R.group_start(), "ncclGroupStart");
    counts_ops(e, s);
    check(R, R.group_end(), "ncclGroupEnd (counts)");
  }
  L(2);
  counts_post(e, t, n, s);
  L(3);
}

// the host wait for slot s's counts, checked against the batch size n, into split[s]: a short spin on the slot's
// sequence word (the counts usually landed during the previous step), then a sleeping poll that also asks the
// stream (an error ends the wait; an idle stream with the word still behind means the publish was lost) and gives
// up after the engine's comm_timeout_ms (a peer that never posts its counts: dead rank, different call pattern)
void comm_wait_counts(Engine& e, int s, int64_t n, HostLaps& L) {
  ShardComm& c = e.comm;
  const int G = c.world;
  const auto* hseq = reinterpret_cast<const unsigned long long*>(reinterpret_cast<const char*>(c.h_cnt[s]) + kCntSeqOff);
  const unsigned long long want = c.cnt_seq[s];
  auto arrived = [&] { return __atomic_load_n(hseq, __ATOMIC_ACQUIRE) == want; };
  if (!arrived()) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const auto spin_until = t0 + std::chrono::microseconds(40);
    while (!arrived() && clk::now() < spin_until) __builtin_ia32_pause();
    const auto deadline = t0 + std::chrono::milliseconds(c.timeout_ms);
    long nap_ns = 2000;
    // every failure below aborts the communicators first: the count exchange (and whatever RCCL queued behind it)
    // would otherwise keep waiting on the device for the missing peer, and the next sync or the teardown would hang
    auto fail = [&](const std::string& why) {
      comm_abort(e, why);
      throw Error(FD_ERR_HIP, why);
    };
    while (!arrived()) {
      const hipError_t q = hipStreamQuery(c.x_fwd);
      if (q == hipSuccess) {
        if (!arrived())
          fail("split sizes never arrived (slot " + std::to_string(s) + ", sequence " + std::to_string(want) + ")");
        break;
      }
      if (q != hipErrorNotReady) fail(std::string("count exchange: ") + hipGetErrorString(q));
      if (clk::now() >= deadline)
        fail("count exchange timed out after " + std::to_string(c.timeout_ms) + " ms (slot " + std::to_string(s) +
             ", sequence " + std::to_string(want) + ", rank " + std::to_string(c.rank) + " of " + std::to_string(G) +
             "): a peer did not post its counts; communicators aborted");
      const timespec ts{0, nap_ns};
      nanosleep(&ts, nullptr);
      nap_ns = std::min(nap_ns * 2, 50000L);
    }
  }
  int64_t sent = 0;
  for (int p = 0; p < 2 * G; ++p) {
    const int64_t v = __atomic_load_n(&c.h_cnt[s][p], __ATOMIC_RELAXED);
    FD_REQUIRE(v >= 0, FD_ERR_HIP, "corrupt split sizes");
    c.split[s][p] = v;
    if (p < G) sent += v;
  }
  FD_REQUIRE(sent == n, FD_ERR_HIP, "split sizes do not add up to the batch");
  L(0);
}

void exchange_ops(Engine& e, bool back, hipStream_t st, const void* sendbuf, const int64_t* send, void* recvbuf,
                  const int64_t* recv, size_t elem);

// slot s's records to their owners on the forward stream, into the next inbox of the ring (after the scoring
// that last read it); with `next`, the next batch's count exchange in the same group (one RCCL launch for both:
// per peer pair the records' send / receive precede the counts' on every rank), then its publish + places
void comm_forward_group(Engine& e, int s, const fd_txn_batch* next, int64_t next_n, hipEvent_t next_ready, int ns,
                        HostLaps& L) {
  ShardComm& c = e.comm;
  const RcclApi& R = api(c);
  const int G = c.world;
  const int64_t* send = c.split[s];
  const int64_t* recv = c.split[s] + G;
  int64_t m = 0;
  for (int p = 0; p < G; ++p) m += recv[p];
  if (next) counts_pre(e, *next, next_n, next_ready, ns);
  L(1);
  const int q = c.inbox_next;
  c.inbox_next = (q + 1) % ShardComm::kInbox;
  c.inbox_of[s] = q;
  if (c.inbox_live[q]) FD_HIP(hipStreamWaitEvent(c.x_fwd, c.inbox_ev[q], 0));
  c.inbox[q].ensure_headroom((size_t)std::max<int64_t>(m, 1) * sizeof(RouteRecord));
  c.res[q].ensure_headroom((size_t)std::max<int64_t>(m, 1) * sizeof(ResultRecord));
  check(R, R.group_start(), "ncclGroupStart");
  exchange_ops(e, false, c.x_fwd, c.rec[s].ptr, send, c.inbox[q].ptr, recv, sizeof(RouteRecord));
  if (next && !c.count_gather) counts_ops(e, ns);
  check(R, R.group_end(), "ncclGroupEnd (records + counts)");
  FD_HIP(hipEventRecord(c.in_ev[q], c.x_fwd));
  if (next && c.count_gather) counts_gather(e, ns);
  L(4);
  if (next) counts_post(e, *next, next_n, ns);
  L(3);
}

// uneven all-to-all of `elem`-byte items: send[p] items (consecutive in sendbuf, peers in rank order) to peer p,
// recv[p] items from peer p into recvbuf (peers in rank order) — the concatenation order the unsharded order needs
void exchange_ops(Engine& e, bool back, hipStream_t st, const void* sendbuf, const int64_t* send, void* recvbuf,
                  const int64_t* recv, size_t elem) {
  ShardComm& c = e.comm;
  const RcclApi& R = api(c);
  const ncclComm_t k = static_cast<ncclComm_t>(back ? c.back : c.fwd);
  const char* sb = static_cast<const char*>(sendbuf);
  char* rb = static_cast<char*>(recvbuf);
  size_t os = 0, orr = 0;
  unsigned long long n_ops = 0;
  for (int p = 0; p < c.world; ++p) {
    if (p == c.rank) {  // this rank's own share: a device copy on the same stream, not an RCCL send / receive pair
      // (2 x world -> 2 x (world - 1) operations per exchange). Enqueued inside the caller's group, so it runs
      // before the group's RCCL kernel on `st`: its source and destination are ready then (the scatter / scoring
      // that wrote sendbuf and the inbox wait precede the group on `st`). send[rank] == recv[rank] by construction.
      FD_REQUIRE(send[p] == recv[p], FD_ERR_HIP, "corrupt split sizes (own share)");
      if (send[p] > 0)
        FD_HIP(hipMemcpyAsync(rb + orr * elem, sb + os * elem, (size_t)send[p] * elem, hipMemcpyDeviceToDevice, st));
    } else {
      if (send[p] > 0) check(R, R.send(sb + os * elem, (size_t)send[p] * elem, ncclUint8, p, k, st), "ncclSend");
      if (recv[p] > 0) check(R, R.recv(rb + orr * elem, (size_t)recv[p] * elem, ncclUint8, p, k, st), "ncclRecv");
      n_ops += (send[p] > 0) + (recv[p] > 0);
    }
    os += (size_t)send[p];
    orr += (size_t)recv[p];
  }
  c.ops.fetch_add(n_ops, std::memory_order_relaxed);
}

void comm_exchange(Engine& e, bool back, hipStream_t st, const void* sendbuf, const int64_t* send, void* recvbuf,
                   const int64_t* recv, size_t elem) {
  const RcclApi& R = api(e.comm);
  check(R, R.group_start(), "ncclGroupStart");
  exchange_ops(e, back, st, sendbuf, send, recvbuf, recv, elem);
  check(R, R.group_end(), "ncclGroupEnd");
}

}  // namespace fd
