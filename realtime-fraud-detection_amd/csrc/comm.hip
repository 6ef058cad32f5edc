// Card-hash sharding over RCCL, driven by the engine itself (fd_comm_* / fd_sharded_step, engine.hip).
//
// The reference partitions per-card work by key across Kafka partitions and Flink's keyBy(userId)
// (fl/FraudDetectionJob.java, WindowProcessor.java:44,63). Here each GPU owns the cards of its hash range and a
// micro-batch's transactions travel to their owners as 48-B records and come back as 24-B results, point to point
// over xGMI: grouped ncclSend / ncclRecv with per-peer counts (uneven all-to-all), on the engine's own streams, so a
// step is one C-ABI call and no Python collective sits between the kernels.
//
// RCCL is the one the host process already loaded (torch's librccl.so, passed by path): dlopen on the same file
// returns that instance, so the process keeps one RCCL and one HIP runtime. Two communicators per engine: `fwd`
// (count and record exchanges, on the engine's forward stream) and `back` (results, on the engine stream); each
// carries its operations in the same order on every rank.
#include <dlfcn.h>

#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>

#include "fd_internal.h"

namespace fd {

struct RcclApi {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

namespace {
std::mutex g_rccl_mu;
RcclApi g_rccl;
std::string g_rccl_path;

template <class F>
void sym(void* h, const char* name, F& out) {
  out = reinterpret_cast<F>(dlsym(h, name));
  FD_REQUIRE(out != nullptr, FD_ERR_UNSUPPORTED, std::string("RCCL symbol missing: ") + name);
}

const RcclApi& rccl(const char* path) {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (g_rccl.send) {
    FD_REQUIRE(!path || !*path || g_rccl_path == path, FD_ERR_INVALID_ARG,
               "RCCL already loaded from " + g_rccl_path + " (one RCCL per process)");
    return g_rccl;
  }
  FD_REQUIRE(path && *path, FD_ERR_INVALID_ARG, "RCCL library path required");
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  FD_REQUIRE(h != nullptr, FD_ERR_UNSUPPORTED, std::string("dlopen RCCL failed: ") + dlerror());
  RcclApi a;
  sym(h, "ncclGetUniqueId", a.get_unique_id);
  sym(h, "ncclCommInitRank", a.comm_init_rank);
  sym(h, "ncclCommDestroy", a.comm_destroy);
  sym(h, "ncclGroupStart", a.group_start);
  sym(h, "ncclGroupEnd", a.group_end);
  sym(h, "ncclSend", a.send);
  sym(h, "ncclRecv", a.recv);
  sym(h, "ncclGetErrorString", a.error_string);
  g_rccl = a;
  g_rccl_path = path;
  return g_rccl;
}

void check(const RcclApi& R, ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw Error(FD_ERR_HIP, std::string(what) + ": " + R.error_string(r));
}
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
  c.fwd = f;
  c.back = k;
  c.rank = rank;
  c.world = world;
  if (!c.x_fwd) FD_HIP(hipStreamCreateWithFlags(&c.x_fwd, hipStreamNonBlocking));
  for (int s = 0; s < 2; ++s) {
    if (!c.h_cnt[s]) FD_HIP(hipHostMalloc(reinterpret_cast<void**>(&c.h_cnt[s]), 2 * FD_MAX_SHARDS * sizeof(int64_t)));
    if (!c.cnt_ev[s]) FD_HIP(hipEventCreateWithFlags(&c.cnt_ev[s], hipEventDisableTiming));  // the host reads
    if (!c.in_ev[s]) FD_HIP(hipEventCreateWithFlags(&c.in_ev[s], hipEventDisableTiming | hipEventDisableSystemFence));
    if (!c.inbox_ev[s])
      FD_HIP(hipEventCreateWithFlags(&c.inbox_ev[s], hipEventDisableTiming | hipEventDisableSystemFence));
    c.inbox_live[s] = false;
  }
  c.pending = false;
  c.next_slot = 0;
  c.ready = true;
}

void comm_destroy(Engine& e) {
  ShardComm& c = e.comm;
  if (c.x_fwd) (void)hipStreamSynchronize(c.x_fwd);
  (void)hipStreamSynchronize(e.stream);
  if (c.ready) {
    const RcclApi& R = rccl(nullptr);
    if (c.fwd) (void)R.comm_destroy(static_cast<ncclComm_t>(c.fwd));
    if (c.back) (void)R.comm_destroy(static_cast<ncclComm_t>(c.back));
  }
  c.fwd = c.back = nullptr;
  for (int s = 0; s < 2; ++s) {
    for (auto* b : {&c.rec[s], &c.cnt[s], &c.inbox[s], &c.res[s]}) b->release();
    if (c.h_cnt[s]) (void)hipHostFree(c.h_cnt[s]);
    if (c.cnt_ev[s]) (void)hipEventDestroy(c.cnt_ev[s]);
    if (c.in_ev[s]) (void)hipEventDestroy(c.in_ev[s]);
    if (c.inbox_ev[s]) (void)hipEventDestroy(c.inbox_ev[s]);
    c.h_cnt[s] = nullptr;
    c.cnt_ev[s] = c.in_ev[s] = c.inbox_ev[s] = nullptr;
  }
  c.back_buf.release();
  if (c.x_fwd) (void)hipStreamDestroy(c.x_fwd);
  c.x_fwd = nullptr;
  c.ready = false;
  c.pending = false;
}

// partition `t` by owner on the forward stream, exchange the per-owner counts (send[p] to peer p, recv[p] from
// it: one int64 each way per peer), both count vectors to pinned host memory behind cnt_ev[s]
void comm_launch_counts(Engine& e, const fd_txn_batch& t, int64_t n, hipEvent_t ready, int s) {
  ShardComm& c = e.comm;
  const RcclApi& R = rccl(nullptr);
  const int G = c.world;
  if (ready) FD_HIP(hipStreamWaitEvent(c.x_fwd, ready, 0));
  c.rec[s].ensure((size_t)std::max<int64_t>(n, 1) * sizeof(RouteRecord));
  c.cnt[s].ensure(2 * (size_t)G * sizeof(int64_t));
  int64_t* cnt = c.cnt[s].as<int64_t>();
  launch_route_partition(e, t, nullptr, n, G, c.rec[s].ptr, cnt, c.x_fwd, &e.route_blk_stream);
  const ncclComm_t f = static_cast<ncclComm_t>(c.fwd);
  check(R, R.group_start(), "ncclGroupStart");
  for (int p = 0; p < G; ++p) {
    check(R, R.send(cnt + p, 1, ncclInt64, p, f, c.x_fwd), "ncclSend (counts)");
    check(R, R.recv(cnt + G + p, 1, ncclInt64, p, f, c.x_fwd), "ncclRecv (counts)");
  }
  check(R, R.group_end(), "ncclGroupEnd (counts)");
  FD_HIP(hipMemcpyAsync(c.h_cnt[s], cnt, 2 * (size_t)G * sizeof(int64_t), hipMemcpyDeviceToHost, c.x_fwd));
  FD_HIP(hipEventRecord(c.cnt_ev[s], c.x_fwd));
}

// uneven all-to-all of `elem`-byte items: send[p] items (consecutive in sendbuf, peers in rank order) to peer p,
// recv[p] items from peer p into recvbuf (peers in rank order) — the concatenation order the unsharded order needs
void comm_exchange(Engine& e, bool back, hipStream_t st, const void* sendbuf, const int64_t* send, void* recvbuf,
                   const int64_t* recv, size_t elem) {
  ShardComm& c = e.comm;
  const RcclApi& R = rccl(nullptr);
  const ncclComm_t k = static_cast<ncclComm_t>(back ? c.back : c.fwd);
  const char* sb = static_cast<const char*>(sendbuf);
  char* rb = static_cast<char*>(recvbuf);
  size_t os = 0, orr = 0;
  check(R, R.group_start(), "ncclGroupStart");
  for (int p = 0; p < c.world; ++p) {
    if (send[p] > 0) check(R, R.send(sb + os * elem, (size_t)send[p] * elem, ncclUint8, p, k, st), "ncclSend");
    if (recv[p] > 0) check(R, R.recv(rb + orr * elem, (size_t)recv[p] * elem, ncclUint8, p, k, st), "ncclRecv");
    os += (size_t)send[p];
    orr += (size_t)recv[p];
  }
  check(R, R.group_end(), "ncclGroupEnd");
}

}  // namespace fd
