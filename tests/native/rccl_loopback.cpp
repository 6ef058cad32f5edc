// TEST INFRASTRUCTURE ONLY — never loaded by the product path.
//
// An in-process loopback of the ten RCCL entry points the engine's sharded step uses (csrc/comm.hip dlopens its
// RCCL by path and calls only these): ncclGetUniqueId, ncclCommInitRank, ncclCommDestroy, ncclCommAbort,
// ncclGroupStart, ncclGroupEnd, ncclSend, ncclRecv, ncclAllGather, ncclGetErrorString. An all-gather is its
// point-to-point form here (a send of the rank's buffer to every rank and a receive from every rank into its place,
// posted as one group). It lets one process run several ranks — one engine and one
// host thread per rank, all on the test box's one GPU — through the very fd_sharded_step the driver runs across
// GPUs, so the N >= 2 step is executed and checked against the oracle without a multi-GPU node
// (tests/test_gpu_sharding_loopback.py). RCCL itself refuses two ranks on one device.
//
// Semantics (NCCL point-to-point): a send from rank a to rank b pairs with a recv on rank b from rank a, in the order
// each side issued them on that communicator; counts x type sizes must agree; ops inside ncclGroupStart/End are
// posted together. Here each op records an event on its stream when posted (send: the data is ready; recv: the
// buffer is free); a matched pair becomes one device-to-device copy on a private copy stream behind both events,
// and each side's stream waits for that copy before anything queued after the op. ncclGroupEnd blocks the calling
// host thread until every op of the group is matched (the peers are other threads), so every stream wait is on an
// event recorded earlier: nothing here can deadlock a hardware queue. A group left unmatched for LOOPBACK_TIMEOUT_S
// seconds (default 60) fails with ncclInvalidUsage and a message on stderr — the test fails instead of hanging.
//
// LOOPBACK_STALL=1 (read per group) models RCCL's device-side blocking instead: the group returns ncclSuccess at once
// and each op's stream is parked behind a host function that waits until its communicator is aborted
// (ncclCommAbort) — or LOOPBACK_TIMEOUT_S passes, so nothing can park a stream for good. No op is ever matched: the
// peers are taken to be dead. The engine's own comm_timeout_ms must then notice, abort and report
// (tests/test_gpu_sharding_loopback.py::test_count_timeout_aborts_the_communicators).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

namespace {

struct Done {  // the copy of one matched pair; shared by its two ops
  hipEvent_t ev = nullptr;
  ~Done() {
    if (ev) (void)hipEventDestroy(ev);
  }
};

struct Op {
  bool send = false;
  const void* sbuf = nullptr;
  void* rbuf = nullptr;
  size_t bytes = 0;
  int src = 0, dst = 0;
  hipStream_t stream = nullptr;
  hipEvent_t posted = nullptr;
  bool matched = false;
  std::string err;
  std::shared_ptr<Done> done;
};

struct Group {
  int nranks = 0;
  int refs = 0;
  std::map<std::pair<int, int>, std::deque<Op*>> sends, recvs;  // unmatched, by (src, dst)
};

std::mutex g_mu;
std::condition_variable g_cv;
std::map<unsigned long long, Group>* g_groups = nullptr;
unsigned long long g_next_id = 1;
hipStream_t g_copy = nullptr;

struct Pending {
  bool send;
  const void* sbuf;
  void* rbuf;
  size_t bytes;
  int peer;
  ncclComm_t comm;
  hipStream_t stream;
};
thread_local int t_depth = 0;
thread_local std::vector<Pending> t_ops;

size_t type_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: case ncclFloat8e4m3: case ncclFloat8e5m2: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
  }
}

double timeout_s() {
  const char* v = std::getenv("LOOPBACK_TIMEOUT_S");
  return v && *v ? std::atof(v) : 60.0;
}

}  // namespace

struct ncclComm {
  unsigned long long group = 0;
  int rank = 0, nranks = 0;
  bool aborted = false;  // (under g_mu) ncclCommAbort: parked streams of this communicator go on
};

namespace {

// under g_mu: one matched (send, recv) pair -> one copy on the private stream
void match(Op* s, Op* r) {
  if (!s->send) std::swap(s, r);
  s->matched = r->matched = true;
  if (s->bytes != r->bytes) {
    s->err = r->err = "size mismatch: send " + std::to_string(s->bytes) + " B from rank " + std::to_string(s->src) +
                      ", recv " + std::to_string(r->bytes) + " B on rank " + std::to_string(r->dst);
    return;
  }
  auto d = std::make_shared<Done>();
  hipError_t e = hipSuccess;
  if (!g_copy) e = hipStreamCreateWithFlags(&g_copy, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&d->ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipStreamWaitEvent(g_copy, s->posted, 0);
  if (e == hipSuccess) e = hipStreamWaitEvent(g_copy, r->posted, 0);
  if (e == hipSuccess && s->bytes) e = hipMemcpyAsync(r->rbuf, s->sbuf, s->bytes, hipMemcpyDeviceToDevice, g_copy);
  if (e == hipSuccess) e = hipEventRecord(d->ev, g_copy);
  if (e != hipSuccess) {
    s->err = r->err = std::string("HIP: ") + hipGetErrorString(e);
    return;
  }
  s->done = r->done = d;
}

bool stall_mode() {
  const char* v = std::getenv("LOOPBACK_STALL");
  return v && *v == '1';
}

// the stream side of a stalled op: a host function holding its stream until the communicator is aborted
void stall_fn(void* arg) {
  auto* comm = static_cast<ncclComm*>(arg);
  std::unique_lock<std::mutex> lk(g_mu);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s());
  if (!g_cv.wait_until(lk, deadline, [&] { return comm->aborted; }))
    std::fprintf(stderr, "rccl_loopback: stalled op released by LOOPBACK_TIMEOUT_S, never aborted\n");
}

ncclResult_t flush(std::vector<Pending>& ops) {
  if (stall_mode()) {
    for (const Pending& p : ops)
      if (hipLaunchHostFunc(p.stream, stall_fn, p.comm) != hipSuccess) {
        ops.clear();
        return ncclUnhandledCudaError;
      }
    ops.clear();
    return ncclSuccess;
  }
  std::vector<std::unique_ptr<Op>> mine;
  mine.reserve(ops.size());
  for (const Pending& p : ops) {
    auto o = std::make_unique<Op>();
    o->send = p.send;
    o->sbuf = p.sbuf;
    o->rbuf = p.rbuf;
    o->bytes = p.bytes;
    o->src = p.send ? p.comm->rank : p.peer;
    o->dst = p.send ? p.peer : p.comm->rank;
    o->stream = p.stream;
    if (hipEventCreateWithFlags(&o->posted, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(o->posted, p.stream) != hipSuccess) {
      std::fprintf(stderr, "rccl_loopback: event record failed\n");
      return ncclUnhandledCudaError;
    }
    mine.push_back(std::move(o));
  }
  ncclResult_t rc = ncclSuccess;
  {
    std::unique_lock<std::mutex> lk(g_mu);
    for (size_t i = 0; i < mine.size(); ++i) {
      Op* o = mine[i].get();
      Group& g = (*g_groups)[ops[i].comm->group];
      const auto key = std::make_pair(o->src, o->dst);
      auto& other = o->send ? g.recvs[key] : g.sends[key];
      if (!other.empty()) {
        Op* m = other.front();
        other.pop_front();
        match(o, m);
      } else {
        (o->send ? g.sends[key] : g.recvs[key]).push_back(o);
      }
    }
    g_cv.notify_all();
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s());
    auto all = [&] {
      for (auto& o : mine)
        if (!o->matched) return false;
      return true;
    };
    if (!g_cv.wait_until(lk, deadline, all)) {
      for (size_t i = 0; i < mine.size(); ++i) {  // withdraw the unmatched ops (the peers never came)
        Op* o = mine[i].get();
        if (o->matched) continue;
        Group& g = (*g_groups)[ops[i].comm->group];
        auto& q = (o->send ? g.sends : g.recvs)[std::make_pair(o->src, o->dst)];
        for (auto it = q.begin(); it != q.end(); ++it)
          if (*it == o) {
            q.erase(it);
            break;
          }
        std::fprintf(stderr, "rccl_loopback: %s rank %d -> rank %d (%zu B) unmatched after %.0f s\n",
                     o->send ? "send" : "recv", o->src, o->dst, o->bytes, timeout_s());
      }
      rc = ncclInvalidUsage;
    }
  }
  for (auto& o : mine) {
    if (!o->err.empty()) {
      std::fprintf(stderr, "rccl_loopback: %s\n", o->err.c_str());
      rc = ncclInvalidUsage;
    }
    if (o->done && hipStreamWaitEvent(o->stream, o->done->ev, 0) != hipSuccess) rc = ncclUnhandledCudaError;
    (void)hipEventDestroy(o->posted);
  }
  ops.clear();
  return rc;
}

ncclResult_t post(bool send, const void* sbuf, void* rbuf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm,
                  hipStream_t stream) {
  if (!comm || peer < 0 || peer >= comm->nranks || type_size(t) == 0) return ncclInvalidArgument;
  t_ops.push_back(Pending{send, sbuf, rbuf, count * type_size(t), peer, comm, stream});
  if (t_depth > 0) return ncclSuccess;
  return flush(t_ops);
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  std::memset(id->internal, 0, sizeof(id->internal));
  std::lock_guard<std::mutex> lk(g_mu);
  const unsigned long long v = g_next_id++;
  std::memcpy(id->internal, "LOOPBACK", 8);
  std::memcpy(id->internal + 8, &v, sizeof(v));
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks || std::memcmp(id.internal, "LOOPBACK", 8) != 0)
    return ncclInvalidArgument;
  unsigned long long gid = 0;
  std::memcpy(&gid, id.internal + 8, sizeof(gid));
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_groups) g_groups = new std::map<unsigned long long, Group>();
  Group& g = (*g_groups)[gid];
  if (g.refs == 0) g.nranks = nranks;
  if (g.nranks != nranks) return ncclInvalidUsage;
  ++g.refs;
  *comm = new ncclComm{gid, rank, nranks};
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_groups->find(comm->group);
    if (it != g_groups->end() && --it->second.refs == 0) g_groups->erase(it);
  }
  delete comm;
  return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(g_mu);
  comm->aborted = true;  // the object stays allocated: a parked host function may still read it
  auto it = g_groups->find(comm->group);
  if (it != g_groups->end() && --it->second.refs == 0) g_groups->erase(it);
  g_cv.notify_all();
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
  ++t_depth;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (t_depth <= 0) return ncclInvalidUsage;
  if (--t_depth > 0) return ncclSuccess;
  return flush(t_ops);
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
  return post(true, sendbuff, nullptr, count, datatype, peer, comm, stream);
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
  return post(false, nullptr, recvbuff, count, datatype, peer, comm, stream);
}

ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t datatype,
                           ncclComm_t comm, hipStream_t stream) {
  if (!comm || type_size(datatype) == 0) return ncclInvalidArgument;
  const size_t bytes = sendcount * type_size(datatype);
  ncclGroupStart();
  ncclResult_t rc = ncclSuccess;
  for (int p = 0; p < comm->nranks && rc == ncclSuccess; ++p) {
    rc = post(true, sendbuff, nullptr, sendcount, datatype, p, comm, stream);
    if (rc == ncclSuccess)
      rc = post(false, nullptr, static_cast<char*>(recvbuff) + (size_t)p * bytes, sendcount, datatype, p, comm, stream);
  }
  const ncclResult_t g = ncclGroupEnd();
  return rc != ncclSuccess ? rc : g;
}

const char* ncclGetErrorString(ncclResult_t result) {
  switch (result) {
    case ncclSuccess: return "no error";
    case ncclUnhandledCudaError: return "loopback: HIP call failed";
    case ncclInvalidArgument: return "loopback: invalid argument";
    case ncclInvalidUsage: return "loopback: invalid usage (unmatched or mismatched send/recv; see stderr)";
    default: return "loopback: error";
  }
}

}  // extern "C"
