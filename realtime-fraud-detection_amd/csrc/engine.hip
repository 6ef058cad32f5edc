// engine.hip — C-ABI surface of libfdengine.so (declared in include/fdengine.h).
// Every entry point catches everything: status codes + a thread-local message cross the ABI,
// exceptions never do (mirrors the reference's log-and-raise contract, ml/models/model_manager.py:302-307,
// with the raise done by the Python shim).
#include <chrono>
#include <mutex>
#include <cstring>
#include <string>

#include "blend_row.h"
#include "fd_internal.h"
#include "ingest_parse.h"

namespace fd {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

Engine::Timed* Engine::next_event_pair(int kind) {
  if (timing_every > 1 && kind >= 0 && kind < 16 && (timing_seq[kind]++ % (unsigned)timing_every) != 0)
    return nullptr;  // sampled timing: this launch runs without event records
  if (events_used == events.size()) {
    // timing events only: no system-scope fence at record (a fenced record costs ~4 us of stream time)
    hipEvent_t a, b;
    FD_HIP(hipEventCreateWithFlags(&a, hipEventDisableSystemFence));
    FD_HIP(hipEventCreateWithFlags(&b, hipEventDisableSystemFence));
    events.push_back({a, b, 0});
  }
  Timed* t = &events[events_used++];
  t->kind = kind;
  t->split = false;
  return t;
}

}  // namespace fd

using fd::Engine;

#define FD_API_BEGIN try {
#define FD_API_END                    \
  return FD_OK;                       \
  }                                   \
  catch (const fd::Error& e) {        \
    fd::set_error(e.what());          \
    return e.code;                    \
  }                                   \
  catch (const std::bad_alloc&) {     \
    fd::set_error("out of memory");   \
    return FD_ERR_OOM;                \
  }                                   \
  catch (const std::exception& e) {   \
    fd::set_error(e.what());          \
    return FD_ERR_INVALID_ARG;        \
  }

struct fd_engine {
  Engine e;
  // every entry point on this engine holds it (FD_ENGINE_LOCK): calls from several host threads are serialised
  // per engine (e.g. ModelManager.predict in an executor thread beside a reload on the event loop's thread);
  // recursive so an entry point may call another
  std::recursive_mutex mu;
};

static std::recursive_mutex& lock_of(fd_engine* p) {
  static std::recursive_mutex none;  // null engine: E() reports it
  return p ? p->mu : none;
}
#define FD_ENGINE_LOCK(p) std::lock_guard<std::recursive_mutex> fd_engine_guard_(lock_of(p))

// Engine of an entry point that may queue work on e.stream: the next fd_score_batch_pipelined orders its
// feature stream after e.stream again (pipe_dirty).
static Engine& E(fd_engine* p) {
  FD_REQUIRE(p != nullptr, FD_ERR_INVALID_ARG, "null engine");
  p->e.activate();
  p->e.pipe_dirty = true;
  return p->e;
}

// Engine of an entry point that queues no device work touching engine state (options, timing reads)
static Engine& E_quiet(fd_engine* p) {
  FD_REQUIRE(p != nullptr, FD_ERR_INVALID_ARG, "null engine");
  p->e.activate();
  return p->e;
}

// Events that only order one device's streams: no system-scope release at record (that is an L2 writeback
// per record, several us of stream time between a kernel and its cross-stream dependents)
constexpr unsigned kStreamEventFlags = hipEventDisableTiming | hipEventDisableSystemFence;

static fd::PackedForest& slot_of(Engine& e, int slot) {
  FD_REQUIRE(slot >= 0 && slot < fd::kMaxSlots, FD_ERR_INVALID_ARG, "slot out of range");
  return e.forests[slot];
}

// Score the same feature matrix with every forest model, then blend (all on e.stream). A model in slot
// FD_SLOT_LSTM runs the LSTM head over d_seq (n x T x 16) on the auxiliary stream, forked after
// everything already queued on e.stream (the feature kernel that wrote d_seq) and joined before the blend.
// Returns true when the route result records were written too (the fused ensemble kernel writes them in its
// epilogue); otherwise the caller packs them from the columns.
static bool score_matrix(Engine& e, const fd_blend_params& p, const int32_t* slots, const double* const* ext,
                         const uint8_t* present, const float* dX, int64_t n, int32_t ld, double* dMP,
                         double* dfp, double* dconf, uint8_t* ddec, uint8_t* drisk, const float* d_seq = nullptr,
                         int T = 0, const fd::RouteRecord* records = nullptr, fd::ResultRecord* results = nullptr,
                         int compact = 0, const unsigned long long* d_seq_desc = nullptr) {
  FD_REQUIRE(p.n_models > 0 && p.n_models <= FD_MAX_MODELS, FD_ERR_INVALID_ARG, "n_models out of range");
  FD_REQUIRE(slots != nullptr && (dfp != nullptr || results != nullptr), FD_ERR_INVALID_ARG, "null slots/output");
  if (n == 0) return false;
  // one XGBoost + one IsolationForest, large batch: both forests and the blend in one kernel
  if (fd::launch_ensemble(e, p, slots, present, dX, n, ld, dMP, dfp, dconf, ddec, drisk, records, results, compact))
    return results != nullptr;
  // compact vectors are written only when the fused kernel applies (pipe_step): any other path is a bug
  FD_REQUIRE(!compact, FD_ERR_UNSUPPORTED, "internal: compact vectors without the fused ensemble kernel");
  FD_REQUIRE(dfp != nullptr, FD_ERR_INVALID_ARG, "null output");
  const int M = p.n_models;
  if (!dMP) {
    e.scratch_probs.ensure((size_t)n * M * sizeof(double));
    dMP = e.scratch_probs.as<double>();
  }
  const double* cols[FD_MAX_MODELS] = {};
  // small (latency) batches, small_streams: 0 (default) everything on e.stream — the kernels of a 1 k batch are
  // short and the cross-queue fork / join hops cost more than the overlap gains (config 5: 0.088 vs 0.095 ms);
  // 1 the LSTM and every forest after the first on aux; 2 the LSTM on aux, the other forests on aux2 (forked
  // after everything queued so far, i.e. the feature kernel). Large batches: the LSTM on aux.
  int n_forests = 0;
  for (int m = 0; m < M; ++m) n_forests += (!(present && !present[m]) && slots[m] >= 0 && slots[m] != FD_SLOT_LSTM);
  const bool latency = (n + fd::kTile - 1) / fd::kTile < fd::kSplitTiles;
  const int ss = latency ? e.small_streams : 2;
  const bool small = latency && n_forests > 1;
  bool aux_forked = false;
  auto fork_aux = [&]() {
    if (aux_forked) return;
    if (!e.aux_stream) {
      FD_HIP(hipStreamCreateWithFlags(&e.aux_stream, hipStreamNonBlocking));
      FD_HIP(hipEventCreateWithFlags(&e.fork_ev, kStreamEventFlags));
      FD_HIP(hipEventCreateWithFlags(&e.join_ev, kStreamEventFlags));
    }
    FD_HIP(hipEventRecord(e.fork_ev, e.stream));
    FD_HIP(hipStreamWaitEvent(e.aux_stream, e.fork_ev, 0));
    aux_forked = true;
  };
  // option latency_prebin: when this call runs the pair path below on e.stream (two forests, every other present
  // model the LSTM head), the LSTM launch bins the vectors for the pair's walks in workgroups ahead of its own, and
  // the pair skips its binning launch (fd::PreBin; the bins are for this call only)
  struct PreBinReset {
    Engine& e;
    ~PreBinReset() { e.prebin.want = e.prebin.done = false; }
  } prebin_reset{e};
  e.prebin.want = e.prebin.done = false;
  if (e.latency_prebin && e.latency_fused && small && n_forests == 2 && ss == 0) {
    int fm[2], k = 0;
    bool lstm = false, others = false;
    for (int m = 0; m < M; ++m) {
      if (present && !present[m]) continue;
      if (slots[m] == FD_SLOT_LSTM) lstm = true;
      else if (slots[m] >= 0 && slots[m] < fd::kMaxSlots && k < 2) fm[k++] = m;
      else others = true;
    }
    if (lstm && !others && k == 2) {
      const fd::PackedForest& pa = e.forests[slots[fm[0]]];
      const fd::PackedForest& pb = e.forests[slots[fm[1]]];
      if (pa.loaded && pb.loaded) fd::forest_pair_prebin(e, pa, pb, dX, n, ld);
    }
  }
  for (int m = 0; m < M; ++m) {  // the LSTM first, so it overlaps the forests
    if ((present && !present[m]) || slots[m] != FD_SLOT_LSTM) continue;
    FD_REQUIRE(d_seq != nullptr, FD_ERR_INVALID_ARG,
               "the LSTM head needs card-history sequences (fd_score_batch_device with seq_len > 0)");
    double* col = dMP + (size_t)m * n;
    if (ss == 0) {
      fd::launch_lstm(e, e.stream, d_seq, n, T, col, d_seq_desc);
    } else {
      fork_aux();
      fd::launch_lstm(e, e.aux_stream, d_seq, n, T, col, d_seq_desc);
    }
    cols[m] = col;
  }
  const bool use2 = small && ss == 2, use1 = small && ss == 1;
  if (use2) {
    if (!e.aux2_stream) {
      FD_HIP(hipStreamCreateWithFlags(&e.aux2_stream, hipStreamNonBlocking));
      FD_HIP(hipEventCreateWithFlags(&e.join2_ev, kStreamEventFlags));
      if (!e.fork_ev) FD_HIP(hipEventCreateWithFlags(&e.fork_ev, kStreamEventFlags));
    }
    FD_HIP(hipEventRecord(e.fork_ev, e.stream));
    FD_HIP(hipStreamWaitEvent(e.aux2_stream, e.fork_ev, 0));
  }
  if (use1) fork_aux();
  // two forests, one stream: one binning launch for both (fd::launch_forest_pair); when every other present model
  // is the LSTM head (already queued above), both walks in one launch and both sums + the blend in another
  // (fd::launch_forest_pair_blend: 3 launches instead of 6)
  bool paired = false;
  if (small && n_forests == 2 && (ss == 0 || (e.latency_fused && !use2))) {
    int fm[2], k = 0;
    for (int m = 0; m < M && k < 2; ++m)
      if (!(present && !present[m]) && slots[m] >= 0 && slots[m] != FD_SLOT_LSTM) fm[k++] = m;
    const fd::PackedForest& pa = slot_of(e, slots[fm[0]]);
    const fd::PackedForest& pb = slot_of(e, slots[fm[1]]);
    if (pa.loaded && pb.loaded) {
      double* ca = dMP + (size_t)fm[0] * n;
      double* cb = dMP + (size_t)fm[1] * n;
      bool others_lstm = true;
      for (int m = 0; m < M; ++m)
        if (!(present && !present[m]) && m != fm[0] && m != fm[1] && slots[m] != FD_SLOT_LSTM) others_lstm = false;
      if (others_lstm && e.latency_fused) {
        const double* pc[FD_MAX_MODELS] = {};
        int q = 0, pos_a = -1, pos_b = -1;
        for (int m = 0; m < M; ++m) {
          if (present && !present[m]) continue;
          if (m == fm[0]) pos_a = q;
          if (m == fm[1]) pos_b = q;
          pc[q++] = m == fm[0] ? ca : m == fm[1] ? cb : cols[m];
        }
        // the LSTM head on the side stream (small_streams 1): the blend launch waits for it
        hipEvent_t lstm_done = nullptr;
        if (aux_forked) {
          FD_HIP(hipEventRecord(e.join_ev, e.aux_stream));
          lstm_done = e.join_ev;
        }
        if (fd::launch_forest_pair_blend(e, pa, pb, dX, n, ld, fd::blend_consts(p, present), pc, pos_a, pos_b, dfp,
                                         dconf, ddec, drisk, lstm_done))
          return false;
      }
      if (ss == 0) {  // (with side streams the per-forest launches below)
        paired = fd::launch_forest_pair(e, pa, pb, dX, n, ld, ca, cb);
        if (paired) {
          cols[fm[0]] = ca;
          cols[fm[1]] = cb;
        }
      }
    }
  }
  int forests_seen = 0;
  for (int m = 0; m < M; ++m) {
    if ((present && !present[m]) || slots[m] == FD_SLOT_LSTM) continue;
    if (paired && slots[m] >= 0) continue;
    double* col = dMP + (size_t)m * n;
    if (slots[m] >= 0) {
      const fd::PackedForest& pf = slot_of(e, slots[m]);
      FD_REQUIRE(pf.loaded, FD_ERR_NOT_LOADED, "Model in slot " + std::to_string(slots[m]) + " not loaded");
      const bool side = small && forests_seen++ > 0;
      const hipStream_t st = side && use2 ? e.aux2_stream : side && use1 ? e.aux_stream : nullptr;
      fd::launch_forest(e, pf, dX, n, ld, col, nullptr, nullptr, st);
      cols[m] = col;
    } else {
      FD_REQUIRE(ext && ext[m], FD_ERR_INVALID_ARG, "model without slot needs an external probability column");
      if (ext[m] != col)
        FD_HIP(hipMemcpyAsync(col, ext[m], (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, e.stream));
      cols[m] = col;
    }
  }
  if (aux_forked) {
    FD_HIP(hipEventRecord(e.join_ev, e.aux_stream));
    FD_HIP(hipStreamWaitEvent(e.stream, e.join_ev, 0));
  }
  if (use2) {
    FD_HIP(hipEventRecord(e.join2_ev, e.aux2_stream));
    FD_HIP(hipStreamWaitEvent(e.stream, e.join2_ev, 0));
  }
  fd::launch_blend(e, p, n, cols, present, dfp, dconf, ddec, drisk);
  return false;
}

// engine scratch for the fused path's LSTM input sequences, when a present model is the LSTM head
static float* lstm_seq_buffer(Engine& e, const fd_blend_params& p, const int32_t* slots, const uint8_t* present,
                              int64_t n) {
  bool want = false;
  for (int m = 0; m < p.n_models && m < FD_MAX_MODELS; ++m)
    want = want || (slots && slots[m] == FD_SLOT_LSTM && !(present && !present[m]));
  if (!want) return nullptr;
  FD_REQUIRE(e.state.ready && e.state.S > 0, FD_ERR_INVALID_ARG,
             "the LSTM head needs card history: fd_state_params.seq_len > 0");
  e.seq_buf.ensure((size_t)n * e.state.S * fd::kSeqInput * sizeof(float));
  return e.seq_buf.as<float>();
}

extern "C" {

const char* fd_last_error(void) { return fd::g_last_error.c_str(); }

int fd_abi_version(void) { return FD_ABI_VERSION; }

int fd_device_count(int* out) {
  FD_API_BEGIN
  FD_REQUIRE(out, FD_ERR_INVALID_ARG, "null out");
  int c = 0;
  FD_HIP(hipGetDeviceCount(&c));
  *out = c;
  FD_API_END
}

int fd_engine_create(int device, fd_engine** out) {
  FD_API_BEGIN
  FD_REQUIRE(out, FD_ERR_INVALID_ARG, "null out");
  *out = nullptr;
  int c = 0;
  FD_HIP(hipGetDeviceCount(&c));
  FD_REQUIRE(device >= 0 && device < c, FD_ERR_INVALID_ARG,
             "device " + std::to_string(device) + " not present (" + std::to_string(c) + " visible)");
  auto* p = new fd_engine();
  p->e.device = device;
  try {
    FD_HIP(hipSetDevice(device));
    FD_HIP(hipStreamCreateWithFlags(&p->e.own_stream, hipStreamNonBlocking));
    p->e.stream = p->e.own_stream;
  } catch (...) {
    delete p;
    throw;
  }
  *out = p;
  FD_API_END
}

int fd_engine_destroy(fd_engine* eng) {
  FD_API_BEGIN
  if (!eng) return FD_OK;
  { FD_ENGINE_LOCK(eng); }  // wait for a call in flight on another thread (destroying while in use is the caller's bug)
  Engine& e = E(eng);
  if (e.comm.aborted) {  // an aborted exchange: every stream gets a bounded wait; one that never drains leaks the engine
    bool ok = fd::comm_sync_stream(e, e.comm.x_fwd);
    ok = fd::comm_sync_stream(e, e.stream) && ok;
    for (hipStream_t st : e.pipe_stream) ok = fd::comm_sync_stream(e, st) && ok;
    ok = fd::comm_sync_stream(e, e.pipe_slot_stream) && ok;
    FD_REQUIRE(ok, FD_ERR_HIP, "engine leaked: streams still busy " + std::to_string(e.comm.timeout_ms) +
                                   " ms after the communicators were aborted (" + e.comm.abort_reason + ")");
  }
  (void)hipStreamSynchronize(e.stream);
  for (auto& f : e.forests) {
    for (auto* b : {&f.split.bins, &f.split.nan, &f.split.leaves}) b->release();
    f.blob.release();
    f.leaf_ids.release();
    f.b_blob.release();
    f.b_thr.release();
    f.b_thr_off.release();
  }
  e.stage_in.release();
  e.stage_out0.release();
  e.stage_out1.release();
  e.stage_out2.release();
  e.stage_out3.release();
  e.scratch_probs.release();
  e.stage_ext.release();
  e.feat_vec.release();
  e.feat_in.release();
  fd::windows_release(e);
  fd::sink_release(e);
  for (auto* b : {&e.route_blk, &e.route_blk_stream, &e.route_out, &e.route_err, &e.seq_buf, &e.seq_desc, &e.lstm.wpk, &e.lstm.wpk4, &e.lstm.bias,
                  &e.lstm.wout, &e.lstm.bout, &e.state.seq})
    b->release();
  if (e.aux_stream) {
    (void)hipStreamSynchronize(e.aux_stream);
    (void)hipStreamDestroy(e.aux_stream);
    (void)hipEventDestroy(e.fork_ev);
    (void)hipEventDestroy(e.join_ev);
  }
  if (e.aux2_stream) {
    (void)hipStreamSynchronize(e.aux2_stream);
    (void)hipStreamDestroy(e.aux2_stream);
    (void)hipEventDestroy(e.join2_ev);
  }
  try {
    fd::comm_destroy(e);
  } catch (...) {
  }
  for (hipStream_t st : e.pipe_stream)
    if (st) {
      (void)hipStreamSynchronize(st);
      (void)hipStreamDestroy(st);
    }
  if (e.pipe_slot_stream) {
    (void)hipStreamSynchronize(e.pipe_slot_stream);
    (void)hipStreamDestroy(e.pipe_slot_stream);
  }
  if (e.pipe_entry_ev) (void)hipEventDestroy(e.pipe_entry_ev);
  for (int k = 0; k < Engine::kPipeSlots; ++k) {
    if (e.pipe_slot_ev[k]) (void)hipEventDestroy(e.pipe_slot_ev[k]);
    if (e.pipe_feat_ev[k]) (void)hipEventDestroy(e.pipe_feat_ev[k]);
    if (e.pipe_copy_ev[k]) (void)hipEventDestroy(e.pipe_copy_ev[k]);
    e.pipe_vec[k].release();
    e.pipe_out[k].release();
    e.pipe_seq[k].release();
  }
  for (int k = 0; k < Engine::kSplitRing; ++k) {
    if (e.pipe_done_ev[k]) (void)hipEventDestroy(e.pipe_done_ev[k]);
    e.pipe_split[k].release();
  }
  for (auto* b : {&e.state.uext, &e.state.mext, &e.state.vocab, &e.feat_ext}) b->release();
  for (auto& P1 : e.ens1)
    for (auto* b : {&P1.nodes[0], &P1.nodes[1], &P1.thr}) b->release();
  for (auto* b : {&e.ens.nodes[0], &e.ens.nodes[1], &e.ens.thr})
    b->release();
  {  // ingest codec tables and staging
    fd::IngestTables& t = e.ingest;
    for (auto* b : {&t.mkeys, &t.mvals, &t.stage_bytes, &t.stage_offsets, &t.stage_out}) b->release();
    for (int w = 0; w < 3; ++w) {
      t.vkeys[w].release();
      t.vvals[w].release();
    }
  }
  for (auto* b : {&e.state.pages, &e.state.keys, &e.state.merchants, &e.state.err, &e.state.sat,
                  &e.state.bucket_scr})
    b->release();
  for (auto& g : e.state.gs)
    for (auto* b : {&g.slot, &g.bucket_fill, &g.pairs, &g.ovf_cnt, &g.ovf_key, &g.ovf_b, &g.prep}) b->release();
  for (auto& ev : e.events) {
    (void)hipEventDestroy(ev.a);
    (void)hipEventDestroy(ev.b);
    if (ev.c) (void)hipEventDestroy(ev.c);
    if (ev.d) (void)hipEventDestroy(ev.d);
  }
  if (e.own_stream) (void)hipStreamDestroy(e.own_stream);
  delete eng;
  FD_API_END
}

// the new engine stream inherits the order of the old one over pipelined batches: their scoring is complete
// before anything queued on it (fd_score_batch_pipelined's outputs stay ordered on the engine stream)
static void rebind_stream(Engine& e, hipStream_t s) {
  for (int k = 0; k < Engine::kDoneRing; ++k)
    if (e.pipe_done_live[k] && s != e.stream) FD_HIP(hipStreamWaitEvent(s, e.pipe_done_ev[k], 0));
  e.stream = s;
}

int fd_engine_set_stream(fd_engine* eng, void* hip_stream) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  rebind_stream(e, static_cast<hipStream_t>(hip_stream));
  FD_API_END
}

int fd_engine_reset_stream(fd_engine* eng) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  rebind_stream(e, e.own_stream);
  FD_API_END
}

int fd_engine_sync(fd_engine* eng) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  if (e.comm.aborted) {  // streams behind an aborted exchange: bounded waits, then the abort's reason
    bool ok = fd::comm_sync_stream(e, e.comm.x_fwd);
    ok = fd::comm_sync_stream(e, e.stream) && ok;
    for (hipStream_t st : e.pipe_stream) ok = fd::comm_sync_stream(e, st) && ok;
    // the slot pass and the aux streams can be queued behind an aborted inbox event too (as fd_engine_destroy)
    for (hipStream_t st : {e.pipe_slot_stream, e.aux_stream, e.aux2_stream}) ok = fd::comm_sync_stream(e, st) && ok;
    FD_REQUIRE(ok, FD_ERR_HIP, "streams still busy " + std::to_string(e.comm.timeout_ms) +
                                   " ms after the communicators were aborted (" + e.comm.abort_reason + ")");
  }
  FD_HIP(hipStreamSynchronize(e.stream));
  if (e.comm.x_fwd) FD_HIP(hipStreamSynchronize(e.comm.x_fwd));
  for (hipStream_t st : e.pipe_stream)
    if (st) FD_HIP(hipStreamSynchronize(st));
  if (e.pipe_slot_stream) FD_HIP(hipStreamSynchronize(e.pipe_slot_stream));
  if (e.aux_stream) FD_HIP(hipStreamSynchronize(e.aux_stream));
  if (e.aux2_stream) FD_HIP(hipStreamSynchronize(e.aux2_stream));
  fd::route_check(e);
  FD_API_END
}

int fd_engine_set_timing(fd_engine* eng, int enable) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E_quiet(eng);
  e.timing = enable != 0;
  FD_API_END
}

int fd_engine_get_counter(fd_engine* eng, const char* key, int64_t* value) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E_quiet(eng);
  FD_REQUIRE(key && value, FD_ERR_INVALID_ARG, "null key/value");
  const std::string k(key);
  if (k == "pipelined_batches") {  // fd_score_batch_pipelined / fd_score_records_pipelined batches so far
    *value = (int64_t)e.pipe_iter_total;
  } else if (k == "ensemble_single_launches") {  // fd_forest_predict batches scored by the fused kernel over one
    // forest (probabilities, optionally raw scores; no leaf ids): config 2's timed kernel, ensemble_kernel<8,2>
    *value = (int64_t)e.ens_single_total;
  } else if (k == "latency_prebinned_batches") {  // latency pair launches that used the feature kernel's bins
    *value = (int64_t)e.prebin_total;
  } else if (k == "pipelined_split_batches") {  // of the compact ones: split rows (compact_vectors 2)
    *value = (int64_t)e.pipe_split_total;
  } else if (k == "pipelined_compact_batches") {  // of those: scored by the fused kernel from the compact 64-B
    // rows (no vectors requested), the variant the config-3/4 bench times
    *value = (int64_t)e.pipe_compact_total;
  } else if (k == "pipelined_host_ns") {  // host nanoseconds inside fd_score_batch_pipelined (HIP launches, event
    // records and waits of the pipelined step)
    *value = (int64_t)e.pipe_host_ns;
  } else if (k == "pipelined_slot_stream_batches") {  // of those: the slot pass on its own stream (slot_stream)
    *value = (int64_t)e.pipe_slot_stream_total;
  } else if (k == "window_saturated") {  // sliding windows: transactions whose 24 h window held K prior events
    // (its count may be truncated at the ring capacity); synchronises the engine's streams
    FD_REQUIRE(e.state.ready, FD_ERR_NOT_LOADED, "card state not initialised (fd_state_init)");
    FD_HIP(hipStreamSynchronize(e.stream));
    for (hipStream_t st : e.pipe_stream)
      if (st) FD_HIP(hipStreamSynchronize(st));
    unsigned long long v = 0;
    FD_HIP(hipMemcpy(&v, e.state.sat.ptr, 8, hipMemcpyDeviceToHost));
    *value = (int64_t)v;
  } else if (k == "sharded_steps") {  // fd_sharded_step calls so far
    *value = (int64_t)e.comm.steps.load();
  } else if (k == "rccl_ops") {  // RCCL operations issued by the engine's exchanges (send, recv, all-gather)
    *value = (int64_t)e.comm.ops.load();
  } else if (k.rfind("sharded_host_ns_", 0) == 0) {  // host time inside fd_sharded_step by phase
    int i = 0;
    while (i < fd::ShardComm::kHostPhases && k.compare(16, std::string::npos, fd::kShardHostPhase[i]) != 0) ++i;
    FD_REQUIRE(i < fd::ShardComm::kHostPhases, FD_ERR_INVALID_ARG, "unknown counter: " + k);
    *value = (int64_t)e.comm.host_ns[i].load();
  } else {
    FD_REQUIRE(false, FD_ERR_INVALID_ARG, "unknown counter: " + k);
  }
  FD_API_END
}

int fd_engine_set_option(fd_engine* eng, const char* key, int64_t value) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E_quiet(eng);
  FD_REQUIRE(key, FD_ERR_INVALID_ARG, "null key");
  const std::string k(key);
  if (k == "forest_kernel") {
    // 0 auto; 1 / 2 / 3 / 8 force kernel 1 / 3 / 4 / 6; 6 the tree-split path (forest.hip launch_forest)
    FD_REQUIRE(value == 0 || value == 1 || value == 2 || value == 3 || value == 6 || value == 8, FD_ERR_INVALID_ARG,
               "forest_kernel must be 0, 1, 2, 3, 6 or 8");
    e.forest_variant = (int)value;
  } else if (k == "ensemble") {  // 1 (default): fused forests + blend when applicable; 0: per-model kernels
    FD_REQUIRE(value == 0 || value == 1, FD_ERR_INVALID_ARG, "ensemble must be 0 or 1");
    e.ensemble_on = value != 0;
  } else if (k == "ensemble_owner") {  // fused kernel: 0 owner tree group rotates per chunk; 1 always group 0
    FD_REQUIRE(value == 0 || value == 1, FD_ERR_INVALID_ARG, "ensemble_owner must be 0 or 1");
    e.ens_owner_fixed = value != 0;
  } else if (k == "ensemble_prio") {  // fused kernel: 1 (default since round 6) its waves issue above the co-running
    // feature kernels' (s_setprio 2); 0 the same priority. Round 4 measured 1 slower (0.0929 vs 0.0908-0.0918 ms,
    // profiles/r04/prio); with round 6's split rows the feature chain is 20 us shorter than the fused kernel beside it
    // and the critical path is the fused kernel: with feature_prio 0, the driver's command 0.0944 -> 0.0897 ms and 200
    // steps 0.0826 -> 0.0812 (profiles/r06/prio)
    FD_REQUIRE(value == 0 || value == 1, FD_ERR_INVALID_ARG, "ensemble_prio must be 0 or 1");
    e.ens_prio = value != 0;
  } else if (k == "ensemble_chunks") {  // fused kernel's chunk layout: 0 auto (compact once the engine has RCCL
    // communicators, else wide), 1 wide (24 / 16 trees), 2 compact (20 / 12: LDS room for an RCCL kernel beside)
    FD_REQUIRE(value >= 0 && value <= 2, FD_ERR_INVALID_ARG, "ensemble_chunks must be 0, 1 or 2");
    e.ens_chunks = (int)value;
  } else if (k == "compact_vectors") {  // pipelined stream, the fused kernel's batches when nobody asked for the
    // vectors: 2 (default) split rows — the card-independent half finished by the slot pass, the bucket pass reads
    // 32-B prep records and writes the card half (features.hip Prep32 / RowA / RowB); 1 the compact 64-B row; 0 the
    // 64-wide vector (outputs identical in every mode)
    FD_REQUIRE(value >= 0 && value <= 2, FD_ERR_INVALID_ARG, "compact_vectors must be 0, 1 or 2");
    e.compact_vectors = (int)value;
  } else if (k == "latency_fused") {  // latency batches: 1 (default) both forests' walks in one launch and their
    // sums + the blend in another (fd::launch_forest_pair_blend); 0 the per-forest walk + sum launches + blend
    FD_REQUIRE(value == 0 || value == 1, FD_ERR_INVALID_ARG, "latency_fused must be 0 or 1");
    e.latency_fused = value != 0;
  } else if (k == "pipeline_lean") {  // fd_score_batch_pipelined's bucket pass: 1 (default) lean + deferred
    FD_REQUIRE(value == 0 || value == 1, FD_ERR_INVALID_ARG, "pipeline_lean must be 0 or 1");
    e.pipe_lean = value != 0;
  } else if (k == "pipeline_gather") {  // fd_score_batch_pipelined, batches of <= 4096 transactions (slot_gather on,
    // no slot stream): 1 (default) the gather bucket kernel (card slots found inside it, one feature launch), 0 the
    // slot + lean bucket pair of the large batches
    FD_REQUIRE(value == 0 || value == 1, FD_ERR_INVALID_ARG, "pipeline_gather must be 0 or 1");
    e.pipe_gather = value != 0;
  } else if (k == "latency_prebin") {  // latency batches with the LSTM head: the XGBoost + IsolationForest pair's
    // tree-split binning in the LSTM launch: 3 (default) inside the LSTM's own workgroups (a lifting level per
    // recurrence step; 2 where a thread would have more than two searches), 2 in extra workgroups after the LSTM's
    // own (they fill the CUs the LSTM's workgroups leave as they finish), 1 ahead of them; 0 the pair's own binning
    // launch
    FD_REQUIRE(value >= 0 && value <= 3, FD_ERR_INVALID_ARG, "latency_prebin must be 0, 1, 2 or 3");
    e.latency_prebin = value != 0;
    if (value) e.latency_prebin_mode = (int)value;
  } else if (k == "small_streams") {  // latency batches: 2 LSTM | other forests on two side streams, 1 one, 0 none
    FD_REQUIRE(value >= 0 && value <= 2, FD_ERR_INVALID_ARG, "small_streams must be 0, 1 or 2");
    e.small_streams = (int)value;
  } else if (k == "count_exchange") {  // fd_sharded_step's per-peer counts: 1 one ncclAllGather per batch, 0 2G
    // point-to-point operations in the records group, -1 (default) the all-gather from 4 ranks; set before
    // fd_comm_init or between steps with no batch prefetched (every rank the same)
    FD_REQUIRE(value >= -1 && value <= 1, FD_ERR_INVALID_ARG, "count_exchange must be -1, 0 or 1");
    FD_REQUIRE(!e.comm.pending, FD_ERR_INVALID_ARG, "count_exchange: a prefetched batch's counts are in flight");
    e.comm.count_mode = (int)value;
    e.comm.count_gather = value == 1 || (value < 0 && e.comm.world >= 4);
  } else if (k == "comm_timeout_ms") {  // fd_sharded_step: the split-size wait gives up (FD_ERR_HIP) after this
    FD_REQUIRE(value >= 1, FD_ERR_INVALID_ARG, "comm_timeout_ms must be >= 1");
    e.comm.timeout_ms = value;
  } else if (k == "stream_priority") {  // HIP stream priorities (ROCm keeps a hardware-queue pool per priority):
    // 0 all default; 1 the two pipeline streams high; 2 + the sharded step's forward stream low; 3 (default) + it
    // high. Set before the first pipelined call / fd_comm_init (the streams are created then). With every stream
    // at the default priority the process's 4 hardware queues are shared by the engine stream, the two pipeline
    // streams, the forward stream and RCCL's own: the engine stream's output copy (waiting for batch i's
    // forests) then sat in front of batch i+1's feature kernels in one queue — the native sharded step measured
    // 0.137 ms per 64 k batch at 0, 0.093 at 2 / 3 (the direct step 0.089 either way).
    FD_REQUIRE(value >= 0 && value <= 3, FD_ERR_INVALID_ARG, "stream_priority must be in 0..3");
    FD_REQUIRE(!e.pipe_stream[0] && !e.comm.x_fwd, FD_ERR_INVALID_ARG,
               "stream_priority: set before the first pipelined call and fd_comm_init");
    e.stream_prio = (int)value;
  } else if (k == "bucket_keys") {  // feature bucket pass: transactions per bucket workgroup, 0 auto (8 up to
    // 2048 transactions, 16 below 8192, else 128), else a power of two in 8..512
    FD_REQUIRE(value == 0 || (value >= 8 && value <= 512 && (value & (value - 1)) == 0), FD_ERR_INVALID_ARG,
               "bucket_keys must be 0 or a power of two in 8..512");
    e.state.bucket_keys = (int)value;
  } else if (k == "ensemble_bin_global") {  // the fused kernel's compact rows: 1 binned by searches of the merged
    // tables where they lie (L2), chunk 0's DMA issued at once; 0 the tables staged in LDS first
    FD_REQUIRE(value == 0 || value == 1, FD_ERR_INVALID_ARG, "ensemble_bin_global must be 0 or 1");
    e.ens_bin_global = value != 0;
  } else if (k == "lean_group") {  // pipelined stream: the lean bucket kernel's grouping of a bucket's keys by card,
    // 0 rank sort (first m threads, whole list each), 1 rank sort split over all threads, 2 (default) LDS hash table
    FD_REQUIRE(value >= 0 && value <= 2, FD_ERR_INVALID_ARG, "lean_group must be 0, 1 or 2");
    e.state.lean_group = (int)value;
  } else if (k == "slot_gather") {  // batches of <= 4096 transactions outside the pipelined stream: card slots found
    // inside the bucket kernel, no slot launch (1, default) / the slot kernel first (0)
    FD_REQUIRE(value == 0 || value == 1, FD_ERR_INVALID_ARG, "slot_gather must be 0 or 1");
    e.state.slot_gather = value != 0;
  } else if (k == "slot_stream") {  // fd_score_batch_pipelined: batch i's slot pass on a stream of its own (1 high
    // priority, 2 low; 0 on pipe_stream[i & 1] behind batch i-2's fused kernel; -1 auto by the card table's size),
    // set before the first pipelined call
    FD_REQUIRE(value >= -1 && value <= 2, FD_ERR_INVALID_ARG, "slot_stream must be -1, 0, 1 or 2");
    FD_REQUIRE(!e.pipe_slot_stream || (int)value == e.pipe_slot_mode, FD_ERR_INVALID_ARG,
               "slot_stream: set before the first pipelined call");
    e.pipe_slot_mode = (int)value;
  } else if (k == "slot_prio") {  // pipelined stream: 1 the slot kernel's waves issue at priority 2, 0 (default) not
    FD_REQUIRE(value == 0 || value == 1, FD_ERR_INVALID_ARG, "slot_prio must be 0 or 1");
    e.state.slot_prio = value != 0;
  } else if (k == "feature_prio") {  // pipelined stream: 1 the lean bucket kernel's waves issue at priority 2 (round 5's
    // default: DESIGN §3, 0.0857 -> 0.0843 ms per config-4 step at 200 steps), 0 (default since round 6) at the
    // default priority, below the fused kernel (ensemble_prio)
    FD_REQUIRE(value == 0 || value == 1, FD_ERR_INVALID_ARG, "feature_prio must be 0 or 1");
    e.state.feat_prio = value != 0;
  } else if (k == "bucket_spread") {  // feature bucket pass, >= 8 k transactions: 1 (default) card segments
    // round-robin over the 4 waves
    FD_REQUIRE(value == 0 || value == 1, FD_ERR_INVALID_ARG, "bucket_spread must be 0 or 1");
    e.state.bucket_spread = value != 0;
  } else if (k == "timing_every") {  // kernel timing (fd_timing_*): HIP events on one launch in N of each kind
    FD_REQUIRE(value >= 1 && value <= 1000000, FD_ERR_INVALID_ARG, "timing_every must be >= 1");
    e.timing_every = (int)value;
    for (auto& q : e.timing_seq) q = 0;  // the next launch of every kind is a timed one
  } else if (k == "seq_ring_lstm") {  // latency batches: 1 (default) the LSTM reads card histories from the ring
    FD_REQUIRE(value == 0 || value == 1, FD_ERR_INVALID_ARG, "seq_ring_lstm must be 0 or 1");
    e.seq_ring_lstm = value != 0;
  } else if (k == "lstm_rows") {  // LSTM tile: 0 auto (4 below 4096 transactions, else 16), 4 or 16
    FD_REQUIRE(value == 0 || value == 4 || value == 16, FD_ERR_INVALID_ARG, "lstm_rows must be 0, 4 or 16");
    e.lstm_rows = (int)value;
  } else if (k == "ingest_stop_after") {  // diagnostics: 0 full; 1 stage; 2 + structure; 3 + members
    FD_REQUIRE(value >= 0 && value <= 3, FD_ERR_INVALID_ARG, "ingest_stop_after must be in 0..3");
    e.ingest.stop_after = (int)value;
  } else if (k == "rule_fraud_threshold_permille") {  // JobConfig.fraudThreshold x 1000
    FD_REQUIRE(value >= 0 && value <= 1000, FD_ERR_INVALID_ARG, "rule_fraud_threshold_permille must be in 0..1000");
    e.state.tp_threshold = (double)value / 1000.0;
  } else {
    throw fd::Error(FD_ERR_INVALID_ARG, "unknown option: " + k);
  }
  FD_API_END
}

int fd_timing_read(fd_engine* eng, int kind, double* total_ms, int64_t* launches) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E_quiet(eng);
  double tot = 0.0;
  int64_t cnt = 0;
  for (size_t i = 0; i < e.events_used; ++i) {
    if (kind >= 0 && e.events[i].kind != kind) continue;
    FD_HIP(hipEventSynchronize(e.events[i].b));
    float ms = 0.f;
    FD_HIP(hipEventElapsedTime(&ms, e.events[i].a, e.events[i].b));
    tot += ms;
    if (e.events[i].split) {
      FD_HIP(hipEventSynchronize(e.events[i].d));
      FD_HIP(hipEventElapsedTime(&ms, e.events[i].c, e.events[i].d));
      tot += ms;
    }
    ++cnt;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = cnt;
  FD_API_END
}

int fd_timing_reset(fd_engine* eng) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E_quiet(eng);
  for (size_t i = 0; i < e.events_used; ++i) {  // pairs on 2+ streams
    FD_HIP(hipEventSynchronize(e.events[i].b));
    if (e.events[i].split) FD_HIP(hipEventSynchronize(e.events[i].d));
  }
  e.events_used = 0;
  FD_API_END
}

int fd_load_forest(fd_engine* eng, int slot, const fd_forest_params* params, const fd_tree_arrays* trees) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(params && trees, FD_ERR_INVALID_ARG, "null params/trees");
  fd::PackedForest& pf = slot_of(e, slot);
  FD_HIP(hipStreamSynchronize(e.stream));  // a reload must not race an in-flight predict
  pf.loaded = false;
  fd::repack_forest(pf, *params, *trees);
  FD_API_END
}

int fd_pack_forest_host(const fd_forest_params* params, const fd_tree_arrays* trees, void* blob,
                        int64_t blob_cap, int32_t* leaf_ids, int64_t ids_cap, fd_pack_info* info) {
  FD_API_BEGIN
  FD_REQUIRE(params && trees && info, FD_ERR_INVALID_ARG, "null params/trees/info");
  const fd::HostPack hp = fd::pack_forest_host(*params, *trees);
  info->n_trees = hp.n_trees;
  info->n_chunks = hp.n_chunks;
  info->chunk = hp.chunk;
  info->depth = hp.depth;
  info->tree_bytes = (int64_t)hp.tree_bytes;
  info->chunk_stride = (int64_t)hp.chunk_stride;
  info->blob_bytes = (int64_t)hp.blob.size();
  info->n_leaf_ids = (int64_t)hp.leaf_ids.size();
  info->base_margin = hp.base_margin;
  info->layout = 0;
  info->n_thresholds = (int64_t)hp.b_thr.size();
  info->bin_steps = hp.bin_steps;
  if (blob) {
    FD_REQUIRE(blob_cap >= (int64_t)hp.blob.size(), FD_ERR_INVALID_ARG, "blob buffer too small");
    std::memcpy(blob, hp.blob.data(), hp.blob.size());
  }
  if (leaf_ids) {
    FD_REQUIRE(ids_cap >= (int64_t)hp.leaf_ids.size(), FD_ERR_INVALID_ARG, "leaf id buffer too small");
    std::memcpy(leaf_ids, hp.leaf_ids.data(), hp.leaf_ids.size() * sizeof(int32_t));
  }
  FD_API_END
}

int fd_pack_forest_binned_host(const fd_forest_params* params, const fd_tree_arrays* trees, void* blob,
                               int64_t blob_cap, float* thresholds, int64_t thr_cap, int32_t* offsets,
                               fd_pack_info* info) {
  FD_API_BEGIN
  FD_REQUIRE(params && trees && info, FD_ERR_INVALID_ARG, "null params/trees/info");
  const fd::HostPack hp = fd::pack_forest_host(*params, *trees);
  FD_REQUIRE(hp.binned, FD_ERR_UNSUPPORTED,
             "forest has no binned layout (depth > 8 or > 65534 distinct thresholds in a feature)");
  info->n_trees = hp.n_trees;
  info->n_chunks = hp.b_n_chunks;
  info->chunk = hp.b_chunk;
  info->depth = hp.depth;
  info->tree_bytes = (int64_t)hp.b_tree_bytes;
  info->chunk_stride = (int64_t)hp.b_chunk_stride;
  info->blob_bytes = (int64_t)hp.b_blob.size();
  info->n_leaf_ids = (int64_t)hp.leaf_ids.size();
  info->base_margin = hp.base_margin;
  info->layout = 1;
  info->n_thresholds = (int64_t)hp.b_thr.size();
  info->bin_steps = hp.bin_steps;
  if (blob) {
    FD_REQUIRE(blob_cap >= (int64_t)hp.b_blob.size(), FD_ERR_INVALID_ARG, "blob buffer too small");
    std::memcpy(blob, hp.b_blob.data(), hp.b_blob.size());
  }
  if (thresholds) {
    FD_REQUIRE(thr_cap >= (int64_t)hp.b_thr.size(), FD_ERR_INVALID_ARG, "threshold buffer too small");
    std::memcpy(thresholds, hp.b_thr.data(), hp.b_thr.size() * sizeof(float));
  }
  if (offsets) std::memcpy(offsets, hp.b_thr_off.data(), hp.b_thr_off.size() * sizeof(int32_t));
  FD_API_END
}

int fd_load_xgboost_json(fd_engine* eng, int slot, const char* path) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::PackedForest& pf = slot_of(e, slot);
  fd::XgbModel m;
  fd::read_xgboost_json(path, m);
  fd_forest_params p{};
  p.kind = FD_FOREST_XGB_BINARY_LOGISTIC;
  p.num_feature = m.num_feature;
  p.base_score = m.base_score;
  fd_tree_arrays t{};
  t.n_trees = (int32_t)(m.offsets.size() - 1);
  t.tree_offsets = m.offsets.data();
  t.left = m.left.data();
  t.right = m.right.data();
  t.feature = m.feature.data();
  t.threshold = m.threshold.data();
  t.default_left = m.default_left.data();
  t.leaf_value = m.leaf_value.data();
  FD_REQUIRE(t.n_trees > 0, FD_ERR_INVALID_ARG, "xgboost json: no trees");
  FD_HIP(hipStreamSynchronize(e.stream));  // a reload must not race an in-flight predict
  pf.loaded = false;
  fd::repack_forest(pf, p, t);
  FD_API_END
}

int fd_xgboost_json_read(const char* path, fd_forest_params* params, int32_t* n_trees, int64_t* n_nodes,
                         fd_tree_arrays* trees) {
  FD_API_BEGIN
  fd::XgbModel m;
  fd::read_xgboost_json(path, m);
  const int32_t T = (int32_t)(m.offsets.size() - 1);
  const int64_t M = (int64_t)m.left.size();
  if (params) {
    *params = fd_forest_params{};
    params->kind = FD_FOREST_XGB_BINARY_LOGISTIC;
    params->num_feature = m.num_feature;
    params->base_score = m.base_score;
  }
  if (n_trees) *n_trees = T;
  if (n_nodes) *n_nodes = M;
  if (trees) {
    FD_REQUIRE(trees->tree_offsets && trees->left && trees->right && trees->feature && trees->threshold &&
                   trees->default_left && trees->leaf_value,
               FD_ERR_INVALID_ARG, "incomplete output arrays");
    trees->n_trees = T;
    std::memcpy(const_cast<int64_t*>(trees->tree_offsets), m.offsets.data(), (size_t)(T + 1) * 8);
    std::memcpy(const_cast<int32_t*>(trees->left), m.left.data(), (size_t)M * 4);
    std::memcpy(const_cast<int32_t*>(trees->right), m.right.data(), (size_t)M * 4);
    std::memcpy(const_cast<int32_t*>(trees->feature), m.feature.data(), (size_t)M * 4);
    std::memcpy(const_cast<double*>(trees->threshold), m.threshold.data(), (size_t)M * 8);
    std::memcpy(const_cast<uint8_t*>(trees->default_left), m.default_left.data(), (size_t)M);
    std::memcpy(const_cast<double*>(trees->leaf_value), m.leaf_value.data(), (size_t)M * 8);
  }
  FD_API_END
}

int fd_unload_forest(fd_engine* eng, int slot) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::PackedForest& pf = slot_of(e, slot);
  FD_HIP(hipStreamSynchronize(e.stream));
  pf.blob.release();
  pf.leaf_ids.release();
  pf.b_blob.release();
  pf.b_thr.release();
  pf.b_thr_off.release();
  for (auto* b : {&pf.split.bins, &pf.split.nan, &pf.split.leaves}) b->release();
  pf.binned = false;
  pf.loaded = false;
  pf.gen = 0;  // any ensemble plan built over this slot is stale
  FD_API_END
}

int fd_forest_info(fd_engine* eng, int slot, int32_t* n_trees, int32_t* depth, int32_t* num_feature) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::PackedForest& pf = slot_of(e, slot);
  FD_REQUIRE(pf.loaded, FD_ERR_NOT_LOADED, "Model in slot " + std::to_string(slot) + " not loaded");
  if (n_trees) *n_trees = pf.n_trees;
  if (depth) *depth = pf.depth;
  if (num_feature) *num_feature = pf.num_feature;
  FD_API_END
}

int fd_forest_predict_device(fd_engine* eng, int slot, const float* d_X, int64_t n, int32_t ld,
                             double* d_prob, double* d_raw, int32_t* d_leaf) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::PackedForest& pf = slot_of(e, slot);
  FD_REQUIRE(pf.loaded, FD_ERR_NOT_LOADED, "Model in slot " + std::to_string(slot) + " not loaded");
  FD_REQUIRE(n >= 0, FD_ERR_INVALID_ARG, "negative n");
  fd::launch_forest(e, pf, d_X, n, ld, d_prob, d_raw, d_leaf);
  FD_API_END
}

int fd_forest_predict_host(fd_engine* eng, int slot, const float* X, int64_t n, int32_t ld, double* prob,
                           double* raw, int32_t* leaf) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::PackedForest& pf = slot_of(e, slot);
  FD_REQUIRE(pf.loaded, FD_ERR_NOT_LOADED, "Model in slot " + std::to_string(slot) + " not loaded");
  FD_REQUIRE(n >= 0 && ld > 0 && X && prob, FD_ERR_INVALID_ARG, "bad arguments");
  if (n == 0) return FD_OK;
  const size_t xb = (size_t)n * ld * sizeof(float);
  e.stage_in.ensure(xb);
  e.stage_out0.ensure((size_t)n * sizeof(double));
  if (raw) e.stage_out1.ensure((size_t)n * sizeof(double));
  if (leaf) e.stage_out2.ensure((size_t)n * pf.n_trees * sizeof(int32_t));
  FD_HIP(hipMemcpyAsync(e.stage_in.ptr, X, xb, hipMemcpyHostToDevice, e.stream));
  fd::launch_forest(e, pf, e.stage_in.as<float>(), n, ld, e.stage_out0.as<double>(),
                    raw ? e.stage_out1.as<double>() : nullptr, leaf ? e.stage_out2.as<int32_t>() : nullptr);
  FD_HIP(hipMemcpyAsync(prob, e.stage_out0.ptr, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, e.stream));
  if (raw)
    FD_HIP(hipMemcpyAsync(raw, e.stage_out1.ptr, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, e.stream));
  if (leaf)
    FD_HIP(hipMemcpyAsync(leaf, e.stage_out2.ptr, (size_t)n * pf.n_trees * sizeof(int32_t),
                          hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  FD_API_END
}

int fd_state_init(fd_engine* eng, const fd_state_params* params) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(params, FD_ERR_INVALID_ARG, "null params");
  FD_HIP(hipStreamSynchronize(e.stream));
  fd::state_init(e, *params);
  FD_API_END
}

int fd_state_clear(fd_engine* eng) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::state_clear(e);
  FD_API_END
}

int fd_state_info(fd_engine* eng, int64_t* capacity, int64_t* cards) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::features_check(e);
  if (capacity) *capacity = e.state.cap;
  if (cards) *cards = fd::state_count(e);
  FD_API_END
}

int fd_state_load_users_host(fd_engine* eng, const fd_users* users) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(users, FD_ERR_INVALID_ARG, "null users");
  fd::load_users(e, *users);
  FD_API_END
}

int fd_load_merchants_host(fd_engine* eng, const fd_merchants* merchants) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(merchants, FD_ERR_INVALID_ARG, "null merchants");
  FD_HIP(hipStreamSynchronize(e.stream));
  fd::load_merchants(e, *merchants);
  FD_API_END
}

int fd_features_device(fd_engine* eng, const fd_txn_batch* txns, int64_t n, float* d_vectors, double* d_raw) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(txns, FD_ERR_INVALID_ARG, "null txns");
  fd::launch_features(e, *txns, n, d_vectors, d_raw);
  FD_API_END
}

int fd_features_host(fd_engine* eng, const fd_txn_batch* txns, int64_t n, float* vectors, double* raw) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(txns && vectors && n >= 0, FD_ERR_INVALID_ARG, "bad arguments");
  if (n == 0) return FD_OK;
  // stage the SoA columns in one device buffer (8-byte aligned segments)
  const size_t seg8 = (size_t)n * 8, seg4 = ((size_t)n * 4 + 7) / 8 * 8, seg1 = ((size_t)n + 7) / 8 * 8;
  const size_t total = 4 * seg8 + seg4 + 3 * seg1;
  e.feat_in.ensure(total);
  char* b = e.feat_in.as<char>();
  fd_txn_batch d{};
  size_t off = 0;
  auto put = [&](const void* src, size_t bytes, size_t seg) -> void* {
    FD_REQUIRE(src, FD_ERR_INVALID_ARG, "incomplete transaction batch");
    void* dst = b + off;
    FD_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, e.stream));
    off += seg;
    return dst;
  };
  d.card_key = (const uint64_t*)put(txns->card_key, n * 8, seg8);
  d.ts_ms = (const int64_t*)put(txns->ts_ms, n * 8, seg8);
  d.amount_cents = (const int64_t*)put(txns->amount_cents, n * 8, seg8);
  d.device_fp = (const uint64_t*)put(txns->device_fp, n * 8, seg8);
  d.merchant = (const int32_t*)put(txns->merchant, n * 4, seg4);
  d.ip_class = (const uint8_t*)put(txns->ip_class, n, seg1);
  d.hour = (const uint8_t*)put(txns->hour, n, seg1);
  d.weekend = (const uint8_t*)put(txns->weekend, n, seg1);
  e.feat_vec.ensure((size_t)n * FD_VECTOR_WIDTH * 4 + (raw ? (size_t)n * FD_RAW_FEATURES * 8 : 0));
  float* dv = e.feat_vec.as<float>();
  double* dr = raw ? reinterpret_cast<double*>(e.feat_vec.as<char>() + (size_t)n * FD_VECTOR_WIDTH * 4) : nullptr;
  fd::launch_features(e, d, n, dv, dr);
  FD_HIP(hipMemcpyAsync(vectors, dv, (size_t)n * FD_VECTOR_WIDTH * 4, hipMemcpyDeviceToHost, e.stream));
  if (raw) FD_HIP(hipMemcpyAsync(raw, dr, (size_t)n * FD_RAW_FEATURES * 8, hipMemcpyDeviceToHost, e.stream));
  fd::features_check(e);  // synchronises
  FD_API_END
}

int fd_score_matrix_device(fd_engine* eng, const fd_blend_params* params, const int32_t* slots,
                           const double* const* ext_probs, const uint8_t* present, const float* d_X,
                           int64_t n, int32_t ld, double* d_model_probs, double* d_fraud_prob,
                           double* d_confidence, uint8_t* d_decision, uint8_t* d_risk) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(params && d_X && ld > 0 && n >= 0, FD_ERR_INVALID_ARG, "bad arguments");
  score_matrix(e, *params, slots, ext_probs, present, d_X, n, ld, d_model_probs, d_fraud_prob, d_confidence,
               d_decision, d_risk);
  FD_API_END
}

int fd_score_matrix_host(fd_engine* eng, const fd_blend_params* params, const int32_t* slots,
                         const double* const* ext_probs, const uint8_t* present, const float* X, int64_t n,
                         int32_t ld, double* model_probs, double* fraud_prob, double* confidence,
                         uint8_t* decision, uint8_t* risk) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(params && slots && X && fraud_prob && ld > 0 && n >= 0, FD_ERR_INVALID_ARG, "bad arguments");
  FD_REQUIRE(params->n_models > 0 && params->n_models <= FD_MAX_MODELS, FD_ERR_INVALID_ARG, "n_models out of range");
  if (n == 0) return FD_OK;
  const int M = params->n_models;
  const size_t xb = (size_t)n * ld * sizeof(float);
  e.stage_in.ensure(xb);
  e.scratch_probs.ensure((size_t)n * M * sizeof(double));
  e.stage_out0.ensure((size_t)n * sizeof(double));
  e.stage_out1.ensure((size_t)n * sizeof(double));
  e.stage_out2.ensure((size_t)n);
  e.stage_out3.ensure((size_t)n);
  FD_HIP(hipMemcpyAsync(e.stage_in.ptr, X, xb, hipMemcpyHostToDevice, e.stream));
  double* dMP = e.scratch_probs.as<double>();
  const double* dext[FD_MAX_MODELS] = {};
  for (int m = 0; m < M; ++m) {
    if (slots[m] >= 0 || (present && !present[m])) continue;
    FD_REQUIRE(ext_probs && ext_probs[m], FD_ERR_INVALID_ARG, "model without slot needs an external probability column");
    FD_HIP(hipMemcpyAsync(dMP + (size_t)m * n, ext_probs[m], (size_t)n * sizeof(double), hipMemcpyHostToDevice,
                          e.stream));
    dext[m] = dMP + (size_t)m * n;
  }
  score_matrix(e, *params, slots, dext, present, e.stage_in.as<float>(), n, ld, dMP, e.stage_out0.as<double>(),
               e.stage_out1.as<double>(), e.stage_out2.as<uint8_t>(), e.stage_out3.as<uint8_t>());
  if (model_probs)
    FD_HIP(hipMemcpyAsync(model_probs, dMP, (size_t)n * M * sizeof(double), hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipMemcpyAsync(fraud_prob, e.stage_out0.ptr, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, e.stream));
  if (confidence)
    FD_HIP(hipMemcpyAsync(confidence, e.stage_out1.ptr, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, e.stream));
  if (decision) FD_HIP(hipMemcpyAsync(decision, e.stage_out2.ptr, (size_t)n, hipMemcpyDeviceToHost, e.stream));
  if (risk) FD_HIP(hipMemcpyAsync(risk, e.stage_out3.ptr, (size_t)n, hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  FD_API_END
}

static void score_batch_body(Engine& e, const fd_blend_params& p, const int32_t* slots, const double* const* ext,
                             const uint8_t* present, const fd_txn_batch& t, int64_t n, float* d_vectors,
                             double* dMP, double* dfp, double* dconf, uint8_t* ddec, uint8_t* drisk) {
  float* vec = d_vectors;
  if (!vec) {
    e.feat_vec.ensure((size_t)n * FD_VECTOR_WIDTH * 4);
    vec = e.feat_vec.as<float>();
  }
  float* seq = lstm_seq_buffer(e, p, slots, present, n);
  // latency batches: the LSTM (4-row kernel) reads each card's last transaction's sequence from the history ring,
  // which nothing rewrites before it runs (the next batch's features follow on this stream); the feature kernel
  // writes only the other rows
  unsigned long long* desc = nullptr;
  if (seq && e.seq_ring_lstm && n < 4096 && (e.lstm_rows == 0 || e.lstm_rows == 4)) {
    e.seq_desc.ensure((size_t)n * sizeof(unsigned long long));
    desc = e.seq_desc.as<unsigned long long>();
    // a transaction whose card probe fails (table full) gets no descriptor from the feature kernel: the gather
    // kernel writes kSeqMaterialized for it; the slot-kernel path starts from all-materialized (bit 63 set)
    if (!e.state.slot_gather) FD_HIP(hipMemsetAsync(desc, 0xff, (size_t)n * sizeof(unsigned long long), e.stream));
  }
  fd::launch_features(e, t, n, vec, nullptr, seq, nullptr, nullptr, false, 0, nullptr, false, desc);
  score_matrix(e, p, slots, ext, present, vec, n, FD_VECTOR_WIDTH, dMP, dfp, dconf, ddec, drisk, seq, e.state.S,
               nullptr, nullptr, false, desc);
}

int fd_score_batch_device(fd_engine* eng, const fd_blend_params* params, const int32_t* slots,
                          const double* const* ext_probs, const uint8_t* present, const fd_txn_batch* txns,
                          int64_t n, float* d_vectors, double* d_model_probs, double* d_fraud_prob,
                          double* d_confidence, uint8_t* d_decision, uint8_t* d_risk) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(params && txns && n >= 0, FD_ERR_INVALID_ARG, "bad arguments");
  if (n == 0) return FD_OK;
  FD_REQUIRE(slots != nullptr && d_fraud_prob != nullptr, FD_ERR_INVALID_ARG, "null slots/output");
  score_batch_body(e, *params, slots, ext_probs, present, *txns, n, d_vectors, d_model_probs, d_fraud_prob,
                   d_confidence, d_decision, d_risk);
  FD_API_END
}

// fd_score_batch_pipelined's outputs: engine staging -> the caller's buffers, on the engine stream (one thread per
// transaction; null destinations are skipped); result records (routed batches) as 8-byte words
__global__ void __launch_bounds__(256)
pipe_out_copy_kernel(const double* __restrict__ fp, const double* __restrict__ conf, const uint8_t* __restrict__ dec,
                     const uint8_t* __restrict__ risk, const double* __restrict__ mp, int n_mp, int64_t n,
                     double* __restrict__ o_fp, double* __restrict__ o_conf, uint8_t* __restrict__ o_dec,
                     uint8_t* __restrict__ o_risk, double* __restrict__ o_mp, const float4* __restrict__ vec,
                     float4* __restrict__ o_vec, const uint64_t* __restrict__ res, uint64_t* __restrict__ o_res) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (o_vec) {  // the vectors: 16 float4 per row, one float4 per thread over the whole grid
    const int64_t total = n * (FD_VECTOR_WIDTH / 4);
    for (int64_t q = i; q < total; q += stride) o_vec[q] = vec[q];
  }
  if (o_res) {
    const int64_t total = n * (int64_t)(sizeof(fd::ResultRecord) / 8);
    for (int64_t q = i; q < total; q += stride) o_res[q] = res[q];
  }
  if (i >= n) return;
  if (o_fp) o_fp[i] = fp[i];
  if (o_conf) o_conf[i] = conf[i];
  if (o_dec) o_dec[i] = dec[i];
  if (o_risk) o_risk[i] = risk[i];
  for (int m = 0; m < n_mp; ++m) o_mp[(size_t)m * n + i] = mp[(size_t)m * n + i];
}

// One micro-batch of the pipelined stream: transaction columns (txns) or routed 48-B records (records, whose scores
// leave as 24-B result records in d_results). Shared by fd_score_batch_pipelined and fd_score_records_pipelined.
static void pipe_step(Engine& e, const fd_blend_params* params, const int32_t* slots, const double* const* ext_probs,
                      const uint8_t* present, const fd_txn_batch* txns, const void* records, int64_t n,
                      float* d_vectors, double* d_model_probs, double* d_fraud_prob, double* d_confidence,
                      uint8_t* d_decision, uint8_t* d_risk, void* d_results, void* input_ready,
                      bool results_in_place = false) {
  for (int k = 0; k < 2; ++k)
    if (!e.pipe_stream[k]) e.pipe_stream[k] = fd::make_stream(e.stream_prio >= 1 ? 1 : 0);
  if (e.pipe_slot_mode < 0)  // auto: where the feature chain outlasts the fused kernel (random card traffic over a
    // large table), not where an earlier slot pass only adds contention beside it
    e.pipe_slot_mode = (e.state.ready && e.state.cap >= (1ll << 26)) ? 2 : 0;
  if (e.pipe_slot_mode && !e.pipe_slot_stream) {
    e.pipe_slot_stream = fd::make_stream(e.pipe_slot_mode == 1 ? 1 : -1);
    for (int k = 0; k < Engine::kPipeSlots; ++k) FD_HIP(hipEventCreateWithFlags(&e.pipe_slot_ev[k], kStreamEventFlags));
  }
  if (!e.pipe_entry_ev) {
    FD_HIP(hipEventCreateWithFlags(&e.pipe_entry_ev, kStreamEventFlags));
    for (int k = 0; k < Engine::kPipeSlots; ++k) {
      FD_HIP(hipEventCreateWithFlags(&e.pipe_feat_ev[k], kStreamEventFlags));
      FD_HIP(hipEventCreateWithFlags(&e.pipe_copy_ev[k], kStreamEventFlags));
    }
    for (int k = 0; k < Engine::kDoneRing; ++k) FD_HIP(hipEventCreateWithFlags(&e.pipe_done_ev[k], kStreamEventFlags));
  }
  // Batch i: buffer slot s = i mod 2, its features and its scoring on Sc = pipe_stream[i & 1] (Sf: the same
  // stream). Card-state order: batch i's bucket pass after batch i-1's (an event). Buffer s is free once batch
  // i-2's scoring is done (the same queue). Outputs: the engine stream waits for batch i's scoring. (Measured and
  // dropped: one feature stream for every batch + two scoring streams, ring of three buffers — the third stream
  // shares a hardware queue with a scoring stream: 567 vs 742 M txn/s)
  constexpr int nbuf = 2;
  const int s = (int)(e.pipe_iter % (unsigned long long)nbuf);
  const int prev = s ^ 1;
  hipStream_t Sc = e.pipe_stream[e.pipe_iter & 1];
  hipStream_t Sf = Sc;
  // option slot_stream: the slot pass on Ss, after what it reads (the entry order, the inputs) and batch i-2's
  // bucket pass (scratch set s: its fill counts and keys are consumed and reset there); feat_slot_kernel only
  // finds / inserts card keys, which the bucket passes of earlier batches never change
  hipStream_t Ss = e.pipe_slot_stream;
  if (e.pipe_dirty) {  // work queued on e.stream by other calls (state loads, snapshots, ...) comes first
    FD_HIP(hipEventRecord(e.pipe_entry_ev, e.stream));
    FD_HIP(hipStreamWaitEvent(Sf, e.pipe_entry_ev, 0));
    if (Ss) FD_HIP(hipStreamWaitEvent(Ss, e.pipe_entry_ev, 0));
    e.pipe_dirty = false;
  }
  if (input_ready) FD_HIP(hipStreamWaitEvent(Sf, static_cast<hipEvent_t>(input_ready), 0));
  if (Ss && input_ready) FD_HIP(hipStreamWaitEvent(Ss, static_cast<hipEvent_t>(input_ready), 0));
  if (Ss && e.pipe_feat_live[s]) FD_HIP(hipStreamWaitEvent(Ss, e.pipe_feat_ev[s], 0));
  // the slot's vectors are rewritten below: after batch i-nbuf's output copy if that one read them
  if (e.pipe_copy_live[s] && e.pipe_copy_vec[s]) FD_HIP(hipStreamWaitEvent(Sf, e.pipe_copy_ev[s], 0));
  // mode 1: the slot pass (scratch set s & 1, untouched by batch i-1) runs at once; the bucket pass waits for
  // batch i-1's card updates
  hipEvent_t before_buckets = e.pipe_feat_live[prev] ? e.pipe_feat_ev[prev] : nullptr;
  // the fused kernel alone reads the vectors and nobody asked for them: the compact form (64 instead of 256 B per
  // transaction written here and read by the ensemble kernel, fd_internal.h kCompactSlot), or split rows
  // (compact 2: the slot pass writes the card-independent half, the bucket pass reads 32-B instead of 64-B prep
  // records; the lean bucket pass only, and not with LSTM history in the card state)
  int compact = (e.compact_vectors && d_vectors == nullptr && fd::ensemble_applies(e, *params, slots, present, n))
                    ? e.compact_vectors : 0;
  e.pipe_vec[s].ensure((size_t)n * FD_VECTOR_WIDTH * 4);
  float* vec = e.pipe_vec[s].as<float>();
  const int sr = (int)(e.pipe_iter % (unsigned long long)Engine::kSplitRing);  // split rows: this batch's ring buffer
  float* seq = nullptr;
  bool want_seq = false;
  for (int m = 0; m < params->n_models && m < FD_MAX_MODELS; ++m)
    want_seq = want_seq || (slots && slots[m] == FD_SLOT_LSTM && !(present && !present[m]));
  if (want_seq) {
    FD_REQUIRE(e.state.ready && e.state.S > 0, FD_ERR_INVALID_ARG,
               "the LSTM head needs card history: fd_state_params.seq_len > 0");
    e.pipe_seq[s].ensure((size_t)n * e.state.S * fd::kSeqInput * sizeof(float));
    seq = e.pipe_seq[s].as<float>();
  }
  // latency-sized batches: the gather kernel (slot pass inside the bucket launch) instead of the slot + lean pair,
  // whose two launches cost 39 us per 1 k batch against its 18; it waits for batch i-1's card updates
  // (before_buckets) like the lean pass
  const bool lean = e.pipe_lean && !(e.pipe_gather && e.state.slot_gather && n <= fd::kGatherBatchMax && !Ss);
  if (compact == 2 && (!lean || want_seq || e.state.S > 0)) compact = 1;
  if (compact == 2) {  // RowA | RowB in the ring; the slot pass (which writes RowA) after the last fused kernel that
    // read this buffer — on the slot stream that is an explicit wait, on the batch's own stream the stream order
    e.pipe_split[sr].ensure((size_t)n * 64);
    vec = e.pipe_split[sr].as<float>();
    if (Ss && e.pipe_done_live[sr]) FD_HIP(hipStreamWaitEvent(Ss, e.pipe_done_ev[sr], 0));  // batch i - 4's
  }
  {
    struct SlotPass {  // launch_grouped reads these for this call only
      Engine& e;
      ~SlotPass() { e.slot_pass_stream = nullptr, e.slot_pass_ev = nullptr; }
    } slot_pass{e};
    e.slot_pass_stream = Ss;
    e.slot_pass_ev = Ss ? e.pipe_slot_ev[s] : nullptr;
    if (records)
      fd::launch_features_records(e, records, n, vec, seq, Sf, lean, s, before_buckets, compact);
    else
      fd::launch_features(e, *txns, n, vec, nullptr, seq, nullptr, Sf, lean, s, before_buckets, compact);
  }
  FD_HIP(hipEventRecord(e.pipe_feat_ev[s], Sf));
  e.pipe_feat_live[s] = true;
  // scoring paths other than the fused kernel share engine scratch (per-model columns, tree-split and LSTM
  // buffers): those batches also wait for the previous batch's scoring
  const int pr = (sr + Engine::kDoneRing - 1) % Engine::kDoneRing;  // batch i - 1's done event
  if (e.pipe_done_live[pr] && !compact && !fd::ensemble_applies(e, *params, slots, present, n))
    FD_HIP(hipStreamWaitEvent(Sc, e.pipe_done_ev[pr], 0));
  // this slot's output staging: free once batch i-nbuf's copy to its caller (on e.stream) is done. Routed batches
  // always stage the four columns (the result records are packed from them when the fused kernel does not apply).
  const int n_mp = d_model_probs ? params->n_models : 0;
  const size_t n8 = (size_t)n * 8, a8 = ((size_t)n + 7) & ~(size_t)7;
  // results_in_place (fd_sharded_step: d_results is the engine's own res[q], free by the step's event order, see
  // ShardComm::res): the scoring writes the result records there, no staging copy; otherwise they are staged and
  // copied on the engine stream like the columns (a caller's buffer is written only in the engine stream's order)
  const bool in_place = records && results_in_place;
  const size_t rbytes = records && !in_place ? (size_t)n * sizeof(fd::ResultRecord) : 0;
  e.pipe_out[s].ensure((2 + (size_t)n_mp) * n8 + 2 * a8 + rbytes);
  char* so = e.pipe_out[s].as<char>();
  double* s_fp = reinterpret_cast<double*>(so);
  double* s_conf = (d_confidence || records) ? reinterpret_cast<double*>(so + n8) : nullptr;
  double* s_mp = n_mp ? reinterpret_cast<double*>(so + 2 * n8) : nullptr;
  uint8_t* s_dec = (d_decision || records) ? reinterpret_cast<uint8_t*>(so + (2 + (size_t)n_mp) * n8) : nullptr;
  uint8_t* s_risk = (d_risk || records) ? reinterpret_cast<uint8_t*>(so + (2 + (size_t)n_mp) * n8 + a8) : nullptr;
  auto* s_res = !records ? nullptr
                         : in_place ? static_cast<fd::ResultRecord*>(d_results)
                                    : reinterpret_cast<fd::ResultRecord*>(so + (2 + (size_t)n_mp) * n8 + 2 * a8);
  if (e.pipe_copy_live[s]) FD_HIP(hipStreamWaitEvent(Sc, e.pipe_copy_ev[s], 0));
  ++e.pipe_iter;
  ++e.pipe_iter_total;
  e.pipe_compact_total += compact != 0;
  e.pipe_split_total += compact == 2;
  e.pipe_slot_stream_total += Ss != nullptr;
  {  // the scoring launches go on Sc: score_matrix launches on e.stream
    struct Swap {
      Engine& e;
      hipStream_t saved;
      ~Swap() { e.stream = saved; }
    } swap{e, e.stream};
    e.stream = Sc;
    const auto* rec = static_cast<const fd::RouteRecord*>(records);
    if (!score_matrix(e, *params, slots, ext_probs, present, vec, n, FD_VECTOR_WIDTH, s_mp, s_fp, s_conf, s_dec,
                      s_risk, seq, e.state.S, rec, s_res, compact) &&
        records)
      fd::launch_result_pack(e, s_fp, s_conf, s_dec, s_risk, rec, n, s_res);
  }
  // (split rows: this event also releases ring buffer sr to batch i + 4's slot pass — no event of its own, which
  // cost a record per step on the engine stream; recorded on Sc beside the fused kernel it cost 4 % in round 6)
  FD_HIP(hipEventRecord(e.pipe_done_ev[sr], Sc));
  e.pipe_done_live[sr] = true;
  FD_HIP(hipStreamWaitEvent(e.stream, e.pipe_done_ev[sr], 0));
  if (in_place) {  // nothing to copy: the next use of staging slot s (batch i + 2) is on this batch's stream Sc
    e.pipe_copy_live[s] = false;
    return;
  }
  hipLaunchKernelGGL(pipe_out_copy_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e.stream, s_fp, s_conf,
                     s_dec, s_risk, s_mp, n_mp, n, records ? nullptr : d_fraud_prob, d_confidence, d_decision, d_risk,
                     d_model_probs, reinterpret_cast<const float4*>(vec), reinterpret_cast<float4*>(d_vectors),
                     reinterpret_cast<const uint64_t*>(s_res), static_cast<uint64_t*>(d_results));
  FD_HIP(hipGetLastError());
  FD_HIP(hipEventRecord(e.pipe_copy_ev[s], e.stream));
  e.pipe_copy_live[s] = true;
  e.pipe_copy_vec[s] = d_vectors != nullptr;
}

int fd_score_batch_pipelined(fd_engine* eng, const fd_blend_params* params, const int32_t* slots,
                             const double* const* ext_probs, const uint8_t* present, const fd_txn_batch* txns,
                             int64_t n, float* d_vectors, double* d_model_probs, double* d_fraud_prob,
                             double* d_confidence, uint8_t* d_decision, uint8_t* d_risk, void* input_ready) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E_quiet(eng);
  FD_REQUIRE(params && txns && n >= 0, FD_ERR_INVALID_ARG, "bad arguments");
  if (n == 0) return FD_OK;
  FD_REQUIRE(d_fraud_prob != nullptr, FD_ERR_INVALID_ARG, "null fraud_prob output");
  FD_REQUIRE(params->n_models >= 1 && params->n_models <= FD_MAX_MODELS, FD_ERR_INVALID_ARG, "bad n_models");
  const auto t0 = std::chrono::steady_clock::now();
  pipe_step(e, params, slots, ext_probs, present, txns, nullptr, n, d_vectors, d_model_probs, d_fraud_prob,
            d_confidence, d_decision, d_risk, nullptr, input_ready);
  e.pipe_host_ns += (unsigned long long)std::chrono::duration_cast<std::chrono::nanoseconds>(
                        std::chrono::steady_clock::now() - t0).count();
  FD_API_END
}

int fd_score_records_pipelined(fd_engine* eng, const fd_blend_params* params, const int32_t* slots,
                               const uint8_t* present, const void* d_records, int64_t n, void* d_results,
                               void* input_ready) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E_quiet(eng);
  FD_REQUIRE(params && slots && n >= 0, FD_ERR_INVALID_ARG, "bad arguments");
  FD_REQUIRE(params->n_models >= 1 && params->n_models <= FD_MAX_MODELS, FD_ERR_INVALID_ARG, "bad n_models");
  for (int m = 0; m < params->n_models; ++m)
    FD_REQUIRE(slots[m] >= 0 || (present && !present[m]), FD_ERR_INVALID_ARG,
               "routed scoring needs every present model in a forest slot or FD_SLOT_LSTM");
  if (n == 0) return FD_OK;
  FD_REQUIRE(d_records != nullptr && d_results != nullptr, FD_ERR_INVALID_ARG, "null records / results");
  pipe_step(e, params, slots, nullptr, present, nullptr, d_records, n, nullptr, nullptr, nullptr, nullptr, nullptr,
            nullptr, d_results, input_ready);
  FD_API_END
}

extern "C++" hipStream_t fd::make_stream(int level) {
  hipStream_t st = nullptr;
  if (level == 0) {
    FD_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    return st;
  }
  int least = 0, greatest = 0;
  FD_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
  FD_HIP(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, level > 0 ? greatest : least));
  return st;
}

// ---------------------------------------------------------------- card-hash sharded step over RCCL (comm.hip)
int fd_comm_unique_id(const char* rccl_path, uint8_t* id_out) {
  FD_API_BEGIN
  FD_REQUIRE(id_out, FD_ERR_INVALID_ARG, "null id");
  fd::comm_unique_id(rccl_path, id_out);
  FD_API_END
}

int fd_comm_init(fd_engine* eng, const char* rccl_path, int32_t rank, int32_t world, const uint8_t* id_fwd,
                 const uint8_t* id_back) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E_quiet(eng);
  fd::comm_init(e, rccl_path, rank, world, id_fwd, id_back);
  FD_API_END
}

int fd_comm_destroy(fd_engine* eng) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E_quiet(eng);
  fd::comm_destroy(e);
  FD_API_END
}

int fd_sharded_step(fd_engine* eng, const fd_blend_params* params, const int32_t* slots, const uint8_t* present,
                    const fd_txn_batch* txns, int64_t n, uint64_t batch_id, void* input_ready,
                    const fd_txn_batch* next, int64_t next_n, uint64_t next_id, void* next_ready,
                    double* d_fraud_prob, double* d_confidence, uint8_t* d_decision, uint8_t* d_risk,
                    int64_t* split_sizes) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E_quiet(eng);
  fd::ShardComm& c = e.comm;
  FD_REQUIRE(c.ready, FD_ERR_NOT_LOADED, "no communicators (fd_comm_init)");
  FD_REQUIRE(!c.aborted, FD_ERR_HIP, "communicators aborted (" + c.abort_reason + "): fd_comm_destroy, then fd_comm_init");
  FD_REQUIRE(params && slots && txns && n >= 0 && (!next || next_n >= 0), FD_ERR_INVALID_ARG, "bad arguments");
  FD_REQUIRE(!next || next_id != 0, FD_ERR_INVALID_ARG, "a prefetched batch needs a nonzero next_id");
  FD_REQUIRE(params->n_models >= 1 && params->n_models <= FD_MAX_MODELS, FD_ERR_INVALID_ARG, "bad n_models");
  for (int m = 0; m < params->n_models; ++m)
    FD_REQUIRE(slots[m] >= 0 || (present && !present[m]), FD_ERR_INVALID_ARG,
               "routed scoring needs every present model in a forest slot or FD_SLOT_LSTM");
  FD_REQUIRE(n == 0 || d_fraud_prob, FD_ERR_INVALID_ARG, "null fraud_prob output");
  // the prefetched batch is named by its id: batch_id 0 drops a pending prefetch (on every rank alike: its count
  // exchange completes, its records are never sent); any other id must be the pending one
  const bool use_pending = batch_id != 0;
  if (use_pending)
    FD_REQUIRE(c.pending && batch_id == c.pending_id && n == c.pending_n, FD_ERR_INVALID_ARG,
               "batch " + std::to_string(batch_id) + " (n " + std::to_string(n) + ") is not the prefetched batch " +
                   std::to_string(c.pending_id) + " (n " + std::to_string(c.pending_n) +
                   "): pass its id, or 0 to drop the prefetch");
  const int G = c.world;
  fd::HostLaps L{c};
  c.steps.fetch_add(1, std::memory_order_relaxed);
  // Every communicator operation below is issued by this thread in one fixed order on every rank:
  //   [counts of this batch, when not prefetched] -> {records of this batch + counts of `next`: one group}
  //   (x_fwd, fwd comm) -> results of this batch (engine stream, back comm)
  // 1. this batch's split sizes: exchanged by the previous call (prefetch) or now
  int s;
  if (use_pending) {
    s = c.pending_slot;
  } else {
    s = c.next_slot;
    c.next_slot ^= 1;
    fd::comm_launch_counts(e, *txns, n, static_cast<hipEvent_t>(input_ready), s, L);
  }
  c.pending = false;
  fd::comm_wait_counts(e, s, n, L);  // the step's one host wait (a prefetched batch's counts landed a step ago)
  const int64_t* send = c.split[s];
  const int64_t* recv = c.split[s] + G;
  if (split_sizes)
    for (int p = 0; p < 2 * G; ++p) split_sizes[p] = c.split[s][p];
  int64_t m = 0;
  for (int p = 0; p < G; ++p) m += recv[p];
  // 2. this batch's records to their owners and the next batch's counts, one group on the forward stream (after the
  // owner's previous use of the inbox slot): the counts land while this batch is scored, and the next call's wait
  // is satisfied
  int ns = -1;
  if (next) {
    ns = c.next_slot;
    c.next_slot ^= 1;
    c.pending = true;
    c.pending_id = next_id;
    c.pending_n = next_n;
    c.pending_slot = ns;
  }
  fd::comm_forward_group(e, s, next, next_n, static_cast<hipEvent_t>(next_ready), ns, L);
  // 3. the owner's features + scoring on the pipeline (features wait for the records), results on the engine stream
  const int q = c.inbox_of[s];
  if (m)
    pipe_step(e, params, slots, nullptr, present, nullptr, c.inbox[q].ptr, m, nullptr, nullptr, nullptr, nullptr,
              nullptr, nullptr, c.res[q].ptr, c.in_ev[q], /*results_in_place=*/true);
  L(5);
  // 4. results back (reversed splits) and into arrival order, on the engine stream
  c.back_buf.ensure_headroom((size_t)std::max<int64_t>(n, 1) * sizeof(fd::ResultRecord));
  fd::comm_exchange(e, true, e.stream, c.res[q].ptr, recv, c.back_buf.ptr, send, sizeof(fd::ResultRecord));
  FD_HIP(hipEventRecord(c.inbox_ev[q], e.stream));  // the engine stream has passed this batch's results: inbox q
  c.inbox_live[q] = true;                           // and res[q] are free for batch i + 3
  L(6);
  if (n) fd::launch_result_scatter(e, c.back_buf.ptr, n, d_fraud_prob, d_confidence, d_decision, d_risk);
  L(7);
  FD_API_END
}

int fd_state_load_users_ext_host(fd_engine* eng, const fd_users_ext* users) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(users, FD_ERR_INVALID_ARG, "null users");
  fd::load_users_ext(e, *users);
  FD_API_END
}

int fd_load_merchants_ext_host(fd_engine* eng, const fd_merchants_ext* merchants) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(merchants, FD_ERR_INVALID_ARG, "null merchants");
  FD_HIP(hipStreamSynchronize(e.stream));
  fd::load_merchants_ext(e, *merchants);
  FD_API_END
}

int fd_load_vocab_host(fd_engine* eng, const uint8_t* payment_high_risk, const uint8_t* type_is_refund) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_HIP(hipStreamSynchronize(e.stream));
  fd::load_vocab(e, payment_high_risk, type_is_refund);
  FD_API_END
}

int fd_features_full_device(fd_engine* eng, const fd_txn_batch* txns, const fd_txn_context* ctx, int64_t n,
                            float* d_vectors, double* d_raw, double* d_fmap, fd_rule_scores* d_rules) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(txns, FD_ERR_INVALID_ARG, "null txns");
  const fd_txn_context none{};
  fd::launch_features_full(e, *txns, ctx ? *ctx : none, n, d_vectors, d_raw, d_fmap, d_rules);
  FD_API_END
}

int fd_windows_init(fd_engine* eng, const fd_window_params* params) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(params, FD_ERR_INVALID_ARG, "null params");
  FD_HIP(hipStreamSynchronize(e.stream));
  fd::windows_init(e, *params);
  FD_API_END
}

int fd_windows_step_device(fd_engine* eng, const fd_txn_batch* txns, const fd_window_inputs* in, int64_t n,
                           int flush, fd_user_window* user_out, int64_t user_cap, int64_t* n_user,
                           fd_merchant_window* merchant_out, int64_t merchant_cap, int64_t* n_merchant) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(n_user && n_merchant, FD_ERR_INVALID_ARG, "null result counts");
  const fd_txn_batch none_t{};
  const fd_window_inputs none_in{};
  FD_REQUIRE(txns || n == 0, FD_ERR_INVALID_ARG, "null txns");
  Engine::Timed* tm = e.timing ? e.next_event_pair(FD_TIMING_WINDOWS) : nullptr;
  if (tm) FD_HIP(hipEventRecord(tm->a, e.stream));
  fd::windows_step(e, txns ? *txns : none_t, in ? *in : none_in, n, flush != 0, user_out, user_cap, n_user,
                   merchant_out, merchant_cap, n_merchant);
  if (tm) FD_HIP(hipEventRecord(tm->b, e.stream));
  FD_API_END
}

int fd_windows_step_host(fd_engine* eng, const fd_txn_batch* txns, const fd_window_inputs* in, int64_t n, int flush,
                         fd_user_window* user_out, int64_t user_cap, int64_t* n_user,
                         fd_merchant_window* merchant_out, int64_t merchant_cap, int64_t* n_merchant) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(n_user && n_merchant, FD_ERR_INVALID_ARG, "null result counts");
  FD_REQUIRE(n >= 0 && (txns || n == 0), FD_ERR_INVALID_ARG, "bad batch");
  fd_txn_batch dt{};
  fd_window_inputs di{};
  if (n > 0) {
    FD_REQUIRE(txns->card_key && txns->ts_ms && txns->amount_cents && txns->merchant, FD_ERR_INVALID_ARG,
               "batch needs card_key, ts_ms, amount_cents and merchant");
    const fd_window_inputs none_in{};
    const fd_window_inputs& hi = in ? *in : none_in;
    // staging layout: key | ts | cents | fraud_score (8 B each) | merchant (4 B) | pm | fraud (1 B each)
    const size_t n8 = (size_t)n * 8, n4 = (size_t)n * 4;
    e.windows.stage.ensure(4 * n8 + n4 + 2 * (size_t)n + 64);
    char* d = e.windows.stage.as<char>();
    FD_HIP(hipMemcpyAsync(d, txns->card_key, n8, hipMemcpyHostToDevice, e.stream));
    FD_HIP(hipMemcpyAsync(d + n8, txns->ts_ms, n8, hipMemcpyHostToDevice, e.stream));
    FD_HIP(hipMemcpyAsync(d + 2 * n8, txns->amount_cents, n8, hipMemcpyHostToDevice, e.stream));
    FD_HIP(hipMemcpyAsync(d + 4 * n8, txns->merchant, n4, hipMemcpyHostToDevice, e.stream));
    dt.card_key = reinterpret_cast<const uint64_t*>(d);
    dt.ts_ms = reinterpret_cast<const int64_t*>(d + n8);
    dt.amount_cents = reinterpret_cast<const int64_t*>(d + 2 * n8);
    dt.merchant = reinterpret_cast<const int32_t*>(d + 4 * n8);
    if (hi.fraud_score) {
      FD_HIP(hipMemcpyAsync(d + 3 * n8, hi.fraud_score, n8, hipMemcpyHostToDevice, e.stream));
      di.fraud_score = reinterpret_cast<const double*>(d + 3 * n8);
    }
    if (hi.payment_method) {
      FD_HIP(hipMemcpyAsync(d + 4 * n8 + n4, hi.payment_method, (size_t)n, hipMemcpyHostToDevice, e.stream));
      di.payment_method = reinterpret_cast<const uint8_t*>(d + 4 * n8 + n4);
    }
    if (hi.is_fraud) {
      FD_HIP(hipMemcpyAsync(d + 4 * n8 + n4 + n, hi.is_fraud, (size_t)n, hipMemcpyHostToDevice, e.stream));
      di.is_fraud = reinterpret_cast<const uint8_t*>(d + 4 * n8 + n4 + n);
    }
  }
  fd::windows_step(e, dt, di, n, flush != 0, user_out, user_cap, n_user, merchant_out, merchant_cap, n_merchant);
  FD_API_END
}

int fd_windows_stats(fd_engine* eng, int64_t* watermark, int64_t* user_events, int64_t* merchant_events) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(e.windows.ready, FD_ERR_NOT_LOADED, "windows not initialised (fd_windows_init)");
  if (watermark) *watermark = e.windows.wm;
  if (user_events) *user_events = e.windows.ucount;
  if (merchant_events) *merchant_events = e.windows.mcount;
  FD_API_END
}

int fd_windows_observe(fd_engine* eng, int64_t max_event_ts) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  fd::windows_observe(E(eng), max_event_ts);
  FD_API_END
}

int fd_merchant_windows_merge(const fd_merchant_window* parts, int64_t n, fd_merchant_window* out, int64_t* n_out) {
  FD_API_BEGIN
  fd::merchant_windows_merge(parts, n, out, n_out);
  FD_API_END
}

int fd_sink_init(fd_engine* eng, const fd_sink_params* params) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(params, FD_ERR_INVALID_ARG, "null params");
  FD_HIP(hipStreamSynchronize(e.stream));
  fd::sink_init(e, *params);
  FD_API_END
}

int fd_sink_update_device(fd_engine* eng, const fd_txn_batch* txns, const fd_window_inputs* in, int64_t n) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(txns, FD_ERR_INVALID_ARG, "null batch");
  const fd_window_inputs none{nullptr, nullptr, nullptr};
  fd::sink_update(e, *txns, in ? *in : none, n);
  FD_API_END
}

int fd_sink_update_host(fd_engine* eng, const fd_txn_batch* txns, const fd_window_inputs* in, int64_t n) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(txns && n >= 0, FD_ERR_INVALID_ARG, "bad arguments");
  if (n == 0) return FD_OK;
  FD_REQUIRE(txns->card_key && txns->ts_ms && txns->amount_cents && txns->merchant, FD_ERR_INVALID_ARG,
             "batch needs card_key, ts_ms, amount_cents and merchant");
  const size_t nn = (size_t)n;
  const size_t fo = ((nn * 4 + 15) & ~(size_t)15), so = fo + ((nn + 15) & ~(size_t)15);
  e.stage_in.ensure(nn * 24 + so + nn * 8 + 64);
  char* b = e.stage_in.as<char>();
  FD_HIP(hipMemcpyAsync(b, txns->card_key, nn * 8, hipMemcpyHostToDevice, e.stream));
  FD_HIP(hipMemcpyAsync(b + nn * 8, txns->ts_ms, nn * 8, hipMemcpyHostToDevice, e.stream));
  FD_HIP(hipMemcpyAsync(b + nn * 16, txns->amount_cents, nn * 8, hipMemcpyHostToDevice, e.stream));
  char* x = b + nn * 24;
  FD_HIP(hipMemcpyAsync(x, txns->merchant, nn * 4, hipMemcpyHostToDevice, e.stream));
  fd_window_inputs din{nullptr, nullptr, nullptr};
  if (in && in->is_fraud) {
    FD_HIP(hipMemcpyAsync(x + fo, in->is_fraud, nn, hipMemcpyHostToDevice, e.stream));
    din.is_fraud = reinterpret_cast<const uint8_t*>(x + fo);
  }
  if (in && in->fraud_score) {
    FD_HIP(hipMemcpyAsync(x + so, in->fraud_score, nn * 8, hipMemcpyHostToDevice, e.stream));
    din.fraud_score = reinterpret_cast<const double*>(x + so);
  }
  fd_txn_batch d{};
  d.card_key = reinterpret_cast<const uint64_t*>(b);
  d.ts_ms = reinterpret_cast<const int64_t*>(b + nn * 8);
  d.amount_cents = reinterpret_cast<const int64_t*>(b + nn * 16);
  d.merchant = reinterpret_cast<const int32_t*>(x);
  fd::sink_update(e, d, din, n);
  FD_API_END
}

int fd_sink_query_host(fd_engine* eng, int32_t kind, const int64_t* bucket, const int32_t* merchant, int64_t n,
                       fd_aggregate* out) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::sink_query(e, kind, bucket, merchant, n, out);
  FD_API_END
}

int fd_sink_evict_before(fd_engine* eng, int64_t hour_key, int64_t* kept_entries, int64_t* kept_users) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::sink_evict_before(e, hour_key, kept_entries, kept_users);
  FD_API_END
}

int fd_hash64(const uint8_t* bytes, int64_t n, uint64_t* out) {
  FD_API_BEGIN
  FD_REQUIRE(out && n >= 0 && (n == 0 || bytes), FD_ERR_INVALID_ARG, "bad arguments");
  *out = fd::hash_bytes(bytes, n);
  FD_API_END
}

int fd_ingest_set_vocab(fd_engine* eng, int32_t which, const uint8_t* bytes, const int64_t* offsets, int64_t n) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::ingest_set_vocab(e, which, bytes, offsets, n);
  FD_API_END
}

int fd_ingest_set_merchants(fd_engine* eng, const uint8_t* bytes, const int64_t* offsets, int64_t n) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::ingest_set_merchants(e, bytes, offsets, n);
  FD_API_END
}

int fd_ingest_json_device(fd_engine* eng, const uint8_t* d_bytes, const int64_t* d_offsets, int64_t n,
                          const fd_ingest_out* d_out) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(d_out, FD_ERR_INVALID_ARG, "null outputs");
  fd::launch_ingest(e, d_bytes, d_offsets, n, *d_out);
  FD_API_END
}

int fd_ingest_json_host(fd_engine* eng, const uint8_t* bytes, const int64_t* offsets, int64_t n,
                        const fd_ingest_out* out) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(out && offsets && n >= 0, FD_ERR_INVALID_ARG, "bad arguments");
  if (n == 0) return FD_OK;
  FD_REQUIRE(offsets[0] == 0 && offsets[n] >= 0, FD_ERR_INVALID_ARG, "offsets must start at 0");
  const size_t nb = (size_t)offsets[n];
  fd::IngestTables& t = e.ingest;
  t.stage_bytes.ensure(std::max<size_t>(nb, 16));
  t.stage_offsets.ensure((size_t)(n + 1) * 8);
  if (nb) FD_HIP(hipMemcpyAsync(t.stage_bytes.ptr, bytes, nb, hipMemcpyHostToDevice, e.stream));
  FD_HIP(hipMemcpyAsync(t.stage_offsets.ptr, offsets, (size_t)(n + 1) * 8, hipMemcpyHostToDevice, e.stream));
  // device columns: one staging block, 8-byte columns first
  struct Col { void* host; size_t w; };
  const Col cols[] = {{out->card_key, 8}, {out->ts_ms, 8}, {out->amount_cents, 8}, {out->device_fp, 8},
                      {out->geo_lat, 8}, {out->geo_lon, 8}, {out->merchant_lat, 8}, {out->merchant_lon, 8},
                      {out->fraud_score, 8}, {out->txn_hash, 8}, {out->merchant, 4}, {out->ip_class, 1},
                      {out->hour, 1}, {out->weekend, 1}, {out->payment_method, 1}, {out->transaction_type, 1},
                      {out->card_type, 1}, {out->user_agent_flag, 1}, {out->is_fraud, 1}, {out->status, 1}};
  constexpr int NC = sizeof(cols) / sizeof(cols[0]);
  size_t offs[NC], total = 0;
  for (int c = 0; c < NC; ++c) {
    offs[c] = total;
    if (cols[c].host) total += ((size_t)n * cols[c].w + 15) & ~(size_t)15;
  }
  t.stage_out.ensure(std::max<size_t>(total, 16));
  char* base = t.stage_out.as<char>();
  auto dev = [&](int c) -> void* { return cols[c].host ? base + offs[c] : nullptr; };
  fd_ingest_out d{};
  d.card_key = (uint64_t*)dev(0);
  d.ts_ms = (int64_t*)dev(1);
  d.amount_cents = (int64_t*)dev(2);
  d.device_fp = (uint64_t*)dev(3);
  d.geo_lat = (double*)dev(4);
  d.geo_lon = (double*)dev(5);
  d.merchant_lat = (double*)dev(6);
  d.merchant_lon = (double*)dev(7);
  d.fraud_score = (double*)dev(8);
  d.txn_hash = (uint64_t*)dev(9);
  d.merchant = (int32_t*)dev(10);
  d.ip_class = (uint8_t*)dev(11);
  d.hour = (uint8_t*)dev(12);
  d.weekend = (uint8_t*)dev(13);
  d.payment_method = (uint8_t*)dev(14);
  d.transaction_type = (uint8_t*)dev(15);
  d.card_type = (uint8_t*)dev(16);
  d.user_agent_flag = (uint8_t*)dev(17);
  d.is_fraud = (uint8_t*)dev(18);
  d.status = (uint8_t*)dev(19);
  fd::launch_ingest(e, t.stage_bytes.as<const uint8_t>(), t.stage_offsets.as<const int64_t>(), n, d);
  for (int c = 0; c < NC; ++c)
    if (cols[c].host)
      FD_HIP(hipMemcpyAsync(cols[c].host, base + offs[c], (size_t)n * cols[c].w, hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  FD_API_END
}

int fd_ingest_scalar_host(int32_t kind, const uint8_t* text, int32_t n, double* f64_out, int64_t* i64_out,
                          int32_t* flags_out) {
  FD_API_BEGIN
  FD_REQUIRE(text && n >= 0 && flags_out, FD_ERR_INVALID_ARG, "bad arguments");
  *flags_out = 0;
  if (kind == 0 || kind == 1) {
    fd::Decimal d;
    const int end = fd::scan_number(text, 0, n, d);
    if (end != n) {
      *flags_out = 1;
      return FD_OK;
    }
    if (kind == 0) {
      bool amb = false;
      const double v = fd::decimal_to_double(d.w, d.q, d.neg, d.many, &amb);
      if (f64_out) *f64_out = v;
      if (amb) *flags_out |= 2;
    } else {
      bool inexact = false;
      int64_t c = 0;
      if (!fd::decimal_to_cents(d, &c, &inexact)) *flags_out |= 1;
      if (inexact) *flags_out |= 2;
      if (i64_out) *i64_out = c;
    }
  } else if (kind == 2) {
    int64_t ms = 0;
    if (!fd::parse_iso_instant(text, 0, n, &ms)) *flags_out = 1;
    if (i64_out) *i64_out = ms;
  } else {
    throw fd::Error(FD_ERR_INVALID_ARG, "unknown scalar kind");
  }
  FD_API_END
}

int fd_state_snapshot(fd_engine* eng, const char* path, int32_t shard, int32_t n_shards, int64_t* bytes_written) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::features_check(e);
  fd::state_snapshot(e, path, shard, n_shards, bytes_written);
  FD_API_END
}

int fd_state_restore(fd_engine* eng, const char* path, int32_t shard, int32_t n_shards, int32_t flags,
                     int64_t* cards_restored) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::features_check(e);
  fd::state_restore(e, path, shard, n_shards, flags, cards_restored);
  FD_API_END
}

int fd_load_lstm(fd_engine* eng, const fd_lstm_params* params) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(params, FD_ERR_INVALID_ARG, "null params");
  FD_HIP(hipStreamSynchronize(e.stream));
  if (e.aux_stream) FD_HIP(hipStreamSynchronize(e.aux_stream));
  fd::load_lstm(e, *params);
  FD_API_END
}

int fd_unload_lstm(fd_engine* eng) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_HIP(hipStreamSynchronize(e.stream));
  if (e.aux_stream) FD_HIP(hipStreamSynchronize(e.aux_stream));
  for (auto* b : {&e.lstm.wpk, &e.lstm.wpk4, &e.lstm.bias, &e.lstm.wout, &e.lstm.bout}) b->release();
  e.lstm.loaded = false;
  FD_API_END
}

int fd_lstm_predict_device(fd_engine* eng, const float* d_seq, int64_t n, int32_t T, double* d_prob) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::launch_lstm(e, e.stream, d_seq, n, T, d_prob);
  FD_API_END
}

int fd_lstm_predict_host(fd_engine* eng, const float* seq, int64_t n, int32_t T, double* prob) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(n >= 0 && T >= 1 && T <= FD_MAX_SEQ_LEN, FD_ERR_INVALID_ARG, "bad arguments");
  if (n == 0) return FD_OK;
  FD_REQUIRE(seq && prob, FD_ERR_INVALID_ARG, "null sequence / output");
  const size_t sb = (size_t)n * T * fd::kSeqInput * sizeof(float);
  e.stage_in.ensure(sb);
  e.stage_out0.ensure((size_t)n * sizeof(double));
  FD_HIP(hipMemcpyAsync(e.stage_in.ptr, seq, sb, hipMemcpyHostToDevice, e.stream));
  fd::launch_lstm(e, e.stream, e.stage_in.as<float>(), n, T, e.stage_out0.as<double>());
  FD_HIP(hipMemcpyAsync(prob, e.stage_out0.ptr, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  FD_API_END
}

int fd_features_seq_device(fd_engine* eng, const fd_txn_batch* txns, int64_t n, float* d_vectors, double* d_raw,
                           float* d_seq) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(txns, FD_ERR_INVALID_ARG, "null txns");
  fd::launch_features(e, *txns, n, d_vectors, d_raw, d_seq);
  FD_API_END
}

int fd_shard_of_host(const uint64_t* keys, int64_t n, int32_t n_shards, int32_t* out) {
  FD_API_BEGIN
  FD_REQUIRE(n >= 0 && (n == 0 || (keys && out)), FD_ERR_INVALID_ARG, "bad arguments");
  FD_REQUIRE(n_shards >= 1 && n_shards <= FD_MAX_SHARDS, FD_ERR_INVALID_ARG, "n_shards must be in [1, 64]");
  for (int64_t i = 0; i < n; ++i) out[i] = (int32_t)fd::shard_of_host(keys[i], (unsigned)n_shards);
  FD_API_END
}

int fd_route_partition_device(fd_engine* eng, const fd_txn_batch* txns, int64_t n, int32_t n_shards,
                              void* d_records, int64_t* d_counts) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(txns, FD_ERR_INVALID_ARG, "null txns");
  fd::launch_route_partition(e, *txns, nullptr, n, n_shards, d_records, d_counts);
  FD_API_END
}

int fd_route_partition_ex_device(fd_engine* eng, const fd_txn_batch* txns, const fd_window_inputs* extra, int64_t n,
                                 int32_t n_shards, void* d_records, int64_t* d_counts) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(txns, FD_ERR_INVALID_ARG, "null txns");
  fd::launch_route_partition(e, *txns, extra, n, n_shards, d_records, d_counts);
  FD_API_END
}

int fd_route_partition_stream(fd_engine* eng, const fd_txn_batch* txns, const fd_window_inputs* extra, int64_t n,
                              int32_t n_shards, void* d_records, int64_t* d_counts, void* stream) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E_quiet(eng);  // touches no card state: the pipelined stream stays undisturbed
  FD_REQUIRE(txns, FD_ERR_INVALID_ARG, "null txns");
  fd::launch_route_partition(e, *txns, extra, n, n_shards, d_records, d_counts, static_cast<hipStream_t>(stream),
                             &e.route_blk_stream);
  FD_API_END
}

int fd_route_unpack_device(fd_engine* eng, const void* d_records, const void* d_results, int64_t n,
                           const fd_txn_batch* out, uint8_t* d_payment_method, uint8_t* d_is_fraud,
                           double* d_fraud_score) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(out, FD_ERR_INVALID_ARG, "null output columns");
  fd::launch_route_unpack(e, d_records, d_results, n, *out, d_payment_method, d_is_fraud, d_fraud_score);
  FD_API_END
}

int fd_score_records_device(fd_engine* eng, const fd_blend_params* params, const int32_t* slots,
                            const uint8_t* present, const void* d_records, int64_t n, void* d_results) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(params && slots && n >= 0, FD_ERR_INVALID_ARG, "bad arguments");
  for (int m = 0; m < params->n_models && m < FD_MAX_MODELS; ++m)
    FD_REQUIRE(slots[m] >= 0 || (present && !present[m]), FD_ERR_INVALID_ARG,
               "routed scoring needs every present model in a forest slot or FD_SLOT_LSTM");
  if (n == 0) return FD_OK;
  e.feat_vec.ensure((size_t)n * FD_VECTOR_WIDTH * 4);
  e.route_out.ensure((size_t)n * (2 * sizeof(double) + 2));
  double* fp = e.route_out.as<double>();
  double* conf = fp + n;
  uint8_t* dec = reinterpret_cast<uint8_t*>(conf + n);
  uint8_t* risk = dec + n;
  float* sq = lstm_seq_buffer(e, *params, slots, present, n);
  fd::launch_features_records(e, d_records, n, e.feat_vec.as<float>(), sq);  // reads the records in place
  const auto* rec = static_cast<const fd::RouteRecord*>(d_records);
  if (!score_matrix(e, *params, slots, nullptr, present, e.feat_vec.as<float>(), n, FD_VECTOR_WIDTH, nullptr, fp,
                    conf, dec, risk, sq, e.state.S, rec, static_cast<fd::ResultRecord*>(d_results)))
    fd::launch_result_pack(e, fp, conf, dec, risk, rec, n, d_results);
  FD_API_END
}

int fd_route_scatter_results_device(fd_engine* eng, const void* d_results, int64_t n, double* d_fraud_prob,
                                    double* d_confidence, uint8_t* d_decision, uint8_t* d_risk) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  fd::launch_result_scatter(e, d_results, n, d_fraud_prob, d_confidence, d_decision, d_risk);
  FD_API_END
}

int fd_blend_device(fd_engine* eng, const fd_blend_params* params, int64_t n, const double* const* d_probs,
                    const uint8_t* present, double* d_fraud_prob, double* d_confidence, uint8_t* d_decision,
                    uint8_t* d_risk) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(params, FD_ERR_INVALID_ARG, "null params");
  fd::launch_blend(e, *params, n, d_probs, present, d_fraud_prob, d_confidence, d_decision, d_risk);
  FD_API_END
}

int fd_blend_host(fd_engine* eng, const fd_blend_params* params, int64_t n, const double* const* probs,
                  const uint8_t* present, double* fraud_prob, double* confidence, uint8_t* decision,
                  uint8_t* risk) {
  FD_API_BEGIN
  FD_ENGINE_LOCK(eng);
  Engine& e = E(eng);
  FD_REQUIRE(params && probs && fraud_prob, FD_ERR_INVALID_ARG, "bad arguments");
  FD_REQUIRE(params->n_models >= 0 && params->n_models <= FD_MAX_MODELS, FD_ERR_INVALID_ARG,
             "n_models out of range");
  if (n == 0) return FD_OK;
  const int M = params->n_models;
  // stage_in holds the M probability columns; outputs in stage_out0..3
  e.stage_in.ensure((size_t)n * sizeof(double) * (M > 0 ? M : 1));
  e.stage_out0.ensure((size_t)n * sizeof(double));
  e.stage_out1.ensure((size_t)n * sizeof(double));
  e.stage_out2.ensure((size_t)n);
  e.stage_out3.ensure((size_t)n);
  const double* dcols[FD_MAX_MODELS] = {};
  for (int m = 0; m < M; ++m) {
    double* col = e.stage_in.as<double>() + (size_t)m * n;
    dcols[m] = col;
    if (present && !present[m]) continue;
    FD_REQUIRE(probs[m], FD_ERR_INVALID_ARG, "null probability column");
    FD_HIP(hipMemcpyAsync(col, probs[m], (size_t)n * sizeof(double), hipMemcpyHostToDevice, e.stream));
  }
  fd::launch_blend(e, *params, n, dcols, present, e.stage_out0.as<double>(), e.stage_out1.as<double>(),
                   e.stage_out2.as<uint8_t>(), e.stage_out3.as<uint8_t>());
  FD_HIP(hipMemcpyAsync(fraud_prob, e.stage_out0.ptr, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, e.stream));
  if (confidence)
    FD_HIP(hipMemcpyAsync(confidence, e.stage_out1.ptr, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, e.stream));
  if (decision) FD_HIP(hipMemcpyAsync(decision, e.stage_out2.ptr, (size_t)n, hipMemcpyDeviceToHost, e.stream));
  if (risk) FD_HIP(hipMemcpyAsync(risk, e.stage_out3.ptr, (size_t)n, hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  FD_API_END
}

}  // extern "C"
