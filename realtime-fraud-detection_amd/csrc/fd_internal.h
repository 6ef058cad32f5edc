// fd_internal.h — engine internals shared by the HIP translation units of libfdengine.so.
// Not part of the ABI (see include/fdengine.h).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "fdengine.h"

namespace fd {

constexpr int kMaxSlots = 8;      // forest slots per engine
constexpr int kTile = 256;        // transactions per workgroup in the forest kernel (one per thread)
constexpr int kGatherBatchMax = 4096;  // largest batch the gather bucket kernel takes (features.hip kChunkCap)
constexpr int kMaxFeatures = 64;  // model columns held in LDS ([feature][kTile] f32 = 64 KiB max)
// The compact scoring vector of the fused pipeline (features.hip write_vector -> ensemble.hip prologue): of the 64
// slots of the engine's vector (FeatureProcessor's 41 definitions + derived features + pad, _prepare_features) only
// these 22 vary per transaction; slots 12, 24, 25, 33, 34 are always 0.5 (defaults with no bridged source) and the
// rest 0. The pipelined stream writes a 64-B row per transaction instead of 64 floats (256 B) when nothing else reads
// the vectors, and the ensemble kernel expands it: the 14 slots with arbitrary values as f32 in words
// 0..13 (compact-index order), the 8 that are always small integers — hour, day of week, weekend, the 1 h / 24 h /
// 5 min counts, the account age (each clip10 of an integer), the new-device flag — as bytes 56..63.
constexpr int kCompactWidth = 16;  // row stride in 4-B words
constexpr int kCompactSlots = 22;
constexpr int kCompactSlot[kCompactSlots] = {0, 1, 5, 6, 7, 14, 15, 16, 17, 19, 21, 23,
                                             26, 27, 31, 32, 41, 42, 43, 44, 45, 46};
constexpr int kIntSlots = 8;
constexpr int kIntCompact[kIntSlots] = {2, 3, 4, 5, 6, 9, 12, 15};  // compact indices (features 5 6 7 14 15 19 26 32)
// the byte (0..7) of a small-integer compact slot, -1 for the others
__host__ __device__ constexpr int int_slot(int ci) {
  for (int k = 0; k < kIntSlots; ++k)
    if (kIntCompact[k] == ci) return k;
  return -1;
}
// the f32 word (0..13) of a compact slot with arbitrary values, -1 for the small-integer ones
__host__ __device__ constexpr int compact_word(int ci) {
  if (int_slot(ci) >= 0) return -1;
  int w = 0;
  for (int k = 0; k < ci; ++k) w += int_slot(k) < 0 ? 1 : 0;
  return w;
}
static_assert(compact_word(kCompactSlots - 1) == kCompactSlots - kIntSlots - 1 && kCompactSlots - kIntSlots <= 14,
              "14 f32 words, then the 8 bytes");
// the slot's place in the compact row, -2 for the constant 0.5, -1 for the constant 0
__host__ __device__ constexpr int compact_src(int f) {
  for (int k = 0; k < kCompactSlots; ++k)
    if (kCompactSlot[k] == f) return k;
  return (f == 12 || f == 24 || f == 25 || f == 33 || f == 34) ? -2 : -1;
}
constexpr int kMaxDepth = 10;     // deepest tree the repacker accepts
constexpr size_t kLdsBudget = 160 * 1024;  // LDS per CU (one workgroup per CU at 64k batches)
constexpr int kMaxBins = 65534;   // distinct thresholds per feature in the binned layout
constexpr int kSplitTiles = 128;  // below this many 256-txn tiles the forest runs the tree-split path
constexpr int kSeqInput = 16;     // LSTM per-event input width (the bridged raw features)
constexpr unsigned long long kSeqMaterialized = 1ull << 63;  // sequence descriptor: row i of the sequence buffer
constexpr int kLstmHidden = 128;  // lstm_sequential hidden_units (ml/utils/config.py:152-156)

#ifdef FD_FOREST_PROFILE
// Latency-path timeline (profiling build only; tools/c5_phases.py): per (kernel id, linear workgroup < 1024)
// {start, mark 1, mark 2, end} of thread 0 in the GPU-wide 100 MHz clock. Each translation unit keeps its own buffer
// (FD_TL_BUF) and exports it (fd_debug_tl_<unit>); the last launch of each kernel id wins.
constexpr int kTlKernels = 8;
#define FD_TL_BUF(name) __device__ unsigned long long name[fd::kTlKernels * 1024 * 4]
#define FD_TL(buf, kid, k)                                                                            \
  do {                                                                                                \
    const unsigned tl_b = blockIdx.x + blockIdx.y * gridDim.x;                                        \
    if (threadIdx.x == 0 && tl_b < 1024u) buf[((kid) * 1024 + tl_b) * 4 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define FD_TL(buf, kid, k) \
  do {                     \
  } while (0)
#endif

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_error(const std::string& msg);

#define FD_HIP(call)                                                                       \
  do {                                                                                     \
    hipError_t _e = (call);                                                                \
    if (_e != hipSuccess)                                                                  \
      throw ::fd::Error(FD_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(_e));    \
  } while (0)

#define FD_REQUIRE(cond, code, msg)              \
  do {                                           \
    if (!(cond)) throw ::fd::Error((code), (msg)); \
  } while (0)

// Device allocation owned by the engine; grows, never shrinks.

struct DeviceBuffer {
  void* ptr = nullptr;
  size_t bytes = 0;
  void ensure(size_t need) {
    if (need <= bytes) return;
    release();
    FD_HIP(hipMalloc(&ptr, need));
    bytes = need;
  }
  // grow by a quarter more than asked: buffers sized per batch by a count that wanders (a shard's inbox) then
  // reallocate O(log) times instead of at every new maximum (hipFree waits for the device)
  void ensure_headroom(size_t need) {
    if (need > bytes) ensure(need + need / 4);
  }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(ptr); }
};

// small-batch tree-split scratch of one forest (forest.hip launch_split)
struct SplitScratch {
  DeviceBuffer bins, nan, leaves;  // nan: per-tile "holds a NaN" flags, cleared by the step's sum kernel
};

// Latency batches, option "latency_prebin": the tree-split binning of the XGBoost / IsolationForest pair done by
// workgroups of the LSTM head's launch, ahead of its own (lstm.hip lstm_kernel4), so the pair's binning launch and its
// queue gap go (forest.hip launch_forest_pair_blend). Filled by forest_pair_prebin before the LSTM launch (score_matrix);
// `done` set by the LSTM launch that binned (these vectors), consumed by the pair launch.
struct PreBin {
  const float* thr[2] = {};        // [0] XGBoost, [1] IsolationForest: distinct thresholds, feature-major
  const int32_t* thr_off[2] = {};
  uint32_t* bins[2] = {};          // [feature][n_pad]
  uint32_t* nan[2] = {};           // per-tile NaN flags
  int nf[2] = {};
  int64_t n = 0, n_pad = 0;
  int ld = 0;
  int steps[2] = {};               // each forest's largest lifting step (PackedForest::bin_steps)
  bool thr_nonempty = false;       // both tables hold a threshold (the inline searches read clamped positions)
  const void* fx = nullptr;        // the forests and the vectors the bins are for
  const void* ff = nullptr;
  const float* X = nullptr;
  bool want = false, done = false;
};

// A forest repacked into perfect depth-D trees stored as 1-based heaps (see forest.hip header and
// DESIGN.md "Forest layout"): per tree 2^D node records {f32 thr, u32 meta} (slot 0 unused; children
// of slot s are 2s / 2s+1) then 2^D leaf values (f32 XGBoost, f64 Isolation Forest); chunks of
// `chunk` trees, each `chunk_stride` bytes (1 KiB multiple, LDS-DMA staging).
//   meta = feature * kTile * 4 (byte offset of the feature row in the LDS tile) | default_left << 31.
struct PackedForest {
  bool loaded = false;
  int kind = 0;
  int n_trees = 0;
  int n_chunks = 0;
  int chunk = 0;
  int depth = 0;
  int num_feature = 0;
  size_t tree_bytes = 0;
  size_t chunk_stride = 0;
  float base_margin = 0.f;  // XGB: -logf(1/base_score - 1)
  double if_offset = 0.0;
  double if_denominator = 0.0;
  DeviceBuffer blob;      // n_chunks * chunk_stride
  DeviceBuffer leaf_ids;  // n_trees_padded * 2^D original node ids (parity output)
  // binned layout (forest_kernel4), present when every feature has <= 65534 distinct thresholds
  bool binned = false;
  int b_chunk = 0, b_n_chunks = 0, bin_steps = 0;
  size_t b_tree_bytes = 0, b_chunk_stride = 0;
  DeviceBuffer b_blob;     // b_n_chunks * b_chunk_stride
  DeviceBuffer b_thr;      // distinct thresholds, feature-major ascending (f32)
  DeviceBuffer b_thr_off;  // num_feature + 1 offsets (int32)
  int b_n_thr = 0;         // distinct thresholds in b_thr
  // node-only chunks of the binned layout (forest_kernel6): CH trees' node words per chunk, leaf
  // values in a separate [tree][2^D] array read from global memory
  int n_chunk = 0, n_n_chunks = 0;
  size_t n_chunk_stride = 0;
  DeviceBuffer n_blob;    // n_n_chunks * n_chunk_stride
  DeviceBuffer n_leaves;  // n_n_chunks * n_chunk * 2^D leaf values (f32 XGBoost / f64 IsolationForest)
  mutable SplitScratch split;
  // the model as loaded (host copy): the fused ensemble kernel repacks it jointly with the other forest
  uint64_t gen = 0;  // changes on every load / unload (ensemble plan cache key)
  fd_forest_params params{};
  std::vector<int64_t> t_off;
  std::vector<int32_t> t_left, t_right, t_feature;
  std::vector<double> t_threshold, t_leaf;
  std::vector<uint8_t> t_dleft;
};

// The fused ensemble kernel's joint repack of one XGBoost and/or one IsolationForest (ensemble.hip): both
// padded to one depth D, node words rewritten against the MERGED per-feature threshold tables, so one bin
// tile serves both forests; chunks of CH[k] node-only trees, leaf values [tree][2^D] per forest.
// binning passes of one row form (ensemble.hip): pass p covers features [f[p], f[p + 1]); bit p of glob: searched in
// global memory (a table larger than the staging area); img_off[p] .. img_off[p + 1]: pass p's padded LDS image
struct EnsPassSet {
  std::vector<int> f, img_off;
  unsigned long long glob = 0;
};

struct EnsemblePlan {
  bool valid = false;
  bool wide = true;  // chunk layout: 24 / 16 trees (wide) or 20 / 12 (compact: LDS room for an RCCL kernel beside)
  int slot[2] = {-1, -1};   // forest A = the XGBoost model (or the only forest), forest B = the IsolationForest
  uint64_t gen[2] = {0, 0};
  int n_forests = 0, D = 0, nf = 0;
  int kind[2] = {0, 0}, n_trees[2] = {0, 0}, CH[2] = {0, 0}, n_chunks[2] = {0, 0};
  size_t stride[2] = {0, 0};
  float base_margin = 0.f;
  double if_offset = 0.0, if_denominator = 0.0;
  DeviceBuffer nodes[2], thr;  // per forest: chunk blobs (node blocks + leaf values); merged threshold tables
  std::vector<int32_t> h_thr_off;  // merged table offsets (host copy: binning pass plan)
  std::vector<uint16_t> h_cbin;    // bins of the compact vector's constant slots (ensemble.hip)
  std::vector<uint16_t> h_lut;     // bins of the small-integer compact slots' values 0..31 (ensemble.hip kIntCompact)
  DeviceBuffer img;    // every staged binning pass's padded table image (ensemble.hip plan_passes), LDS-DMA source
  EnsPassSet passes;
  int max_feature_thr = 0;
};

// card-hash routing records (route.hip): one transaction (48 B) / one result (24 B)
struct __attribute__((aligned(16))) RouteRecord {
  unsigned long long key;
  long long ts;
  long long cents;
  unsigned long long dfp;
  int merchant;
  unsigned seq;  // index in the ingest rank's micro-batch
  unsigned char ipc, hour, wk;
  unsigned char pm;  // payment-method code for the owner's windows (255 = null)
  unsigned flags;    // bit 0: Transaction.isFraud (owner's windows / sink)
};
struct __attribute__((aligned(8))) ResultRecord {
  double fraud_prob;
  double confidence;
  unsigned seq;
  unsigned char decision, risk;
  unsigned short pad;
};

// LSTM head (lstm.hip): B operands packed per wave/gate/k-step/lane, summed biases, dense head
struct LstmModel {
  bool loaded = false;
  int input_size = 0, n_out = 0;
  DeviceBuffer wpk, wpk4, bias, wout, bout;  // wpk: 16-row kernel's B operands; wpk4: the 4-row kernel's
  bool hh_finite = false;  // every W_hh weight finite: W_hh h_{-1} = W_hh 0 adds only zeros (lstm_kernel4 skips it)
};

// One card's keyed state header (features.hip): 128 B = one L2 line, so a transaction's state read touches one
// line. Bytes 0-63 hold everything a transaction rewrites (last time, ring cursor, window counts / sums / oldest
// times, the redis_compat session, the LSTM history cursor in flags), bytes 64-127 what only an insert or a profile
// load writes (key, profile, device fingerprints): a transaction's write-back dirties half the line (round 5; the
// oldest times are stored as 32-bit offsets below last_ts to fit — exact, a window spans < 2^32 ms).
struct __attribute__((aligned(128))) CardHeader {
  long long last_ts;               // time of the card's last event (sliding: last appended; redis: last write)
  unsigned char ring_n, ring_head; // sliding: events held (<= K), next write position
  unsigned char unsorted;          // sliding: appends left before the ring is time-sorted again (0 = sorted)
  unsigned char pad0;
  unsigned char wc[3], pad1;       // sliding: events of the ring's newest suffix inside the 5m / 1h / 24h window
  unsigned flags;                  // bit 0 user profile; bit 1 redis session live; bits 8-15 LSTM events held;
                                   // bits 16-23 LSTM history write position
  int rc_cnt;                      // redis_compat: session count
  long long ws[3];                 // sliding: window sums (cents); redis_compat: ws[0] is the session amount
  unsigned wod[3];                 // sliding: last_ts - time of the oldest in-window event (valid when wc > 0)
  unsigned pad2;
  unsigned long long key;          // 0 = empty slot
  double avg;                      // profile: avg_transaction_amount (NaN = null)
  int age;                         // profile: account_age_days
  int pad3;
  unsigned long long fp[3];        // profile: device fingerprints (0 = none)
  long long pad4[2];
};
static_assert(sizeof(CardHeader) == 128, "CardHeader must be one 128-B line");
static_assert(offsetof(CardHeader, key) == 64 && offsetof(CardHeader, wod) + sizeof(unsigned) * 3 <= 64,
              "the mutable fields in bytes 0-63, the key at 64 (snapshot.hip reads it there)");
constexpr int kCardHeaderBytes = (int)sizeof(CardHeader);

// one event of a card's ring (sliding windows): time and cents
struct __attribute__((aligned(16))) RingEvent {
  long long ts;
  long long cents;
};

// The card table's state pages: slot s owns bytes [s * stride, (s + 1) * stride) of one allocation — its
// 128-B header, then (sliding mode) its K ring events of 16 B. A transaction's state (header and the ring
// entries it evicts / appends) lies in one contiguous page: one address translation per card instead of one
// per array (round 4; before, headers and rings were two arrays of their own).
struct CardPages {
  char* base;
  long long stride;  // bytes per slot: 128 + 16 K (sliding), 128 (redis_compat)
  __host__ __device__ __forceinline__ CardHeader* hdr(long long s) const {
    return reinterpret_cast<CardHeader*>(base + s * stride);
  }
  __host__ __device__ __forceinline__ RingEvent* ring(long long s) const {
    return reinterpret_cast<RingEvent*>(base + s * stride + kCardHeaderBytes);
  }
};

#ifdef __HIP_DEVICE_COMPILE__
#define FD_CARD_SLOT_QUAL __device__ __forceinline__
#else
#define FD_CARD_SLOT_QUAL __device__ inline
#endif
// Card-table probe (murmur3 fmix64 home slot, linear probing) over the compact key array `keys` (8 B per slot,
// CardStore::keys): the probes' random accesses stay inside 8 x capacity bytes, a range the GPU's TLBs reach,
// instead of the 128-B headers. The probe sequence is read as aligned groups of 8 keys (64 B, four 16-B loads in
// flight): at the bench's load factor (~0.75, where a linear probe runs ~2.5 slots on a hit and ~8 on a miss) one
// dependent load round instead of one per slot. A key seen as 0 is claimed by CAS, whose result also corrects a
// stale read (another CU's insert): it returns the key that is there. An insert mirrors the key into the slot's
// header (snapshots and occupancy read it there). Returns the slot, -1 when the table is full.
FD_CARD_SLOT_QUAL long long card_slot(unsigned long long* keys, CardPages pg, long long mask, unsigned long long key) {
  if (key == 0ull) key = 1ull;  // 0 marks an empty slot
  unsigned long long m = key;
  m ^= m >> 33;
  m *= 0xff51afd7ed558ccdULL;
  m ^= m >> 33;
  m *= 0xc4ceb9fe1a85ec53ULL;
  m ^= m >> 33;
  long long h = (long long)(m & (unsigned long long)mask);
  if (mask >= 7) {
    long long g = h & ~7ll;
    int j0 = (int)(h & 7);
    for (long long p = 0; p <= mask + 8; p += 8) {  // the first group twice: its slots before j0 come last
      const uint4* q = reinterpret_cast<const uint4*>(keys + g);
      uint4 w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) w[u] = q[u];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (j < j0) continue;
        const uint4 v = w[j >> 1];
        const unsigned long long k = (j & 1) ? (((unsigned long long)v.w << 32) | v.z)
                                             : (((unsigned long long)v.y << 32) | v.x);
        if (k == key) return g + j;
        if (k == 0ull) {
          const unsigned long long old = atomicCAS(&keys[g + j], 0ull, key);
          if (old == 0ull) {
            pg.hdr(g + j)->key = key;
            return g + j;
          }
          if (old == key) return g + j;
        }
      }
      j0 = 0;
      g = (g + 8) & mask;
    }
    return -1;
  }
  for (long long p = 0; p <= mask; ++p) {
    const unsigned long long k = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == key) return h;
    if (k == 0ull) {
      const unsigned long long old = atomicCAS(&keys[h], 0ull, key);
      if (old == 0ull) {
        pg.hdr(h)->key = key;
        return h;
      }
      if (old == key) return h;
    }
    h = (h + 1) & mask;
  }
  return -1;
}

// HBM-resident keyed card state (features.hip)
struct CardStore {
  bool ready = false;
  int64_t cap = 0;   // slots (power of two)
  int mode = 0;      // fd_window_mode
  int K = 1;         // ring events per card (sliding)
  int S = 0;         // LSTM history events per card (0 = off)
  int bucket_keys = 0;  // option "bucket_keys": transactions per bucket workgroup (0 auto, features.hip)
  bool bucket_spread = true;  // option "bucket_spread": a bucket's card segments dealt over all 4 waves
  // option "slot_gather": batches of <= 4096 transactions outside the pipelined stream find their card slots inside
  // the bucket kernel (each bucket workgroup takes the keys that hash to it), no slot launch (features.hip)
  bool slot_gather = true;
  // option "lean_group": how the lean bucket kernel groups a bucket's keys by card — 0 rank sort, 1 rank sort split
  // over every thread (rank_sort_split), 2 (default) LDS hash table (no sort)
  int lean_group = 2;
  bool slot_prio = false;  // option "slot_prio": the pipelined stream's slot kernel issues at priority 2
  bool feat_prio = false;  // option "feature_prio": the pipelined stream's lean bucket kernel issues at priority 2 (the
                           // default in round 5; off since round 6's split rows, engine.hip)
  int64_t n_merchants = 0;
  DeviceBuffer pages, keys, merchants, err, seq;  // pages: CardPages (header + ring per slot); keys: the compact
                                                  // key array card_slot probes
  long long page_bytes = kCardHeaderBytes;
  CardPages view() const { return CardPages{static_cast<char*>(pages.ptr), page_bytes}; }
  DeviceBuffer sat;  // u64: transactions whose 24 h window held K prior events (counter "window_saturated")
  // per-batch card grouping (feat_slot -> feat_bucket): per-txn slots, keys per bucket, [NB][C] bucket regions,
  // overflow counters by batch parity + the overflow list (key, bucket), prep records. Two sets: the pipelined
  // stream alternates them, so batch i+1's slot kernel runs while batch i's bucket kernel still reads its set.
  struct GroupScratch {
    DeviceBuffer slot, bucket_fill, pairs, ovf_cnt, ovf_key, ovf_b, prep;
    int batch_parity = 0;
  } gs[2];
  DeviceBuffer bucket_scr;  // lean bucket kernel: per-bucket global working set of its slow path
  DeviceBuffer uext, mext, vocab;  // extended profiles + vocabulary flags (feature map, rule scores)
  int64_t n_mext = 0;
  bool vocab_loaded = false;
  double tp_threshold = 0.7;  // JobConfig.fraudThreshold (fl/config/JobConfig.java:47)
};

// Flink window aggregates (windows.hip): device event logs (double-buffered for compaction), sort scratch
struct WindowState {
  bool ready = false;
  int64_t cap = 0, cand_cap = 0;
  int64_t ooo = 10000;                    // watermark lag (ms)
  int64_t wm = INT64_MIN;                 // current watermark
  int64_t min_seen = INT64_MAX;           // smallest event time added (bases the first firing's keys)
  int64_t max_seen = INT64_MIN;           // largest event time added (flush) or observed (sharded)
  bool observed = false;                  // fd_windows_observe since the last step: advance even with n == 0
  DeviceBuffer ulog[2], mlog[2];
  int ucur = 0, mcur = 0;
  int64_t ucount = 0, mcount = 0;
  DeviceBuffer keys, vals, sort_tmp, uout, mout, scalars, stage;
};

// RedisTransactionSink bucket aggregates (sink.hip)
struct SinkState {
  bool ready = false;
  unsigned long long cap = 0, ucap = 0;
  DeviceBuffer table, users, err;
};

// JSON ingest codec lookup tables (ingest.hip): merchant ids and the three vocabularies, hash -> index
struct IngestTables {
  DeviceBuffer mkeys, mvals, vkeys[3], vvals[3];
  unsigned long long mmask = 0, vmask[3] = {0, 0, 0};
  bool mloaded = false, vloaded[3] = {false, false, false};
  int stop_after = 0;  // diagnostics option "ingest_stop_after"
  DeviceBuffer stage_bytes, stage_offsets, stage_out;  // host-API staging
};

// the engine's own RCCL communicators and buffers for the sharded step (comm.hip, fd_sharded_step in engine.hip);
// per-batch buffers in two slots (a step's batch and the next one, prefetched)
struct ShardComm {
  bool ready = false;
  // a step that timed out or failed on the device aborts both communicators (ncclCommAbort: RCCL's blocked
  // kernels exit) before it throws, so no stream is left parked on a peer; afterwards the engine refuses sharded
  // steps, and its syncs / fd_comm_destroy wait on the forward stream only up to comm_timeout_ms
  bool aborted = false;
  std::string abort_reason;
  int rank = 0, world = 1;
  const void* api = nullptr;  // the RcclApi (comm.hip) of the library fd_comm_init was given
  void* fwd = nullptr;   // ncclComm_t: counts + records, on x_fwd
  void* back = nullptr;  // ncclComm_t: results, on the engine stream
  hipStream_t x_fwd = nullptr;
  DeviceBuffer rec[2], cnt[2], back_buf;
  // received records: a ring of three inboxes, so a batch's records exchange waits for the scoring three batches
  // back (long done) instead of two (still running beside the pipeline) — x_fwd is then never parked on an inbox,
  // and the next batch's counts queued behind the records are not held up either (the process has 4 hardware
  // queues for 4+ streams: a parked stream stalls whatever shares its queue)
  static constexpr int kInbox = 3;
  DeviceBuffer inbox[kInbox];
  // the owner's result records, by inbox: the fused kernel writes them in place (round 6: no staging copy). Batch i's
  // scoring follows its records' arrival (in_ev), which followed x_fwd's wait for inbox_ev of batch i - 3 — recorded
  // after that batch's results exchange — so res[q] is free when batch i writes it, with no event of its own
  DeviceBuffer res[kInbox];
  hipEvent_t in_ev[kInbox] = {}, inbox_ev[kInbox] = {};  // records arrived / the engine stream passed their results
  bool inbox_live[kInbox] = {};
  int inbox_next = 0;                                     // the next batch's inbox
  int inbox_of[2] = {0, 0};                               // slot s's batch's inbox
  DeviceBuffer route_blk;                  // the partition's block counts (x_fwd)
  // coherent host-mapped memory per slot: send counts [G], receive counts [G] (FD_MAX_SHARDS each), then a u64
  // sequence word; count_publish_kernel writes the counts and then the sequence, the host polls the sequence
  int64_t* h_cnt[2] = {nullptr, nullptr};
  int64_t* d_hcnt[2] = {nullptr, nullptr};  // the same buffers' device addresses
  unsigned long long cnt_seq[2] = {0, 0};  // the sequence the slot's latest publish writes
  // the prefetched batch (fd_sharded_step's `next`): its caller-given id, size and count slot; its counts are in
  // flight on x_fwd. A later call names it by that id (never by its address: torch's allocator recycles them).
  bool pending = false;
  unsigned long long pending_id = 0;
  int64_t pending_n = 0;
  int pending_slot = 0, next_slot = 0;
  int64_t split[2][2 * FD_MAX_SHARDS] = {};  // a slot's checked split sizes, send [G] then recv [G]
  // Every communicator operation of a step is issued by the calling thread, in one fixed order on every rank
  // (counts of batch i+1, records of batch i on x_fwd; results of batch i on the engine stream): RCCL kernels block
  // on their peers, and ops of two communicators issued from two threads could reach a shared hardware queue in
  // opposite orders on two ranks. (Round 3 ran the next batch's forward half on a worker thread; it measured no
  // faster - 0.0932 vs 0.0943 ms per step, profiles/r03/route_overhead_stream_priority_p1.log - and had that hazard.)
  int64_t timeout_ms = 120000;  // option "comm_timeout_ms": the split-size wait gives up (FD_ERR_HIP) after this
  // option "count_exchange": 1 a batch's per-peer counts travel as ONE ncclAllGather of every rank's send vector
  // (cnt[s]: send [G], then the G x G matrix), issued right after the records group; 0 as 2G point-to-point
  // operations inside it (send [G], receive [G]); -1 (default) the all-gather from 4 ranks (a separate RCCL launch
  // costs ~2 us more host time than the world-1 group's two self operations; at 8 ranks it replaces 16)
  int count_mode = -1;
  bool count_gather = false;  // the form in use (count_mode, world)
  int device = 0;
  // host time inside fd_sharded_step by phase (ns, counters "sharded_host_ns_<phase>", kShardHostPhase order)
  static constexpr int kHostPhases = 8;
  std::atomic<unsigned long long> steps{0}, host_ns[kHostPhases] = {};
  std::atomic<unsigned long long> ops{0};  // RCCL operations issued (send, recv, all-gather; counter "rccl_ops")
};
// "wait": the split sizes; "partition", "counts", "count_copy": a batch's route kernels, count exchange and copy to
// the host; "records": the records exchange; "score": the owner's pipeline; "back", "scatter": results
inline const char* const kShardHostPhase[ShardComm::kHostPhases] = {
    "wait", "partition", "counts", "count_copy", "records", "score", "back", "scatter"};
// per-thread phase clock: lap(ph) adds the time since the previous lap to phase ph
struct HostLaps {
  ShardComm& c;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void operator()(int ph) {
    const auto now = std::chrono::steady_clock::now();
    c.host_ns[ph].fetch_add((unsigned long long)std::chrono::duration_cast<std::chrono::nanoseconds>(now - t).count(),
                            std::memory_order_relaxed);
    t = now;
  }
};

inline int64_t floor_div_host(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}

struct Engine {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  PackedForest forests[kMaxSlots];
  CardStore state;
  LstmModel lstm;
  WindowState windows;
  IngestTables ingest;
  SinkState sink;
  hipStream_t aux_stream = nullptr;            // LSTM head runs here, concurrent with the forests
  hipEvent_t fork_ev = nullptr, join_ev = nullptr;
  hipStream_t aux2_stream = nullptr;           // small batches: the second forest, concurrent with the first
  hipEvent_t join2_ev = nullptr;
  DeviceBuffer seq_buf;                        // per-txn LSTM input sequences of the fused path
  DeviceBuffer seq_desc;                       // latency path: per-txn sequence descriptors (kSeqMaterialized)
  DeviceBuffer feat_vec, feat_in, feat_ext;  // host-API / fused-pipeline staging for features
  // fd_score_batch_pipelined (engine.hip): features and scoring of batch i on pipe_stream[i & 1] (no cross-stream
  // wait between a batch's features and its forests; batch i-1's features waited for by event); vectors / LSTM
  // sequences double-buffered by batch parity
  static constexpr int kPipeSlots = 2;
  hipStream_t pipe_stream[2] = {nullptr, nullptr};
  // batch i's scoring-done event is pipe_done_ev[i mod kDoneRing]: the engine stream, the next batch of a per-model
  // scoring path and — split rows — batch i + 4's slot pass (which rewrites the ring buffer batch i's fused kernel
  // read) wait on it
  static constexpr int kDoneRing = 4;
  hipEvent_t pipe_entry_ev = nullptr, pipe_feat_ev[kPipeSlots] = {}, pipe_done_ev[kDoneRing] = {};
  bool pipe_feat_live[kPipeSlots] = {}, pipe_done_live[kDoneRing] = {};
  bool pipe_dirty = true;  // another engine call since the last pipelined one: order after `stream` first
  // option "slot_stream" (0 off, 1 high-priority stream, 2 low): batch i's slot pass on a stream of its own, so it
  // does not queue behind batch i-2's fused kernel on pipe_stream[i & 1]; its bucket pass waits for it by event.
  // -1 (default) auto: 2 when the card table has >= 2^26 slots, else 0. Config 4 (2^27 slots): 0.0915 -> 0.0897 ms
  // per step at 2 (1: 0.0906); config 3 (10 M cards): 0.0876 -> 0.0948
  int pipe_slot_mode = -1;
  hipStream_t pipe_slot_stream = nullptr;
  hipEvent_t pipe_slot_ev[kPipeSlots] = {};
  // launch_grouped's slot pass goes to this stream (then an event the bucket pass's stream waits for) while set
  hipStream_t slot_pass_stream = nullptr;
  hipEvent_t slot_pass_ev = nullptr;
  unsigned long long pipe_iter = 0;
  unsigned long long pipe_iter_total = 0;  // counter "pipelined_batches"
  unsigned long long ens_single_total = 0;    // counter "ensemble_single_launches": fd_forest_predict batches run by
                                              // the fused kernel over one forest (config 2's timed kernel)
  unsigned long long pipe_split_total = 0;    // counter "pipelined_split_batches": of those, split rows
  unsigned long long pipe_compact_total = 0;  // counter "pipelined_compact_batches": batches scored from compact vectors
  unsigned long long pipe_host_ns = 0;  // counter "pipelined_host_ns": host time inside fd_score_batch_pipelined
  unsigned long long pipe_slot_stream_total = 0;  // counter "pipelined_slot_stream_batches": slot pass on its own stream
  bool pipe_lean = true;   // "pipeline_lean" option: lean bucket kernel (fits beside the ensemble kernel)
  bool pipe_gather = true;  // "pipeline_gather" option: batches of <= kGatherBatchMax take the gather bucket kernel
  DeviceBuffer pipe_vec[kPipeSlots], pipe_seq[kPipeSlots];
  // split rows (compact_vectors 2): RowA | RowB of batch i in ring buffer i mod kSplitRing. With the slot pass on its
  // own stream, batch i's slot kernel writes RowA while batch i - 2's fused kernel (the same pipe_vec parity) may
  // still read its rows — the slot stream waits only for batch i - 2's bucket pass — so the split rows get a deeper
  // ring, and the slot pass waits for the fused kernel that last read its buffer (batch i - 4's pipe_done_ev: long
  // done)
  static constexpr int kSplitRing = 4;
  static_assert(kSplitRing == kDoneRing, "the split-row ring's buffers are released by the done events");
  DeviceBuffer pipe_split[kSplitRing];
  // the scoring streams write a batch's outputs into pipe_out[slot]; one copy kernel on `stream` moves them to the
  // caller's buffers, so the caller's memory is written only in the engine stream's order (torch's caching
  // allocator may hand batch i's freed outputs to batch i+1); batch i+nbuf's scoring waits for pipe_copy_ev[slot]
  DeviceBuffer pipe_out[kPipeSlots];
  hipEvent_t pipe_copy_ev[kPipeSlots] = {};
  bool pipe_copy_live[kPipeSlots] = {};
  bool pipe_copy_vec[kPipeSlots] = {};  // that copy also read the slot's vectors (the slot's next features wait)
  int small_streams = 0;  // score_matrix, latency batches: side streams for the LSTM / other forests (engine.hip)
  bool latency_fused = true;  // "latency_fused": latency pair walk + sums + blend in 2 launches (forest.hip)
  bool seq_ring_lstm = true;  // "seq_ring_lstm": latency batches' LSTM reads card histories from the ring
  bool latency_prebin = true;  // "latency_prebin": the latency pair's binning in the LSTM head's launch (PreBin)
  int latency_prebin_mode = 3;  // its value: 1 the binning workgroups ahead of the LSTM's, 2 after them, 3 (default)
                                // the searches inside the LSTM's own workgroups (lstm.hip InlineSearch; 2 where a
                                // thread would take more than two)
  PreBin prebin;
  unsigned long long prebin_total = 0;  // counter "latency_prebinned_batches"
  bool ens_prio = true;   // "ensemble_prio": the fused kernel's waves issue at priority 2 (above the feature kernels;
                          // the default since round 6's split rows, engine.hip)
  bool ens_bin_global = false;  // "ensemble_bin_global": compact rows binned by searches in global memory (no staging)
  int compact_vectors = 2;      // "compact_vectors": the pipelined stream's scoring rows for the fused kernel when
                                // nobody asked for vectors: 0 the 64-wide vector, 1 compact 64-B rows, 2 split rows
                                // (card-independent half from the slot pass; engine.hip, features.hip Prep32)
  int stream_prio = 3;    // option "stream_priority": the pipeline / forward streams' HIP priorities (engine.hip)
  // host-API staging
  DeviceBuffer stage_in, stage_out0, stage_out1, stage_out2, stage_out3;
  DeviceBuffer scratch_probs, stage_ext;  // score_matrix per-model columns / staged external columns
  DeviceBuffer route_blk, route_out, route_err;  // card-hash routing scratch (route.hip)
  DeviceBuffer route_blk_stream;                 // fd_route_partition_stream's block counts (its own stream)
  ShardComm comm;                                // card-hash sharding over RCCL (comm.hip)
  EnsemblePlan ens;                              // fused XGBoost + IsolationForest + blend (ensemble.hip)
  EnsemblePlan ens1[kMaxSlots];                  // the same kernel over one forest (forest predict), per slot
  bool route_err_live = false;
  // optional per-launch kernel timing (HIP events on the launch stream)
  int forest_variant = 0;  // "forest_kernel" option
  bool ens_owner_fixed = true;  // "ensemble_owner" option (A/B of the fused kernel's chunk-owner schedule)
  int ens_chunks = 0;           // "ensemble_chunks": 0 auto, 1 wide, 2 compact chunk layout (ensemble.hip)
  int lstm_rows = 0;  // "lstm_rows" option: transactions per LSTM workgroup tile (0 auto, 4 or 16)
  bool ensemble_on = true;  // "ensemble" option: the fused XGBoost + IsolationForest + blend kernel (auto)
  bool timing = false;
  int timing_every = 1;               // "timing_every" option: time one launch in N of each kind
  unsigned long long timing_seq[16] = {};
  struct Timed {
    hipEvent_t a, b;
    int kind;
    // a launch split over two streams (the pipelined slot pass on its own stream, then the bucket pass): its
    // second part is c..d, the launch's time the sum of both (the wait between them excluded)
    hipEvent_t c = nullptr, d = nullptr;
    bool split = false;
  };
  std::vector<Timed> events;  // pool
  size_t events_used = 0;
  void activate() const { FD_HIP(hipSetDevice(device)); }
  Timed* next_event_pair(int kind);
};

// forest.hip
struct HostPack {
  std::vector<char> blob;
  std::vector<int32_t> leaf_ids;
  int kind = 0, n_trees = 0, n_chunks = 0, chunk = 0, depth = 0, num_feature = 0;
  size_t tree_bytes = 0, chunk_stride = 0;
  float base_margin = 0.f;
  // binned layout
  bool binned = false;
  std::vector<char> b_blob;
  std::vector<float> b_thr;
  std::vector<int32_t> b_thr_off;
  int b_chunk = 0, b_n_chunks = 0, bin_steps = 0;
  size_t b_tree_bytes = 0, b_chunk_stride = 0;
  // node-only chunks (forest_kernel6); n_chunk == 0 when no supported chunk size fits
  std::vector<char> n_blob, n_leaves;
  int n_chunk = 0, n_n_chunks = 0;
  size_t n_chunk_stride = 0;
  std::vector<uint8_t> pad;  // [tree][2^D] heap slot is a pad node (a leaf above depth D): either way is right
};
// min_depth: pad every tree to at least this depth (the ensemble kernel's common depth)
HostPack pack_forest_host(const fd_forest_params& p, const fd_tree_arrays& t, int min_depth = 0);
void repack_forest(PackedForest& pf, const fd_forest_params& p, const fd_tree_arrays& t);
// two forests of a latency batch, one binning launch (forest.hip); false: not applicable, nothing launched
bool launch_forest_pair(Engine& e, const PackedForest& pa, const PackedForest& pb, const float* d_X, int64_t n,
                        int32_t ld, double* d_prob_a, double* d_prob_b);
void launch_forest(Engine& e, const PackedForest& pf, const float* d_X, int64_t n, int32_t ld,
                   double* d_prob, double* d_raw, int32_t* d_leaf, hipStream_t stream = nullptr);
// a latency batch's XGBoost + IsolationForest and the blend: bin (one launch), both walks (one launch), both
// sequential sums + blend_row over every present model (one launch); cols = the present models' probability columns
// in present order (the two forests' are written, the others read), pos1 / pos2 = p1's / p2's place in it.
// false: not applicable (not one of each kind on the split path at depth 8); nothing launched.
struct BlendConsts;
bool launch_forest_pair_blend(Engine& e, const PackedForest& p1, const PackedForest& p2, const float* d_X, int64_t n,
                              int32_t ld, const BlendConsts& bc, const double* const* cols, int pos1, int pos2,
                              double* dfp, double* dconf, uint8_t* ddec, uint8_t* drisk,
                              hipEvent_t before_blend = nullptr);
// e.prebin for the pair launch_forest_pair_blend will run over d_X (n rows): false (e.prebin.want cleared) when it
// does not apply
bool forest_pair_prebin(Engine& e, const PackedForest& p1, const PackedForest& p2, const float* d_X, int64_t n,
                        int32_t ld);
// windows.hip
void windows_init(Engine& e, const fd_window_params& p);
void windows_step(Engine& e, const fd_txn_batch& t, const fd_window_inputs& in, int64_t n, bool flush,
                  fd_user_window* u_out, int64_t u_cap, int64_t* n_user, fd_merchant_window* m_out, int64_t m_cap,
                  int64_t* n_merch);
void windows_release(Engine& e);
void windows_observe(Engine& e, int64_t max_event_ts);
void merchant_windows_merge(const fd_merchant_window* p, int64_t n, fd_merchant_window* out, int64_t* n_out);
// ingest.hip
void ingest_set_vocab(Engine& e, int which, const uint8_t* bytes, const int64_t* offsets, int64_t n);
void ingest_set_merchants(Engine& e, const uint8_t* bytes, const int64_t* offsets, int64_t n);
void launch_ingest(Engine& e, const uint8_t* d_bytes, const int64_t* d_offsets, int64_t n, const fd_ingest_out& out);
// sink.hip
void sink_init(Engine& e, const fd_sink_params& p);
void sink_update(Engine& e, const fd_txn_batch& t, const fd_window_inputs& in, int64_t n);
void sink_query(Engine& e, int kind, const int64_t* bucket, const int32_t* merchant, int64_t n, fd_aggregate* out);
void sink_evict_before(Engine& e, int64_t hour, int64_t* kept_entries, int64_t* kept_users);
void sink_release(Engine& e);
// snapshot.hip
void state_snapshot(Engine& e, const char* path, int shard, int n_shards, int64_t* bytes_written);
void state_restore(Engine& e, const char* path, int shard, int n_shards, int flags, int64_t* cards_restored);
// features.hip
void state_init(Engine& e, const fd_state_params& p);
void state_clear(Engine& e);
int64_t state_count(Engine& e);
void load_users(Engine& e, const fd_users& u);
void load_merchants(Engine& e, const fd_merchants& m);
// compact: 0 the 64-wide vector; 1 the fused pipeline's compact form (64-B rows: kCompactWidth words, fd_internal.h);
// 2 split rows (features.hip Prep32 / RowA / RowB: RowA [n] then RowB [n], 32 B each; lean bucket pass only)
void launch_features(Engine& e, const fd_txn_batch& t, int64_t n, float* d_vec, double* d_raw,
                     float* d_seq = nullptr, double* d_vel5 = nullptr, hipStream_t stream = nullptr,
                     bool lean = false, int set = 0, hipEvent_t before_buckets = nullptr, int compact = 0,
                     unsigned long long* d_seq_desc = nullptr);
// the same over received 48-B route records (route.hip), no unpack pass; also returns nothing else
void launch_features_records(Engine& e, const void* d_records, int64_t n, float* d_vec, float* d_seq,
                             hipStream_t stream = nullptr, bool lean = false, int set = 0,
                             hipEvent_t before_buckets = nullptr, int compact = 0);
void load_users_ext(Engine& e, const fd_users_ext& u);
void load_merchants_ext(Engine& e, const fd_merchants_ext& m);
void load_vocab(Engine& e, const uint8_t* pay_high_risk, const uint8_t* type_refund);
void launch_features_full(Engine& e, const fd_txn_batch& t, const fd_txn_context& c, int64_t n, float* d_vec,
                          double* d_raw, double* d_fmap, fd_rule_scores* d_rules);
void features_check(Engine& e);
// engine.hip: a non-blocking stream at HIP priority level (+1 the greatest, -1 the least, 0 the default)
hipStream_t make_stream(int level);
// route.hip
unsigned shard_of_host(unsigned long long key, unsigned G);
// stream / scratch: the launch stream and block-count scratch (default: the engine stream and route_blk)
void launch_route_partition(Engine& e, const fd_txn_batch& t, const fd_window_inputs* extra, int64_t n, int G,
                            void* d_records, int64_t* d_counts, hipStream_t stream = nullptr,
                            DeviceBuffer* scratch = nullptr, bool timed = true);
// the sharded step's split form of the partition: block counts + per-shard totals added into `totals` (zero on
// entry) first, so the count exchange can start; then the scan + record scatter (blk: the same scratch)
void launch_route_count(const fd_txn_batch& t, int64_t n, int G, int64_t* totals, hipStream_t st, DeviceBuffer& blk);
// the sharded step's split sizes to the host (comm.hip): cnt[0, 2G) -> host-mapped h, the send half zeroed for the
// next count, then the sequence word h_seq = seq (release); run by the scan kernel of launch_route_place
struct CountPublish {
  int64_t* cnt;
  int G;
  int gather_rank;  // >= 0: the receive counts are column gather_rank of the all-gathered matrix at cnt + G
  int64_t* h;
  unsigned long long* h_seq;
  unsigned long long seq;
};
void launch_route_place(const fd_txn_batch& t, int64_t n, int G, void* d_records, hipStream_t st, DeviceBuffer& blk,
                        const CountPublish* pub = nullptr);
void launch_route_unpack(Engine& e, const void* d_records, const void* d_results, int64_t n, const fd_txn_batch& out,
                         uint8_t* pm, uint8_t* fraud, double* score);
void launch_result_pack(Engine& e, const double* fp, const double* conf, const uint8_t* dec, const uint8_t* risk,
                        const RouteRecord* records, int64_t n, void* d_results);
void launch_result_scatter(Engine& e, const void* d_results, int64_t n, double* fp, double* conf, uint8_t* dec,
                           uint8_t* risk);
void route_check(Engine& e);
// comm.hip
void comm_unique_id(const char* rccl_path, uint8_t* out);
void comm_init(Engine& e, const char* rccl_path, int rank, int world, const uint8_t* id_fwd, const uint8_t* id_back);
void comm_destroy(Engine& e);
// ncclCommAbort both communicators (idempotent); reason is kept for the errors of later calls
void comm_abort(Engine& e, const std::string& reason);
// hipStreamSynchronize, or for an aborted engine a poll bounded by comm_timeout_ms (false: still busy)
bool comm_sync_stream(Engine& e, hipStream_t st);
void comm_launch_counts(Engine& e, const fd_txn_batch& t, int64_t n, hipEvent_t ready, int slot, HostLaps& L);
void comm_wait_counts(Engine& e, int slot, int64_t n, HostLaps& L);  // host wait; split[slot] checked
// records exchange of `slot` behind its inbox slot, + the next batch's count exchange in the same group
void comm_forward_group(Engine& e, int slot, const fd_txn_batch* next, int64_t next_n, hipEvent_t next_ready,
                        int next_slot, HostLaps& L);
void comm_exchange(Engine& e, bool back, hipStream_t st, const void* sendbuf, const int64_t* send, void* recvbuf,
                   const int64_t* recv, size_t elem);
// lstm.hip
void load_lstm(Engine& e, const fd_lstm_params& p);
// d_desc (latency path): per transaction its sequence's place — the card's history ring or row i of d_seq
// (features.hip seq_step); null: every row of d_seq
void launch_lstm(Engine& e, hipStream_t stream, const float* d_seq, int64_t n, int T, double* d_prob,
                 const unsigned long long* d_desc = nullptr);
// model_io.hip: the unchanged XGBoost 2.0.3 JSON model file, flattened (fdengine/forest.py semantics)
struct XgbModel {
  int num_feature = 0;
  double base_score = 0.5;
  std::vector<int64_t> offsets;
  std::vector<int32_t> left, right, feature;
  std::vector<double> threshold, leaf_value;
  std::vector<uint8_t> default_left;
};
void read_xgboost_json(const char* path, XgbModel& out);
// ensemble.hip: the fused path when the present models are one XGBoost and/or one IsolationForest in engine
// slots and the batch is large (false: not applicable, the caller runs the per-model kernels + blend).
// results != nullptr: write route result records (seq from records[i]) instead of the columns.
bool ensemble_applies(Engine& e, const fd_blend_params& p, const int32_t* slots, const uint8_t* present, int64_t n);
// one forest's probabilities through the fused kernel (large batches, no raw / leaf outputs); false: not applicable
bool launch_ensemble_single(Engine& e, int slot, const float* dX, int64_t n, int32_t ld, double* dprob,
                            double* draw, hipStream_t stream);
// compact: 1 dX rows are the compact vector (64-B rows of kCompactWidth words, ld ignored; the plan's features <= 64);
// 2 split rows (RowA [n] then RowB [n] at dX, features.hip)
bool launch_ensemble(Engine& e, const fd_blend_params& p, const int32_t* slots, const uint8_t* present,
                     const float* dX, int64_t n, int32_t ld, double* dMP, double* dfp, double* dconf, uint8_t* ddec,
                     uint8_t* drisk, const RouteRecord* records, ResultRecord* results, int compact = 0);
void forest_loaded(PackedForest& pf, const fd_forest_params& p, const fd_tree_arrays& t);
// blend.hip
void launch_blend(Engine& e, const fd_blend_params& p, int64_t n, const double* const* d_probs,
                  const uint8_t* present, double* d_fp, double* d_conf, uint8_t* d_dec, uint8_t* d_risk);

}  // namespace fd
