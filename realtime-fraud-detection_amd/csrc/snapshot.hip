// snapshot.hip — snapshot / restore of the HBM-resident keyed state.
//
// Reference counterparts: Flink's checkpoints of keyed state (fl/FraudDetectionJob.java:112-136,
// exactly-once, retained on cancellation) and the Redis RDB persistence of the velocity / profile hashes
// (config/redis/redis-master.conf:6-13, `save` + `rdbchecksum yes`). The engine's keyed state replaces both
// on the hot path, so resume / failover needs its own durable image.
//
// The image is KEY-addressed, not a dump of the hash table: one record per occupied card slot
//   { 128-B card header (key, profile + device fingerprints, ring cursor, windows, session) | K ring events |
//     S x 16 f32 LSTM history | 48-B extended user profile (when loaded) }
// followed by the replicated tables (merchants, extended merchants, vocabulary) and the Flink window event
// logs (40-B events, card slots stripped). Restore re-inserts every record by key, so an image restores into
// a table of any capacity and — given (shard, n_shards) — onto a different number of GPUs: each new owner
// reads every old image and keeps the cards it owns (shard_of, route.hip), the counterpart of Flink's
// key-group redistribution on rescale. Sections carry FNV-1a-64 checksums (over 8-byte words).
//
// Snapshot per chunk of 2^18 slots: flag occupied slots -> rocPRIM select (stable: records leave in slot
// order, so an image of the same table is byte-identical) -> gather records (one thread per 16-B word) ->
// D2H (pinned) -> file. Restore per chunk of records: H2D -> find-or-insert by key (shard filter) ->
// scatter words. Both are HBM-bound copies; the file system is the limit.
#include <cstdio>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "fd_internal.h"

namespace fd {
namespace {

constexpr int kHeaderWords = kCardHeaderBytes / 16;  // CardHeader (fd_internal.h)
constexpr int kHeaderKeyWord = (int)(offsetof(CardHeader, key) / 16);  // the 16-B word holding the key (low half)
static_assert(offsetof(CardHeader, key) % 16 == 0, "the key opens its 16-B word");
constexpr int kUextWords = 3;      // 48-B UserExt
constexpr size_t kMerchantBytes = 16, kMerchExtBytes = 16, kWinEventBytes = 40, kVocabBytes = 512;
constexpr int64_t kChunkSlots = 1 << 18;
constexpr size_t kSinkEntryBytes = 48, kSinkUserBytes = 16;  // sink.hip AggEntry / UserEntry

struct __attribute__((packed)) SnapHeader {  // 256 B, little-endian
  char magic[8];
  uint32_t version, header_bytes;
  int32_t window_mode, ring_k, seq_len, has_uext;
  int32_t shard, n_shards, vocab_loaded, windows_present;
  int64_t n_cards, record_bytes, n_merchants, n_mext;
  double tp_threshold;
  int64_t win_ooo, win_wm, win_min_seen, win_max_seen, ucount, mcount;
  uint64_t checksum[6];  // cards, merchants, mext, vocab, user log, merchant log
  int32_t ext_flags;      // trailing extension sections: bit 0 sink aggregates, bit 1 ingest tables
  int32_t ext_pad;
  uint64_t ext_checksum;
  uint8_t pad[56];
};
static_assert(sizeof(SnapHeader) == 256, "SnapHeader must be 256 B");
constexpr char kMagic[8] = {'F', 'D', 'S', 'N', 'A', 'P', 0, 1};
constexpr uint32_t kVersion = 3;  // 3: the mutable fields in the header's first 64 B, the key at byte 64 (round 5);
                                  // 2: 128-B card header with the fingerprints folded in; 1: 64-B + fps plane

struct Fnv {
  uint64_t h = 0xcbf29ce484222325ull;
  void add(const void* p, size_t bytes) {  // bytes: multiple of 8 except the tail
    const unsigned char* c = static_cast<const unsigned char*>(p);
    size_t i = 0;
    for (; i + 8 <= bytes; i += 8) {
      uint64_t w;
      std::memcpy(&w, c + i, 8);
      h = (h ^ w) * 0x100000001b3ull;
    }
    for (; i < bytes; ++i) h = (h ^ c[i]) * 0x100000001b3ull;
  }
};

// per-record word map (16-B words): header | ring | seq | uext
struct RecMap {
  int K, S, uext;
  int w_ring, w_seq, w_uext, words;
};
RecMap rec_map(int K, int S, bool uext) {
  RecMap m{K, S, uext ? 1 : 0, 0, 0, 0, 0};
  m.w_ring = kHeaderWords;
  m.w_seq = m.w_ring + K;
  m.w_uext = m.w_seq + S * 4;
  m.words = m.w_uext + (uext ? kUextWords : 0);
  return m;
}

struct Planes {  // the per-slot state as 16-B words: the card pages (header, then ring), LSTM history, extended profile
  uint4* pages;
  long long page_words;
  bool ring;  // the pages hold the K ring events (sliding mode); redis_compat records carry zero ring words
  uint4* seq;
  uint4* uext;
};

// the word of `slot`'s state that record word w maps to (null: a ring word of a page without a ring)
__device__ __forceinline__ uint4* plane_word(const Planes& P, const RecMap& m, long long slot, int w) {
  if (w < m.w_ring) return P.pages + slot * P.page_words + w;
  if (w < m.w_seq) return P.ring ? P.pages + slot * P.page_words + w : nullptr;  // header words, then ring words
  if (w < m.w_uext) return P.seq + slot * (m.S * 4) + (w - m.w_seq);
  return P.uext + slot * kUextWords + (w - m.w_uext);
}

__device__ __forceinline__ unsigned long long smix64(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

// route.hip shard_of_dev (keys are stored normalised: 0 -> 1)
__device__ __forceinline__ bool owned(unsigned long long key, unsigned shard, unsigned G) {
  if (G <= 1) return true;
  if (key == 0ull) key = 1ull;
  return (unsigned)(((smix64(key) >> 32) * (unsigned long long)G) >> 32) == shard;
}

// features.hip find_or_insert over a strided key array

__global__ void __launch_bounds__(256) snap_flag_kernel(const uint4* __restrict__ pages, long long page_words,
                                                        long long lo, long long n, unsigned char* __restrict__ flags) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 h = pages[(lo + i) * page_words + kHeaderKeyWord];  // the header's key
  flags[i] = (h.x | h.y) != 0u;
}

__global__ void __launch_bounds__(256) snap_gather_kernel(Planes P, RecMap m, const unsigned* __restrict__ slots,
                                                          long long n_words, uint4* __restrict__ out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_words) return;
  const long long r = t / m.words;
  const int w = (int)(t - r * m.words);
  const uint4* src = plane_word(P, m, (long long)slots[r], w);
  out[t] = src ? *src : make_uint4(0u, 0u, 0u, 0u);
}

__global__ void __launch_bounds__(256) restore_slot_kernel(unsigned long long* keys, CardPages pages, long long mask,
                                                           const uint4* __restrict__ recs, int words, long long n,
                                                           unsigned shard, unsigned G, long long* __restrict__ slots,
                                                           unsigned long long* restored, unsigned* err) {
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint4 h = recs[r * words + kHeaderKeyWord];
  const unsigned long long key = ((unsigned long long)h.y << 32) | h.x;
  long long s = -1;
  if (owned(key, shard, G)) {
    s = card_slot(keys, pages, mask, key);
    if (s < 0)
      atomicOr(err, 1u);
    else
      atomicAdd(restored, 1ull);
  }
  slots[r] = s;
}

__global__ void __launch_bounds__(256) restore_scatter_kernel(Planes P, RecMap m, const long long* __restrict__ slots,
                                                              const uint4* __restrict__ recs, long long n_words) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_words) return;
  const long long r = t / m.words;
  const int w = (int)(t - r * m.words);
  const long long s = slots[r];
  if (s < 0) return;
  uint4* dst = plane_word(P, m, s, w);
  if (dst) *dst = recs[t];
}

// window events (windows.hip WinEvent: ts @0, cents @8, card key @16, slot @24): filter by owner, re-slot
// through the card table, append to the log
__global__ void __launch_bounds__(256) restore_events_kernel(unsigned long long* keys, CardPages pages, long long mask,
                                                             const unsigned char* __restrict__ in, long long n,
                                                             unsigned shard, unsigned G, unsigned char* __restrict__ log,
                                                             unsigned long long* count, unsigned* err) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned char* ev = in + i * kWinEventBytes;
  const unsigned long long key = *reinterpret_cast<const unsigned long long*>(ev + 16);
  if (!owned(key, shard, G)) return;
  const long long s = card_slot(keys, pages, mask, key);
  if (s < 0) {
    atomicOr(err, 1u);
    return;
  }
  const unsigned long long at = atomicAdd(count, 1ull);
  unsigned char* o = log + at * kWinEventBytes;
  for (int q = 0; q < (int)kWinEventBytes; q += 8)
    *reinterpret_cast<unsigned long long*>(o + q) = *reinterpret_cast<const unsigned long long*>(ev + q);
  *reinterpret_cast<unsigned*>(o + 24) = (unsigned)s;
}

unsigned blocks(long long n) { return (unsigned)((n + 255) / 256); }

struct File {
  FILE* f = nullptr;
  ~File() {
    if (f) std::fclose(f);
  }
};

struct Pinned {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t need) {
    if (need <= bytes) return;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
    FD_HIP(hipHostMalloc(&p, need, hipHostMallocDefault));
    bytes = need;
  }
  ~Pinned() {
    if (p) (void)hipHostFree(p);
  }
};

void write_all(FILE* f, const void* p, size_t bytes, Fnv* h) {
  if (bytes == 0) return;
  FD_REQUIRE(std::fwrite(p, 1, bytes, f) == bytes, FD_ERR_IO, "snapshot: write failed (disk full?)");
  if (h) h->add(p, bytes);
}

void read_all(FILE* f, void* p, size_t bytes, Fnv* h) {
  if (bytes == 0) return;
  FD_REQUIRE(std::fread(p, 1, bytes, f) == bytes, FD_ERR_IO, "snapshot: truncated file");
  if (h) h->add(p, bytes);
}

// Checksum pass over the whole image before anything is restored: a truncated or corrupt file (a partial copy
// during a re-shard) fails here with the engine's state untouched. Leaves the file at the first section.
// A v2 image's 128-B card header (before the round-5 relayout) rewritten in place as the v3 CardHeader. v2 byte
// offsets: key 0, last_ts 8, avg 16, age 24, flags 28, ring_n / ring_head / unsorted 32-34, wc[3] 36-38, fp[3] 40,
// ws[3] 64, wo[3] 88 (absolute oldest in-window times), rc_sum 112, rc_cnt 120. v3 keeps the oldest times as offsets
// below last_ts and the redis_compat session amount in ws[0].
void header_v2_to_v3(unsigned char* rec, int mode) {
  struct V2 {
    unsigned long long key;
    long long last_ts;
    double avg;
    int age;
    unsigned flags;
    unsigned char ring_n, ring_head, unsorted, pad0, wc[3], pad1;
    unsigned long long fp[3];
    long long ws[3], wo[3], rc_sum;
    int rc_cnt, pad2;
  };
  static_assert(sizeof(V2) == 128 && offsetof(V2, ws) == 64 && offsetof(V2, rc_cnt) == 120, "v2 card header");
  V2 o;
  std::memcpy(&o, rec, sizeof o);
  CardHeader h;
  std::memset(&h, 0, sizeof h);
  h.last_ts = o.last_ts;
  h.ring_n = o.ring_n;
  h.ring_head = o.ring_head;
  h.unsorted = o.unsorted;
  for (int k = 0; k < 3; ++k) {
    h.wc[k] = o.wc[k];
    h.ws[k] = o.ws[k];
    h.wod[k] = o.wc[k] > 0 ? (unsigned)(o.last_ts - o.wo[k]) : 0u;  // an in-window event is < 2^32 ms old
    h.fp[k] = o.fp[k];
  }
  if (mode == FD_WINDOW_REDIS_COMPAT) h.ws[0] = o.rc_sum;
  h.flags = o.flags;
  h.rc_cnt = o.rc_cnt;
  h.key = o.key;
  h.avg = o.avg;
  h.age = o.age;
  std::memcpy(rec, &h, sizeof h);
}

void verify_image(FILE* f, const SnapHeader& hd, size_t rec_bytes) {
  const long start = std::ftell(f);
  std::vector<char> buf(1 << 20);
  auto section = [&](size_t bytes, Fnv* h) {
    for (size_t off = 0; off < bytes;) {
      const size_t b = std::min(bytes - off, buf.size());
      read_all(f, buf.data(), b, h);
      off += b;
    }
  };
  Fnv hc, hm, hx, hv, hu, hl;
  section((size_t)hd.n_cards * rec_bytes, &hc);
  section((size_t)hd.n_merchants * kMerchantBytes, &hm);
  section((size_t)hd.n_mext * kMerchExtBytes, &hx);
  if (hd.vocab_loaded) section(kVocabBytes, &hv);
  section((size_t)hd.ucount * kWinEventBytes, &hu);
  section((size_t)hd.mcount * kWinEventBytes, &hl);
  FD_REQUIRE(hc.h == hd.checksum[0], FD_ERR_IO, "restore: card section checksum mismatch (nothing restored)");
  FD_REQUIRE(hm.h == hd.checksum[1] && hx.h == hd.checksum[2] && hv.h == hd.checksum[3], FD_ERR_IO,
             "restore: table section checksum mismatch (nothing restored)");
  FD_REQUIRE(hu.h == hd.checksum[4] && hl.h == hd.checksum[5], FD_ERR_IO,
             "restore: window log checksum mismatch (nothing restored)");
  if (hd.ext_flags) {
    Fnv he;
    if (hd.ext_flags & 1) {
      int64_t meta[4];
      read_all(f, meta, sizeof meta, &he);
      FD_REQUIRE(meta[0] > 0 && meta[1] > 0 && meta[0] < (1ll << 40) && meta[1] < (1ll << 40), FD_ERR_IO,
                 "restore: corrupt sink section");
      section((size_t)meta[0] * kSinkEntryBytes + (size_t)meta[1] * kSinkUserBytes, &he);
    }
    if (hd.ext_flags & 2) {
      int64_t meta[4];
      read_all(f, meta, sizeof meta, &he);
      for (int t = 0; t < 4; ++t) {
        FD_REQUIRE(meta[t] >= 0 && meta[t] < (1ll << 40), FD_ERR_IO, "restore: corrupt ingest section");
        section((size_t)meta[t] * 8, &he);
        section((size_t)meta[t] * 4, &he);
      }
    }
    FD_REQUIRE(he.h == hd.ext_checksum, FD_ERR_IO, "restore: extension section checksum mismatch (nothing restored)");
  }
  FD_REQUIRE(std::fseek(f, start, SEEK_SET) == 0, FD_ERR_IO, "restore: cannot rewind the snapshot");
}

Planes planes_of(CardStore& st) {
  return Planes{st.pages.as<uint4>(), st.page_bytes / 16, st.mode == FD_WINDOW_SLIDING,
                st.seq.ptr ? st.seq.as<uint4>() : nullptr, st.uext.ptr ? st.uext.as<uint4>() : nullptr};
}

// D2H a device table into the file through the pinned buffer
void dump_device(Engine& e, FILE* f, const void* d, size_t bytes, Pinned& pin, Fnv* h) {
  for (size_t off = 0; off < bytes;) {
    const size_t b = std::min(bytes - off, pin.bytes);
    FD_HIP(hipMemcpyAsync(pin.p, static_cast<const char*>(d) + off, b, hipMemcpyDeviceToHost, e.stream));
    FD_HIP(hipStreamSynchronize(e.stream));
    write_all(f, pin.p, b, h);
    off += b;
  }
}

}  // namespace

void state_snapshot(Engine& e, const char* path, int shard, int n_shards, int64_t* bytes_written) {
  CardStore& st = e.state;
  WindowState& w = e.windows;
  FD_REQUIRE(st.ready, FD_ERR_NOT_LOADED, "card state not initialised (fd_state_init)");
  FD_REQUIRE(path && *path, FD_ERR_INVALID_ARG, "null snapshot path");
  FD_REQUIRE(n_shards >= 1 && shard >= 0 && shard < n_shards, FD_ERR_INVALID_ARG, "bad shard / n_shards");
  FD_HIP(hipStreamSynchronize(e.stream));
  const RecMap m = rec_map(st.K, st.S, st.uext.ptr != nullptr);
  const size_t rec_bytes = (size_t)m.words * 16;

  SnapHeader hd{};
  std::memcpy(hd.magic, kMagic, 8);
  hd.version = kVersion;
  hd.header_bytes = sizeof(SnapHeader);
  hd.window_mode = st.mode;
  hd.ring_k = st.K;
  hd.seq_len = st.S;
  hd.has_uext = m.uext;
  hd.shard = shard;
  hd.n_shards = n_shards;
  hd.vocab_loaded = st.vocab_loaded ? 1 : 0;
  // window state worth restoring: initialised and used (a cleared / never-stepped window state is absent)
  hd.windows_present =
      (w.ready && (w.ucount > 0 || w.mcount > 0 || w.wm != INT64_MIN || w.max_seen != INT64_MIN)) ? 1 : 0;
  hd.record_bytes = (int64_t)rec_bytes;
  hd.n_merchants = st.n_merchants;
  hd.n_mext = st.mext.ptr ? st.n_mext : 0;
  hd.tp_threshold = st.tp_threshold;
  hd.win_ooo = w.ooo;
  hd.win_wm = w.wm;
  hd.win_min_seen = w.min_seen;
  hd.win_max_seen = w.max_seen;
  hd.ucount = hd.windows_present ? w.ucount : 0;
  hd.mcount = hd.windows_present ? w.mcount : 0;

  const std::string tmp = std::string(path) + ".tmp";
  File out;
  out.f = std::fopen(tmp.c_str(), "wb");
  FD_REQUIRE(out.f, FD_ERR_IO, "snapshot: cannot open " + tmp);
  write_all(out.f, &hd, sizeof hd, nullptr);  // placeholder, rewritten at the end

  const int64_t chunk = std::min<int64_t>(kChunkSlots, st.cap);
  DeviceBuffer flags, sel, nsel, tmpbuf, recs;
  flags.ensure((size_t)chunk);
  sel.ensure((size_t)chunk * 4);
  nsel.ensure(8);
  recs.ensure((size_t)chunk * rec_bytes);
  Pinned pin;
  pin.ensure(std::max<size_t>((size_t)chunk * rec_bytes, 1 << 20));
  size_t tb = 0;
  FD_HIP(rocprim::select(nullptr, tb, rocprim::counting_iterator<unsigned>(0u), flags.as<unsigned char>(),
                         sel.as<unsigned>(), nsel.as<unsigned>(), (size_t)chunk, e.stream));
  tmpbuf.ensure(std::max<size_t>(tb, 16));
  const Planes P = planes_of(st);
  Fnv h_cards;
  int64_t n_cards = 0;
  for (int64_t lo = 0; lo < st.cap; lo += chunk) {
    const int64_t n = std::min<int64_t>(chunk, st.cap - lo);
    hipLaunchKernelGGL(snap_flag_kernel, dim3(blocks(n)), dim3(256), 0, e.stream, st.pages.as<const uint4>(),
                       st.page_bytes / 16, (long long)lo, (long long)n, flags.as<unsigned char>());
    FD_HIP(hipGetLastError());
    FD_HIP(rocprim::select(tmpbuf.ptr, tb, rocprim::counting_iterator<unsigned>((unsigned)lo),
                           flags.as<unsigned char>(), sel.as<unsigned>(), nsel.as<unsigned>(), (size_t)n, e.stream));
    unsigned c = 0;
    FD_HIP(hipMemcpyAsync(&c, nsel.ptr, 4, hipMemcpyDeviceToHost, e.stream));
    FD_HIP(hipStreamSynchronize(e.stream));
    if (c == 0) continue;
    const long long words = (long long)c * m.words;
    hipLaunchKernelGGL(snap_gather_kernel, dim3(blocks(words)), dim3(256), 0, e.stream, P, m, sel.as<const unsigned>(),
                       words, recs.as<uint4>());
    FD_HIP(hipGetLastError());
    FD_HIP(hipMemcpyAsync(pin.p, recs.ptr, (size_t)c * rec_bytes, hipMemcpyDeviceToHost, e.stream));
    FD_HIP(hipStreamSynchronize(e.stream));
    write_all(out.f, pin.p, (size_t)c * rec_bytes, &h_cards);
    n_cards += c;
  }
  hd.n_cards = n_cards;
  hd.checksum[0] = h_cards.h;
  Fnv h_m, h_x, h_v, h_u, h_l;
  if (hd.n_merchants) dump_device(e, out.f, st.merchants.ptr, (size_t)hd.n_merchants * kMerchantBytes, pin, &h_m);
  if (hd.n_mext) dump_device(e, out.f, st.mext.ptr, (size_t)hd.n_mext * kMerchExtBytes, pin, &h_x);
  if (hd.vocab_loaded) dump_device(e, out.f, st.vocab.ptr, kVocabBytes, pin, &h_v);
  if (hd.ucount) dump_device(e, out.f, w.ulog[w.ucur].ptr, (size_t)hd.ucount * kWinEventBytes, pin, &h_u);
  if (hd.mcount) dump_device(e, out.f, w.mlog[w.mcur].ptr, (size_t)hd.mcount * kWinEventBytes, pin, &h_l);
  // extension sections: sink aggregates (raw tables; resume on the same shard), ingest lookup tables
  Fnv h_ext;
  SinkState& sk = e.sink;
  if (sk.ready) {
    hd.ext_flags |= 1;
    const int64_t meta[4] = {(int64_t)sk.cap, (int64_t)sk.ucap, shard, n_shards};
    write_all(out.f, meta, sizeof meta, &h_ext);
    dump_device(e, out.f, sk.table.ptr, sk.cap * kSinkEntryBytes, pin, &h_ext);
    dump_device(e, out.f, sk.users.ptr, sk.ucap * kSinkUserBytes, pin, &h_ext);
  }
  IngestTables& it = e.ingest;
  if (it.mloaded || it.vloaded[0] || it.vloaded[1] || it.vloaded[2]) {
    hd.ext_flags |= 2;
    const int64_t meta[4] = {it.mloaded ? (int64_t)it.mmask + 1 : 0, it.vloaded[0] ? (int64_t)it.vmask[0] + 1 : 0,
                             it.vloaded[1] ? (int64_t)it.vmask[1] + 1 : 0, it.vloaded[2] ? (int64_t)it.vmask[2] + 1 : 0};
    write_all(out.f, meta, sizeof meta, &h_ext);
    for (int t = 0; t < 4; ++t) {
      if (!meta[t]) continue;
      DeviceBuffer& kb = t == 0 ? it.mkeys : it.vkeys[t - 1];
      DeviceBuffer& vb = t == 0 ? it.mvals : it.vvals[t - 1];
      dump_device(e, out.f, kb.ptr, (size_t)meta[t] * 8, pin, &h_ext);
      dump_device(e, out.f, vb.ptr, (size_t)meta[t] * 4, pin, &h_ext);
    }
  }
  hd.ext_checksum = h_ext.h;
  hd.checksum[1] = h_m.h;
  hd.checksum[2] = h_x.h;
  hd.checksum[3] = h_v.h;
  hd.checksum[4] = h_u.h;
  hd.checksum[5] = h_l.h;
  const long total = std::ftell(out.f);
  FD_REQUIRE(std::fseek(out.f, 0, SEEK_SET) == 0, FD_ERR_IO, "snapshot: seek failed");
  write_all(out.f, &hd, sizeof hd, nullptr);
  FD_REQUIRE(std::fflush(out.f) == 0, FD_ERR_IO, "snapshot: flush failed");
  std::fclose(out.f);
  out.f = nullptr;
  FD_REQUIRE(std::rename(tmp.c_str(), path) == 0, FD_ERR_IO, std::string("snapshot: cannot rename to ") + path);
  if (bytes_written) *bytes_written = total;
}

void state_restore(Engine& e, const char* path, int shard, int n_shards, int flags_in, int64_t* cards_restored) {
  CardStore& st = e.state;
  WindowState& w = e.windows;
  FD_REQUIRE(st.ready, FD_ERR_NOT_LOADED, "card state not initialised (fd_state_init)");
  FD_REQUIRE(path && *path, FD_ERR_INVALID_ARG, "null snapshot path");
  FD_REQUIRE(n_shards >= 1 && shard >= 0 && shard < n_shards, FD_ERR_INVALID_ARG, "bad shard / n_shards");
  File in;
  in.f = std::fopen(path, "rb");
  FD_REQUIRE(in.f, FD_ERR_IO, std::string("restore: cannot open ") + path);
  SnapHeader hd{};
  read_all(in.f, &hd, sizeof hd, nullptr);
  FD_REQUIRE(std::memcmp(hd.magic, kMagic, 8) == 0, FD_ERR_IO, "restore: not an fdengine state snapshot");
  FD_REQUIRE((hd.version == kVersion || hd.version == 2) && hd.header_bytes == sizeof(SnapHeader),
             FD_ERR_UNSUPPORTED, "restore: unsupported snapshot version (this build reads v2 and v3 images)");
  FD_REQUIRE(hd.window_mode == st.mode && hd.ring_k == st.K && hd.seq_len == st.S, FD_ERR_INVALID_ARG,
             "restore: snapshot window_mode / ring_k / seq_len differ from fd_state_init's");
  const RecMap m = rec_map(st.K, st.S, hd.has_uext != 0);
  FD_REQUIRE(hd.record_bytes == (int64_t)m.words * 16 && hd.n_cards >= 0, FD_ERR_IO, "restore: corrupt header");
  const bool skip_windows = (flags_in & FD_RESTORE_SKIP_WINDOWS) != 0;
  const bool has_events = hd.ucount > 0 || hd.mcount > 0;
  if (hd.windows_present && !skip_windows) {
    FD_REQUIRE(w.ready, FD_ERR_NOT_LOADED,
               "restore: the snapshot holds window state: call fd_windows_init first (or FD_RESTORE_SKIP_WINDOWS)");
    const bool empty = w.ucount == 0 && w.mcount == 0 && w.wm == INT64_MIN && w.max_seen == INT64_MIN;
    FD_REQUIRE(empty || w.wm == hd.win_wm, FD_ERR_INVALID_ARG,
               "restore: window watermarks differ across the merged snapshots");
    FD_REQUIRE(w.ucount + hd.ucount <= w.cap && w.mcount + hd.mcount <= w.cap, FD_ERR_OOM,
               "restore: window event log too small (fd_window_params.log_capacity)");
  }
  verify_image(in.f, hd, (size_t)m.words * 16);
  FD_HIP(hipStreamSynchronize(e.stream));
  if (m.uext && !st.uext.ptr) {
    st.uext.ensure((size_t)st.cap * kUextWords * 16);
    FD_HIP(hipMemsetAsync(st.uext.ptr, 0, (size_t)st.cap * kUextWords * 16, e.stream));
  }
  const Planes P = planes_of(st);

  const size_t rec_bytes = (size_t)m.words * 16;
  const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(kChunkSlots, hd.n_cards));
  DeviceBuffer recs, slots, cnt;
  recs.ensure(std::max<size_t>((size_t)chunk * rec_bytes, kWinEventBytes * 4096));
  slots.ensure((size_t)chunk * 8);
  cnt.ensure(16);
  FD_HIP(hipMemsetAsync(cnt.ptr, 0, 16, e.stream));
  Pinned pin;
  pin.ensure(std::max<size_t>((size_t)chunk * rec_bytes, 1 << 20));
  unsigned long long* d_restored = cnt.as<unsigned long long>();
  unsigned* d_err = reinterpret_cast<unsigned*>(cnt.as<char>() + 8);
  Fnv h_cards;
  for (int64_t lo = 0; lo < hd.n_cards; lo += chunk) {
    const int64_t n = std::min<int64_t>(chunk, hd.n_cards - lo);
    read_all(in.f, pin.p, (size_t)n * rec_bytes, &h_cards);  // the checksum covers the bytes as stored
    if (hd.version == 2)
      for (int64_t r = 0; r < n; ++r) header_v2_to_v3(static_cast<unsigned char*>(pin.p) + (size_t)r * rec_bytes, st.mode);
    FD_HIP(hipMemcpyAsync(recs.ptr, pin.p, (size_t)n * rec_bytes, hipMemcpyHostToDevice, e.stream));
    hipLaunchKernelGGL(restore_slot_kernel, dim3(blocks(n)), dim3(256), 0, e.stream,
                       st.keys.as<unsigned long long>(), st.view(), (long long)(st.cap - 1),
                       recs.as<const uint4>(), m.words, (long long)n, (unsigned)shard, (unsigned)n_shards,
                       slots.as<long long>(), d_restored, d_err);
    FD_HIP(hipGetLastError());
    const long long words = (long long)n * m.words;
    hipLaunchKernelGGL(restore_scatter_kernel, dim3(blocks(words)), dim3(256), 0, e.stream, P, m,
                       slots.as<const long long>(), recs.as<const uint4>(), words);
    FD_HIP(hipGetLastError());
    FD_HIP(hipStreamSynchronize(e.stream));  // the pinned buffer is refilled next
  }
  unsigned long long res = 0;
  FD_HIP(hipMemcpyAsync(&res, d_restored, 8, hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  FD_REQUIRE(h_cards.h == hd.checksum[0], FD_ERR_IO,
             "restore: card section checksum mismatch (state unspecified: fd_state_clear)");

  // replicated tables: replace
  Fnv h_m, h_x, h_v;
  if (hd.n_merchants > 0) {
    std::vector<char> b((size_t)hd.n_merchants * kMerchantBytes);
    read_all(in.f, b.data(), b.size(), &h_m);
    st.merchants.ensure(std::max<size_t>(16, b.size()));
    FD_HIP(hipMemcpy(st.merchants.ptr, b.data(), b.size(), hipMemcpyHostToDevice));
    st.n_merchants = hd.n_merchants;
  }
  if (hd.n_mext > 0) {
    std::vector<char> b((size_t)hd.n_mext * kMerchExtBytes);
    read_all(in.f, b.data(), b.size(), &h_x);
    st.mext.ensure(b.size());
    FD_HIP(hipMemcpy(st.mext.ptr, b.data(), b.size(), hipMemcpyHostToDevice));
    st.n_mext = hd.n_mext;
  }
  if (hd.vocab_loaded) {
    unsigned char b[kVocabBytes];
    read_all(in.f, b, kVocabBytes, &h_v);
    st.vocab.ensure(kVocabBytes);
    FD_HIP(hipMemcpy(st.vocab.ptr, b, kVocabBytes, hipMemcpyHostToDevice));
    st.vocab_loaded = true;
  }
  st.tp_threshold = hd.tp_threshold;
  FD_REQUIRE(h_m.h == hd.checksum[1] && h_x.h == hd.checksum[2] && h_v.h == hd.checksum[3], FD_ERR_IO,
             "restore: table section checksum mismatch");

  // window event logs
  if (hd.windows_present && !skip_windows) {
    const bool empty = w.ucount == 0 && w.mcount == 0 && w.wm == INT64_MIN && w.max_seen == INT64_MIN;
    if (empty) {
      w.wm = hd.win_wm;
      w.min_seen = hd.win_min_seen;
      w.max_seen = hd.win_max_seen;
    } else {
      w.min_seen = std::min<int64_t>(w.min_seen, hd.win_min_seen);
      w.max_seen = std::max<int64_t>(w.max_seen, hd.win_max_seen);
    }
    w.ooo = hd.win_ooo;
    for (int which = 0; which < 2; ++which) {
      const int64_t n_ev = which == 0 ? hd.ucount : hd.mcount;
      Fnv hh;
      DeviceBuffer& log = which == 0 ? w.ulog[w.ucur] : w.mlog[w.mcur];
      int64_t& count = which == 0 ? w.ucount : w.mcount;
      const int64_t ev_chunk = (int64_t)(std::min(pin.bytes, recs.bytes) / kWinEventBytes);
      unsigned long long* d_count = slots.as<unsigned long long>();
      FD_HIP(hipMemcpyAsync(d_count, &count, 8, hipMemcpyHostToDevice, e.stream));
      for (int64_t lo = 0; lo < n_ev; lo += ev_chunk) {
        const int64_t n = std::min<int64_t>(ev_chunk, n_ev - lo);
        read_all(in.f, pin.p, (size_t)n * kWinEventBytes, &hh);
        FD_HIP(hipMemcpyAsync(recs.ptr, pin.p, (size_t)n * kWinEventBytes, hipMemcpyHostToDevice, e.stream));
        hipLaunchKernelGGL(restore_events_kernel, dim3(blocks(n)), dim3(256), 0, e.stream,
                           st.keys.as<unsigned long long>(), st.view(), (long long)(st.cap - 1),
                           recs.as<const unsigned char>(), (long long)n, (unsigned)shard, (unsigned)n_shards,
                           log.as<unsigned char>(), d_count, d_err);
        FD_HIP(hipGetLastError());
        FD_HIP(hipStreamSynchronize(e.stream));
      }
      unsigned long long c = 0;
      FD_HIP(hipMemcpyAsync(&c, d_count, 8, hipMemcpyDeviceToHost, e.stream));
      FD_HIP(hipStreamSynchronize(e.stream));
      count = (int64_t)c;
      FD_REQUIRE(hh.h == hd.checksum[4 + which], FD_ERR_IO, "restore: window log checksum mismatch");
    }
  } else if (has_events && !skip_windows) {
    // windows_present == 0 but events recorded: corrupt
    throw Error(FD_ERR_IO, "restore: corrupt header (window events without window state)");
  } else if (has_events) {
    // skipped window logs: step over them so the extension sections that follow are read in place
    const long skip = (long)((hd.ucount + hd.mcount) * (int64_t)kWinEventBytes);
    FD_REQUIRE(std::fseek(in.f, skip, SEEK_CUR) == 0, FD_ERR_IO, "restore: truncated snapshot (window logs)");
  }
  // extension sections
  if (hd.ext_flags) {
    Fnv h_ext;
    std::vector<char> tmp;
    auto read_to_device = [&](DeviceBuffer& d, size_t bytes) {
      tmp.resize(bytes);
      read_all(in.f, tmp.data(), bytes, &h_ext);
      d.ensure(std::max<size_t>(bytes, 16));
      FD_HIP(hipMemcpy(d.ptr, tmp.data(), bytes, hipMemcpyHostToDevice));
    };
    if (hd.ext_flags & 1) {
      int64_t meta[4];
      read_all(in.f, meta, sizeof meta, &h_ext);
      FD_REQUIRE(meta[0] > 0 && meta[1] > 0 && (meta[0] & (meta[0] - 1)) == 0 && (meta[1] & (meta[1] - 1)) == 0,
                 FD_ERR_IO, "restore: corrupt sink section");
      const bool skip_sink = (flags_in & FD_RESTORE_SKIP_SINK) != 0;
      if (!skip_sink) {
        FD_REQUIRE(meta[2] == shard && meta[3] == n_shards, FD_ERR_INVALID_ARG,
                   "restore: sink aggregates resume only on the same shard of the same shard count "
                   "(FD_RESTORE_SKIP_SINK to re-shard without them)");
        SinkState& sk = e.sink;
        read_to_device(sk.table, (size_t)meta[0] * kSinkEntryBytes);
        read_to_device(sk.users, (size_t)meta[1] * kSinkUserBytes);
        sk.cap = (unsigned long long)meta[0];
        sk.ucap = (unsigned long long)meta[1];
        sk.err.ensure(16);
        FD_HIP(hipMemset(sk.err.ptr, 0, 16));
        sk.ready = true;
      } else {
        tmp.resize((size_t)meta[0] * kSinkEntryBytes + (size_t)meta[1] * kSinkUserBytes);
        read_all(in.f, tmp.data(), tmp.size(), &h_ext);
      }
    }
    if (hd.ext_flags & 2) {
      int64_t meta[4];
      read_all(in.f, meta, sizeof meta, &h_ext);
      IngestTables& it = e.ingest;
      for (int t = 0; t < 4; ++t) {
        if (!meta[t]) continue;
        FD_REQUIRE(meta[t] > 0 && (meta[t] & (meta[t] - 1)) == 0, FD_ERR_IO, "restore: corrupt ingest section");
        read_to_device(t == 0 ? it.mkeys : it.vkeys[t - 1], (size_t)meta[t] * 8);
        read_to_device(t == 0 ? it.mvals : it.vvals[t - 1], (size_t)meta[t] * 4);
        if (t == 0) {
          it.mmask = (unsigned long long)meta[t] - 1;
          it.mloaded = true;
        } else {
          it.vmask[t - 1] = (unsigned long long)meta[t] - 1;
          it.vloaded[t - 1] = true;
        }
      }
    }
    FD_REQUIRE(h_ext.h == hd.ext_checksum, FD_ERR_IO, "restore: extension section checksum mismatch");
  }
  unsigned err = 0;
  FD_HIP(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, e.stream));
  FD_HIP(hipStreamSynchronize(e.stream));
  FD_REQUIRE(err == 0, FD_ERR_OOM, "restore: card table full: raise fd_state_params.capacity");
  if (cards_restored) *cards_restored = (int64_t)res;
}

}  // namespace fd
