// ensemble.hip — the fused scoring kernel of the hot path: the XGBoost primary classifier
// (ml/models/model_manager.py:309-311) and the IsolationForest (:338-346) walked over ONE binned feature
// tile per 256-transaction tile, then the ensemble epilogue (ensemble_predictor.py:185-369: clamp,
// confidence, weighted / voting / stacking blend, decision, risk), in one launch — instead of a forest
// kernel per model (each binning the same vectors in its own prologue) plus a blend kernel.
//
// Joint repack (host, cached per pair of loaded forests): both forests padded to one depth D <= 8 and their
// node words rewritten against the MERGED per-feature table of distinct thresholds (union of the two), so
// one bin word per (feature, transaction) serves both: "x < t" is "bin_merged(x) <= index of t in the
// merged table" for every threshold of either forest. Leaf ids are not produced on this path (the per-model
// kernels keep the leaf-id outputs).
//
// Kernel: 1024 threads = 16 waves per tile (tree group gg = wave >> 2, transaction group wave & 3). Prologue:
// each thread loads 16 features of its row into registers; the merged table is staged in LDS in feature
// ranges (passes) that fit the chunk buffers + leaf-index tiles (dead until chunk 0 is staged) and every
// value is binned into the u16 tile (two features per 1 KiB row, 32 KiB for 64 features). Then the chunk
// stream is XGBoost's 24-tree chunks followed by the IsolationForest's 16-tree chunks (the compact layout: 20 /
// 12, see EnsCfg) (1 KiB node block per tree + the chunk's leaf values, double-buffered by LDS-DMA); per chunk
// each wave walks its TPG trees (6 / 4; 5 / 3) for its 64 transactions (walk_ens: 4 VALU + 2 LDS reads per node
// step) and stores the packed leaf
// indices to the chunk's index tile; the owner tree group (0) then adds each transaction's leaf values of
// that chunk, read from LDS, in tree order into the f32 margin (XGBoost) or the f64 path-length sum
// (IsolationForest): both the reference's sequential sums, bit for bit. Epilogue (tree group 0, one thread
// per transaction): sigmoid / IsolationForest transform, blend_row, outputs (columns, or the 24-B route
// result records of the owner GPU).
#include <algorithm>
#include <atomic>
#include <cstring>

#include "blend_row.h"
#include "walk_common.h"

namespace fd {

static std::atomic<uint64_t> g_forest_gen{0};

void forest_loaded(PackedForest& pf, const fd_forest_params& p, const fd_tree_arrays& t) {
  pf.gen = ++g_forest_gen;
  pf.params = p;
  const int64_t m = t.tree_offsets[t.n_trees];
  pf.t_off.assign(t.tree_offsets, t.tree_offsets + t.n_trees + 1);
  pf.t_left.assign(t.left, t.left + m);
  pf.t_right.assign(t.right, t.right + m);
  pf.t_feature.assign(t.feature, t.feature + m);
  pf.t_threshold.assign(t.threshold, t.threshold + m);
  pf.t_leaf.assign(t.leaf_value, t.leaf_value + m);
  if (t.default_left)
    pf.t_dleft.assign(t.default_left, t.default_left + m);
  else
    pf.t_dleft.assign((size_t)m, 0);
}

namespace {

constexpr int kEnsWG = 1024;
constexpr int kMaxPass = 64;

// Trees per chunk, by layout: wide 24 XGBoost (TPG 6) / 16 IsolationForest (TPG 4) trees in 48 KiB chunk
// buffers; compact 20 (TPG 5) / 12 (TPG 3) in 40 KiB, which leaves the CU the ~20 KiB of LDS an RCCL kernel
// needs beside the scoring (the sharded step's exchanges co-run with it: with the wide layout they waited for a
// whole scoring launch to end). A chunk in LDS: CH node blocks of 1 KiB (walk_ens link addressing), then the CH
// trees' leaf values [CH][2^D]; its buffer is sized for depth 8: max(CHA x (1 KiB + 1 KiB f32), CHB x (1 KiB +
// 2 KiB f64)).
template <bool WIDE>
struct EnsCfg {
  static constexpr int CHA = WIDE ? 24 : 20;
  static constexpr int CHB = WIDE ? 16 : 12;
  static constexpr uint32_t BUF = (uint32_t)(CHA * (1024 + 256 * 4) > CHB * (1024 + 256 * 8) ? CHA * (1024 + 256 * 4)
                                                                                             : CHB * (1024 + 256 * 8));
};
inline uint32_t ens_buf(bool wide) { return wide ? EnsCfg<true>::BUF : EnsCfg<false>::BUF; }
constexpr uint32_t kEnsTile = 4u * kTile * 8u;  // leaf indices of one chunk: [tree group][txn] u64, a byte per tree

// The bin tile: u16 bins, two features per 1 KiB row — feature f of transaction t at byte
// (f >> 1) * 1024 + 4 t + 2 (f & 1) — so a node word's bits [15:10] = f >> 1 and bit 1 = f & 1 address it
// with one AND-OR, and the 64 lanes of a read hit 64 distinct banks whatever features they ask for.
__host__ __device__ constexpr uint32_t ens_xs_bytes(int nf) { return (uint32_t)((nf + 1) / 2) * 1024u; }

// LDS bytes of the kernel: Xs | bufA | bufB | tile0 | tile1 | accA (f32) | accB (f64) | flags + owner counter,
// + 1 KiB alignment
size_t ens_lds(int nf, bool wide) {
  return (size_t)ens_xs_bytes(nf) + 2 * (size_t)ens_buf(wide) + 2 * (size_t)kEnsTile + kTile * 4 + kTile * 8 + 128 +
         1024;
}

struct EnsArgs {
  // Field order: what a wave reads before its first LDS-DMA goes out (rows, pass 0's table image, chunk 0) and the
  // other scalars first, packed into the first few 64-B scalar-cache lines; the per-feature / per-pass tables after
  // them (round 6: the prologue's kernel-argument round trips)
  const float* X;
  int64_t n;
  int ld, nf;
  const float* thr;
  int vec4;                       // rows 16-B aligned (ld % 4 == 0, aligned X): float4 row loads
  int compact;                    // 1: X rows are the compact 64-B rows (fd_internal.h), binned here; 2: split rows
                                  // (RowA [n] at X, RowB [n] after it, 32 B each: features.hip, load_split)
  int owner_fixed;                // chunk owner: tree group 0 (the oldest waves: highest issue priority), else rotating
  int prio;                       // issue priority 2 above the co-running feature kernels (engine option ensemble_prio)
  int n_pass;
  int pad0;
  unsigned long long pass_global;  // bit p: pass p bins from global memory (its table does not fit LDS)
  const char* img;                 // the passes' padded table images (thr_pad layout), 1 KiB pieces
  const char* nodes[2];
  int n_chunks[2];
  int stride[2];
  float base_margin;
  int pad1;
  double if_offset, if_denom;
  int pos[2];   // blend position (present-model order) of forest A / B
  int mcol[2];  // model-probability column (caller's model index) of forest A / B
  double* mp;
  double* fp;
  double* conf;
  uint8_t* dec;
  uint8_t* risk;
  const RouteRecord* rec;
  ResultRecord* res;
  int pass_f[kMaxPass + 1];
  int img_off[kMaxPass + 1];       // pass p's image: bytes [img_off[p], img_off[p + 1]) of img
  int thr_off[kMaxFeatures + 1];  // per-feature table offsets into thr (kernel arguments: scalar loads)
  uint16_t cbin[kMaxFeatures];    // compact mode: the bins of the constant slots (0 or 0.5), per plan
  alignas(4) uint16_t lut[8 * 32];  // compact mode: [kIntSlots][kLutN] bins of the small-integer slots' values 0..31
  BlendConsts blend;
#ifdef FD_FOREST_PROFILE
  int prof_slot;  // which of the kEprofSlots profile buffers this launch writes (launch count mod kEprofSlots)
  int clk_slot;   // this launch's record in g_eclk (launch count mod kEclkSlots)
#endif
};

// Ensemble node word: j << 16 | (feature >> 1) << 10 | link << 3 | (feature & 1) << 1 | default_left. `link`
// makes the next pair address one AND-OR: for a node at heap slot i above the last split level, link = i (its
// children pair is at byte 8 i of the tree's 1 KiB block); at the last split level link = i - 2^(D-1), so the
// leaf is 2 link + right. One step is then v_cmp (u16 bin against the word's high half: SDWA) + v_cndmask
// (child) + v_and_or (bin address) + v_and_or (pair address): 4 VALU, 2 LDS reads.
constexpr uint32_t kLinkMask = 0x3F8u;

template <int D, int TPG, bool NAN_AWARE>
__device__ __forceinline__ void walk_ens(uint32_t buf, int t0, uint32_t lane4, uint32_t (&leaf)[TPG]) {
  uint32_t tb[TPG], node[TPG], kl[TPG], kr[TPG], xw[TPG];
#pragma unroll
  for (int j = 0; j < TPG; ++j) {
    tb[j] = buf + (uint32_t)(t0 + j) * 1024u;  // 1 KiB aligned: the link OR is exact
    // in a VGPR: v_and_or_b32 takes one scalar operand on gfx9 (the mask literal), else it splits in two
    asm volatile("" : "+v"(tb[j]));
    node[j] = lds_load<uint32_t>(tb[j] + 4u);
  }
#pragma unroll
  for (int j = 0; j < TPG; ++j) {
    xw[j] = lds_load<uint16_t>((node[j] & 0xFC02u) | lane4);
    if (D > 1) {
      const u32x2 k = lds_load<u32x2>(tb[j] + 8u);
      kl[j] = k.x;
      kr[j] = k.y;
    }
  }
#pragma unroll
  for (int l = 0; l < D; ++l) {
#pragma unroll
    for (int j = 0; j < TPG; ++j) {
      bool right = xw[j] > (node[j] >> 16);  // bin > j  <=>  !(x < t_j)
      if (NAN_AWARE) {
        if (xw[j] == 0xFFFFu) right = (node[j] & 1u) == 0u;  // missing: default direction
      }
      if (l + 1 < D) {
        uint32_t a = kl[j], b = kr[j];
        asm volatile("" : "+v"(a), "+v"(b));
        node[j] = right ? b : a;
        xw[j] = lds_load<uint16_t>((node[j] & 0xFC02u) | lane4);
        if (l + 2 < D) {
          const u32x2 k = lds_load<u32x2>((node[j] & kLinkMask) | tb[j]);
          kl[j] = k.x;
          kr[j] = k.y;
        }
      } else {
        leaf[j] = ((node[j] & kLinkMask) >> 2) + (right ? 1u : 0u);
      }
    }
  }
}

// Walk this wave's TPG trees of the chunk at `cur` (trees gg*TPG ...) for its 64 transactions; the leaf
// indices (< 2^D <= 256) packed a byte per tree, in tree order, stored as one u64 per (tree group, txn).
// (Measured: byte-per-tree stores of a [txn][16] tile cost ~5 us more per 64k batch; skewing the split
// towards tree group 0 was slower still.)
template <int D, int TPG>
__device__ __forceinline__ unsigned long long walk_pack(uint32_t cur, int gg, uint32_t lane4, bool tile_nan) {
  static_assert(TPG <= 8, "a byte per tree in a u64");
  uint32_t leaf[TPG];
  if (tile_nan)
    walk_ens<D, TPG, true>(cur, gg * TPG, lane4, leaf);
  else
    walk_ens<D, TPG, false>(cur, gg * TPG, lane4, leaf);
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int j = 0; j < TPG; ++j) {
    if (j < 4) lo |= leaf[j] << (8 * j);
    else hi |= leaf[j] << (8 * (j - 4));
  }
  return ((unsigned long long)hi << 32) | lo;
}

// One transaction's share of a finished chunk: its CH leaf values (indices from the tile, values from the
// chunk's leaf block in LDS) added in tree order to the forest's running sum — the reference's sequential
// f32 margin / f64 path-length sum, bit for bit.
template <int D, int TPG, int CH, typename LeafT>
__device__ __forceinline__ void owner_sum(uint32_t buf, uint32_t tile, uint32_t acc, int txn) {
  constexpr int NL = 1 << D;
  unsigned long long w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) w[q] = lds_load<unsigned long long>(tile + (uint32_t)(q * kTile + txn) * 8u);
  LeafT v[CH];
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    const uint32_t idx = (uint32_t)(w[t / TPG] >> (8 * (t % TPG))) & 0xFFu;
    v[t] = lds_load<LeafT>(buf + (uint32_t)(CH * 1024) + ((uint32_t)(t * NL) + idx) * (uint32_t)sizeof(LeafT));
  }
  LeafT s = lds_load<LeafT>(acc + (uint32_t)txn * (uint32_t)sizeof(LeafT));
#pragma unroll
  for (int t = 0; t < CH; ++t) s += v[t];
  lds_store<LeafT>(acc + (uint32_t)txn * (uint32_t)sizeof(LeafT), s);
}

// LDS-DMA of `bytes` (a multiple of 1 KiB) by nparts waves (this one: part), 1 KiB pieces dealt round-robin;
// completed by dma_wait() in the issuing waves (measured: the piece order rotated by workgroup, so that the CUs
// staging the same tables and chunks at once spread over the L2 channels, changed nothing)
__device__ __forceinline__ void stage_pieces(const char* __restrict__ src, uint32_t dst, int bytes, int nparts,
                                             int part) {
  const int lane = threadIdx.x & 63;
  const int pieces = bytes >> 10;
  for (int p = part; p < pieces; p += nparts) {
    const char* g = src + (p << 10) + lane * 16;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(dst + ((uint32_t)p << 10));
    asm volatile(
        "s_mov_b32 m0, %0\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off"
        :
        : "s"(m0), "v"(g)
        : "memory", "m0");
  }
}

// Staged threshold tables hold element g at word g + g / 32: the binary search's power-of-two strides would
// otherwise put every lane of a step on one LDS bank (up to 32-way conflicts); one pad word per 32 spreads them.
__host__ __device__ __forceinline__ int thr_pad(int g) { return g + (g >> 5); }

#ifdef FD_FOREST_PROFILE
// per (workgroup < 256, wave): cycles in prologue, loop top (leaf stores, DMA issue, owner add), walk + leaf
// loads, DMA wait + barrier, epilogue (s_memtime; read by fd_debug_ens_profile)
constexpr int kEprofSlots = 4;  // the last 4 launches (the pipelined stream: launches beside the next features)
__device__ unsigned long long g_eprof[kEprofSlots * 256 * 16 * 16];
static int g_eprof_next = 0;
// per launch, the clocks of wave 0 of workgroups 0, 64, 128, 192: {s_memtime start, end, s_memrealtime start, end}
// (shader clock = memtime cycles / realtime ticks x 100 MHz; tools/clock_ramp.py)
constexpr int kEclkSlots = 1024;
__device__ unsigned long long g_eclk[kEclkSlots * 4 * 4];
static int g_eclk_next = 0;
#define FD_ESTAMP(var) const unsigned long long var = __builtin_amdgcn_s_memtime()
#else
#define FD_ESTAMP(var)
#endif

// bin = #{t <= v} by binary lifting, as bin_of, for L values in lockstep: branch-free (clamped index + select), so
// the L reads of a step issue back to back; tables staged in LDS at tl (element g at thr_pad(g)) or, glob, in global
template <int L>
__device__ __forceinline__ void search_lockstep(const float (&vv)[L], const int (&o)[L], const int (&cnt)[L],
                                                int (&pos)[L], int steps, bool glob, uint32_t tl, int o0,
                                                const float* __restrict__ thr) {
  if (!glob) {
    for (int st = steps; st > 0; st >>= 1) {
      float t[L];
#pragma unroll
      for (int k = 0; k < L; ++k) {
        const int np = pos[k] + st;
        const int idx = np <= cnt[k] ? np - 1 : 0;
        t[k] = lds_load<float>(tl + (uint32_t)thr_pad(o[k] - o0 + idx) * 4u);
      }
#pragma unroll
      for (int k = 0; k < L; ++k) {
        const int np = pos[k] + st;
        pos[k] = (np <= cnt[k] && t[k] <= vv[k]) ? np : pos[k];
      }
    }
  } else {
    for (int st = steps; st > 0; st >>= 1) {
      float t[L];
#pragma unroll
      for (int k = 0; k < L; ++k) {
        const int np = pos[k] + st;
        t[k] = thr[o[k] + (np <= cnt[k] ? np - 1 : 0)];
      }
#pragma unroll
      for (int k = 0; k < L; ++k) {
        const int np = pos[k] + st;
        pos[k] = (np <= cnt[k] && t[k] <= vv[k]) ? np : pos[k];
      }
    }
  }
}

// Compact rows (the pipeline): the 42 constant slots' bins are the plan's (a.cbin), written without a search —
// thread Q of a transaction writes the bin-tile dwords (feature pairs) Q, Q + 4, ... — and the 22 varying slots are
// dealt round-robin to the four threads of the transaction (compact slots Q, Q + 4, ...: 6, 6, 5, 5 searches instead
// of up to 16 per thread over the 64-wide row)
template <int Q>
__device__ __forceinline__ void bin_compact_constants(const EnsArgs& a, uint16_t* Xs, int txn) {
  uint32_t* X32 = reinterpret_cast<uint32_t*>(Xs);
#pragma unroll
  for (int j = Q; j < kMaxFeatures / 2; j += 4) {
    const int f = 2 * j;
    const bool c0 = compact_src(f) < 0 && f < a.nf, c1 = compact_src(f + 1) < 0 && f + 1 < a.nf;
    if (c0 && c1)
      X32[j * 256 + txn] = (uint32_t)a.cbin[f] | ((uint32_t)a.cbin[f + 1] << 16);
    else if (c0)
      Xs[j * 512 + txn * 2] = a.cbin[f];
    else if (c1)
      Xs[j * 512 + txn * 2 + 1] = a.cbin[f + 1];
  }
}

// The compact slots whose values are always small integers — hour, day of week, weekend, the 1 h / 24 h / 5 min
// counts and the account age (each clip10 of an integer), the new-device flag (features.hip write_vector) — are
// binned by one lookup in a per-plan table of the bins of 0..31 (staged in LDS), not searched: each thread keeps 3-4
// searches of its 5-6 (one lockstep group instead of two). A value outside 0..31 or not integral (never, from the
// engine's own feature kernel) takes its own search, so the bins stay #{t <= v} for any input.
constexpr int kLutN = 32;  // (kIntSlots, kIntCompact, int_slot: fd_internal.h, the compact row's byte slots)
static_assert(kIntSlots * kLutN == 8 * 32, "EnsArgs::lut");
// thread Q's compact indices Q + 4 i: the LUT row of each small-integer one (-1: searched), and the searched i's
constexpr int kIntOf[4][6] = {{-1, 2, -1, 6, -1, -1}, {-1, 3, 5, -1, -1, -1}, {0, 4, -1, -1, -1, -1},
                              {1, -1, -1, 7, -1, -1}};
constexpr int kNSearched[4] = {4, 4, 3, 3};
constexpr int kSearched[4][4] = {{0, 2, 4, 5}, {0, 3, 4, 5}, {2, 3, 4, 0}, {1, 2, 4, 0}};
constexpr bool int_tables_agree() {
  for (int q = 0; q < 4; ++q) {
    int ns = 0;
    for (int i = 0; i < 6; ++i) {
      const int ci = q + 4 * i;
      const int want = ci < kCompactSlots ? int_slot(ci) : -1;
      if (kIntOf[q][i] != want) return false;
      if (ci < kCompactSlots && want < 0) {
        if (ns >= 4 || kSearched[q][ns] != i) return false;
        ++ns;
      }
    }
    if (ns != kNSearched[q]) return false;
  }
  return true;
}
static_assert(int_tables_agree(), "kIntOf / kSearched must follow kIntCompact and kCompactSlot");

// thread Q's share of a compact row (fd_internal.h: 14 f32 words, then 8 byte slots): compact slots Q, Q + 4, ...
// into v[0..5], the byte slots as the f32 of their integer (exactly the value the feature kernel computed)
template <int Q>
__device__ __forceinline__ void load_compact(const float* __restrict__ xr, float (&v)[16]) {
  const unsigned long long ib = *reinterpret_cast<const unsigned long long*>(xr + 14);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int ci = Q + 4 * i;
    if (ci >= kCompactSlots) {
      v[i] = 0.f;
    } else if (int_slot(ci) >= 0) {
      v[i] = (float)(unsigned)((ib >> (8 * int_slot(ci))) & 0xFFull);
    } else {
      v[i] = xr[compact_word(ci)];
    }
  }
}

// Split rows (features.hip Prep32 / RowA / RowB): thread Q's compact slots Q, Q + 4, ... from the slot pass's RowA
// (card-independent) and the bucket pass's RowB (card-dependent). The derived features' positions 41..46 follow
// FeatureProcessor's conditional order (feature_processor.py:330-363, write_vector): [amount_sqrt if amount > 0,
// amount / user average if that average > 0, hourly velocity ratio if the 24 h count > 0, combined device-IP risk,
// business hours, late night], the k-th present one at 41 + k, zero after. The values are RowA / RowB's f32 as stored.
template <int Q>
__device__ __forceinline__ void load_split(const uint4* __restrict__ ra, const uint4* __restrict__ rb,
                                           float (&v)[16]) {
  const uint4 a0 = ra[0], a1 = ra[1], b0 = rb[0], b1 = rb[1];
  const unsigned fa = a1.w >> 24;                   // RowA flags
  const int na = (fa & 1u) ? 1 : 0;                 // amount > 0
  const int nu = ((b1.z >> 8) & 1u) ? 1 : 0;        // user average > 0
  const int nc = ((b1.y >> 8) & 0xFFu) ? 1 : 0;     // 24 h count > 0 (its byte: clip10 of an integer)
  const int n2 = na + nu + nc;
  auto byte = [](unsigned w, int k) { return (float)((w >> (8 * k)) & 0xFFu); };
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int ci = Q + 4 * i;
    float x = 0.f;
    switch (ci) {  // compile-time per unrolled i (fd_internal.h kCompactSlot order)
      case 0: x = __uint_as_float(a0.x); break;   // 0 amount
      case 1: x = __uint_as_float(a0.y); break;   // 1 amount_log
      case 2: x = byte(a1.w, 0); break;           // 5 hour
      case 3: x = byte(a1.w, 1); break;           // 6 day of week
      case 4: x = byte(a1.w, 2); break;           // 7 weekend
      case 5: x = byte(b1.y, 0); break;           // 14 1 h count
      case 6: x = byte(b1.y, 1); break;           // 15 24 h count
      case 7: x = __uint_as_float(b0.x); break;   // 16 24 h amount
      case 8: x = __uint_as_float(b0.y); break;   // 17 user average
      case 9: x = byte(b1.y, 2); break;           // 19 account age
      case 10: x = __uint_as_float(a0.w); break;  // 21 merchant fraud rate
      case 11: x = __uint_as_float(a1.x); break;  // 23 merchant risk
      case 12: x = byte(b1.y, 3); break;          // 26 new device
      case 13: x = __uint_as_float(a1.y); break;  // 27 IP risk
      case 14: x = __uint_as_float(b0.z); break;  // 31 1 h amount
      case 15: x = byte(b1.z, 0); break;          // 32 5 min count
      default:
        if (ci < kCompactSlots) {  // 41 + k: the k-th present derived feature
          const int k = ci - 16;
          const float first = (na && k == 0) ? __uint_as_float(a0.z)
                                             : ((nu && k == na) ? __uint_as_float(b0.w) : __uint_as_float(b1.x));
          const int t = k - n2;  // past the conditional three: combined risk, business, late night
          x = k < n2 ? first
                     : (t == 0 ? __uint_as_float(a1.z)
                               : (t == 1 ? ((fa & 2u) ? 1.f : 0.f) : (t == 2 ? ((fa & 4u) ? 1.f : 0.f) : 0.f)));
        }
        break;
    }
    v[i] = x;
  }
}

template <int Q, int L, bool LUT>
__device__ __forceinline__ void bin_compact_pass(const EnsArgs& a, const float (&v)[16], uint16_t* Xs,
                                                 int txn, int f0, int f1, bool glob, uint32_t tl, int o0,
                                                 int& anynan, uint32_t lut) {
  constexpr int NV = (kCompactSlots - Q + 3) / 4;  // compact slots Q, Q + 4, ... below kCompactSlots
  constexpr int NS = LUT ? kNSearched[Q] : NV;
  // the small-integer slots: one LDS lookup each
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int ks = LUT ? kIntOf[Q][i] : -1;
    if (ks < 0) continue;
    const int f = kCompactSlot[Q + 4 * i];
    if (!(f >= f0 && f < f1 && f < a.nf)) continue;  // wave-uniform
    const float x = v[i];
    uint16_t bin;
    if (x != x) {
      anynan = 1;
      bin = (uint16_t)0xFFFFu;
    } else if (x >= 0.f && x < (float)kLutN && x == truncf(x)) {
      bin = lds_load<uint16_t>(lut + (uint32_t)(ks * kLutN + (int)x) * 2u);
    } else {  // #{t <= x} over the feature's merged table in global memory: binary lifting with a fixed trip count
      // (tables hold < 2^16 thresholds), straight-line code, so this loop over i stays unrolled and v[] in registers
      const int o = a.thr_off[f], cnt = a.thr_off[f + 1] - o;
      int pos = 0;
#pragma unroll
      for (int st = 1 << 15; st > 0; st >>= 1)
        if (pos + st <= cnt && a.thr[o + pos + st - 1] <= x) pos += st;
      bin = (uint16_t)pos;
    }
    Xs[(f >> 1) * 512 + txn * 2 + (f & 1)] = bin;
  }
  // the others: binary lifting in lockstep groups of L
#pragma unroll
  for (int g0 = 0; g0 < NS; g0 += L) {
    float vv[L];
    int o[L], cnt[L], pos[L];
    bool act[L];
    int steps = 0;
#pragma unroll
    for (int k = 0; k < L; ++k) {
      const int i = LUT ? kSearched[Q][g0 + k < NS ? g0 + k : 0] : (g0 + k < NS ? g0 + k : 0);
      const int f = kCompactSlot[Q + 4 * i];
      act[k] = g0 + k < NS && f >= f0 && f < f1 && f < a.nf;
      vv[k] = act[k] ? v[i] : 0.f;  // v[i]: compact slot Q + 4 i of the row
      o[k] = act[k] ? a.thr_off[f] : o0;
      cnt[k] = act[k] ? a.thr_off[f + 1] - o[k] : 0;
      pos[k] = 0;
      steps = max(steps, lift_steps(cnt[k]));
    }
    search_lockstep<L>(vv, o, cnt, pos, steps, glob, tl, o0, a.thr);
#pragma unroll
    for (int k = 0; k < L; ++k) {
      const int i = LUT ? kSearched[Q][g0 + k < NS ? g0 + k : 0] : (g0 + k < NS ? g0 + k : 0);
      const int f = kCompactSlot[Q + 4 * i];
      if (act[k]) {
        const bool nan = vv[k] != vv[k];
        anynan |= nan ? 1 : 0;
        Xs[(f >> 1) * 512 + txn * 2 + (f & 1)] = nan ? (uint16_t)0xFFFFu : (uint16_t)pos[k];
      }
    }
  }
}

template <int D, int OUT, bool WIDE, bool LUT = true>
__global__ void __launch_bounds__(kEnsWG) ensemble_kernel(EnsArgs a) {
  constexpr int kCHA = EnsCfg<WIDE>::CHA, kCHB = EnsCfg<WIDE>::CHB;
  constexpr uint32_t kEnsBuf = EnsCfg<WIDE>::BUF;
  constexpr int TPGA = kCHA / 4, TPGB = kCHB / 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t sdyn = (uint32_t)(size_t)((lds_char*)smem);
  const uint32_t s0 = (sdyn + 1023u) & ~1023u;
  char* const lbase = smem + (s0 - sdyn);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int gg = __builtin_amdgcn_readfirstlane(wave >> 2);  // wave-uniform: scalar addressing
  const int txn = ((wave & 3) << 6) + lane;
  const uint32_t lane4 = s0 + (uint32_t)txn * 4u;
  const uint32_t bufA = s0 + ens_xs_bytes(a.nf), bufB = bufA + kEnsBuf;
  const uint32_t tile0 = bufB + kEnsBuf, tile1 = tile0 + kEnsTile;
  const uint32_t accA = tile1 + kEnsTile, accB = accA + kTile * 4;
  const uint32_t flags = accB + kTile * 8, owner_cnt = flags + 64;
  const int64_t row = (int64_t)blockIdx.x * kTile + txn;
  const bool valid = row < a.n;
  const int nA = a.n_chunks[0], G = nA + a.n_chunks[1];

#ifdef FD_FOREST_PROFILE
  unsigned long long pr_top = 0, pr_walk = 0, pr_sync = 0, pr_dma = 0, pr_st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  FD_ESTAMP(pr_t0);
#ifdef FD_FOREST_PROFILE
  const unsigned long long pr_rt0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz, one clock for the whole GPU
#endif
  // every kernel argument the prologue branches on or addresses with, in ONE round of scalar loads: left to itself
  // the compiler issues them lazily, one dependent kernel-argument round trip per branch (five before the row loads
  // went out). The empty asm needs them all in SGPRs at this point; later reads of the same fields reuse them.
  {
    const int k_prio = a.prio, k_compact = a.compact, k_npass = a.n_pass, k_vec4 = a.vec4, k_ld = a.ld;
    const unsigned long long k_pg = a.pass_global;
    const float* k_x = a.X;
    const char* k_img = a.img;
    const int k_i0 = a.img_off[0], k_i1 = a.img_off[1], k_f1 = a.pass_f[1];
    asm volatile("" ::"s"(k_prio), "s"(k_compact), "s"(k_npass), "s"(k_vec4), "s"(k_ld), "s"(k_pg), "s"(k_x),
                 "s"(k_img), "s"(k_i0), "s"(k_i1), "s"(k_f1), "s"(nA), "s"(G), "s"(a.n));
  }
  // above the feature kernels of the next micro-batch that share the CU in the pipelined stream (priority 0):
  // this kernel is the stream's critical path, theirs is latency-bound with slack
  if (a.prio) __builtin_amdgcn_s_setprio(2);
  int anynan = 0;
  const bool early0 = G > 0 && a.n_pass == 1 && (a.pass_global & 1ull) != 0;
  {
    uint16_t* Xs = reinterpret_cast<uint16_t*>(lbase);
    const int q = __builtin_amdgcn_readfirstlane(tid >> 8);  // wave-uniform: the four threads sharing `txn`
    const int fq = q * 16;
    // (1) raw values: thread (q, txn) loads features [16 q, 16 q + 16) of its row in one go (all loads in
    // flight together) and keeps them in registers until they are binned
    // compact mode: thread q's share of the pipeline's compact row, slots q, q + 4, ... (6, 6, 5, 5 of the 22) in
    // v[0..5] — the same registers as the full row's 16 (one value array live through the passes, not two: 54
    // VGPRs, the bucket kernel's wave fits beside the ensemble's four per SIMD); the constant slots' bins straight
    // away
    float v[16];
    if (valid && a.compact == 2) {  // split rows: RowA [n], then RowB [n]
      const uint4* ra = reinterpret_cast<const uint4*>(a.X) + 2 * row;
      const uint4* rb = reinterpret_cast<const uint4*>(a.X) + 2 * (a.n + row);
      switch (q) {  // wave-uniform
        case 0: load_split<0>(ra, rb, v); bin_compact_constants<0>(a, Xs, txn); break;
        case 1: load_split<1>(ra, rb, v); bin_compact_constants<1>(a, Xs, txn); break;
        case 2: load_split<2>(ra, rb, v); bin_compact_constants<2>(a, Xs, txn); break;
        default: load_split<3>(ra, rb, v); bin_compact_constants<3>(a, Xs, txn); break;
      }
    } else if (valid && a.compact) {
      const float* xr = a.X + row * (int64_t)kCompactWidth;
      switch (q) {  // wave-uniform
        case 0: load_compact<0>(xr, v); bin_compact_constants<0>(a, Xs, txn); break;
        case 1: load_compact<1>(xr, v); bin_compact_constants<1>(a, Xs, txn); break;
        case 2: load_compact<2>(xr, v); bin_compact_constants<2>(a, Xs, txn); break;
        default: load_compact<3>(xr, v); bin_compact_constants<3>(a, Xs, txn); break;
      }
    } else if (valid) {
      const float* xr = a.X + row * (int64_t)a.ld;
      const int ncopy = a.ld < a.nf ? a.ld : a.nf;
      if (a.vec4 && fq + 16 <= ncopy) {
        const float4* x4 = reinterpret_cast<const float4*>(xr + fq);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float4 t = x4[k];
          v[4 * k] = t.x;
          v[4 * k + 1] = t.y;
          v[4 * k + 2] = t.z;
          v[4 * k + 3] = t.w;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = fq + k < ncopy ? xr[fq + k] : __builtin_nanf("");  // missing: NaN
      }
    }
    // pass 0's table image goes out by LDS-DMA now, beside the row loads (it lands while they are in flight); every
    // search in global memory instead (engine option ensemble_bin_global): nothing staged, so chunk 0's DMA goes out
    if (a.n_pass > 0 && !(a.pass_global & 1ull))
      stage_pieces(a.img + a.img_off[0], bufA, a.img_off[1] - a.img_off[0], kEnsWG / 64, wave);
    if (early0) stage_chunk_asm(nA > 0 ? a.nodes[0] : a.nodes[1], bufA, nA > 0 ? a.stride[0] : a.stride[1], kEnsWG / 64);
#ifdef FD_FOREST_PROFILE
    pr_st[0] = __builtin_amdgcn_s_memtime();
#endif
    // compact mode: the small-integer slots' bin table into the accumulator area (unused until the chunk loop)
    // (published by the first pass's staging barrier: no barrier of its own)
    if (LUT && a.compact && tid < kIntSlots * kLutN / 2)
      lds_store<uint32_t>(accA + (uint32_t)tid * 4u, reinterpret_cast<const uint32_t*>(a.lut)[tid]);
    // (2) per pass: stage its tables, then bin this thread's features of the pass kLock at a time (independent
    // searches in lockstep, so kLock LDS reads are in flight per step) into the u16 tile
    constexpr int kLock = 4;  // 8 measured slower (bank conflicts of the diverging searches, not latency)
    for (int p = 0; p < a.n_pass; ++p) {
      const int f0 = a.pass_f[p], f1 = a.pass_f[p + 1];
      const bool glob = (a.pass_global >> p) & 1ull;
      const int o0 = a.thr_off[f0];
      const uint32_t tl = bufA;  // this pass's tables: bufA + bufB + the tiles (free until chunk 0 is staged)
      if (!glob) {  // the pass's image (element g at word g + g / 32, thr_pad) in LDS: DMA, then publish
        if (p > 0)
          stage_pieces(a.img + a.img_off[p], bufA, a.img_off[p + 1] - a.img_off[p], kEnsWG / 64, wave);
        dma_wait();
        __syncthreads();
      } else if (LUT && a.compact && p == 0) {
        __syncthreads();  // the small-integer table
      }
#ifdef FD_FOREST_PROFILE
      if (p < 3) pr_st[1 + 2 * p] = __builtin_amdgcn_s_memtime();
#endif
      if (LUT && valid && a.compact) {
        switch (q) {
          case 0: bin_compact_pass<0, kLock, true>(a, v, Xs, txn, f0, f1, glob, tl, o0, anynan, accA); break;
          case 1: bin_compact_pass<1, kLock, true>(a, v, Xs, txn, f0, f1, glob, tl, o0, anynan, accA); break;
          case 2: bin_compact_pass<2, kLock, true>(a, v, Xs, txn, f0, f1, glob, tl, o0, anynan, accA); break;
          default: bin_compact_pass<3, kLock, true>(a, v, Xs, txn, f0, f1, glob, tl, o0, anynan, accA); break;
        }
      } else if (valid && a.compact) {
        switch (q) {
          case 0: bin_compact_pass<0, kLock, false>(a, v, Xs, txn, f0, f1, glob, tl, o0, anynan, accA); break;
          case 1: bin_compact_pass<1, kLock, false>(a, v, Xs, txn, f0, f1, glob, tl, o0, anynan, accA); break;
          case 2: bin_compact_pass<2, kLock, false>(a, v, Xs, txn, f0, f1, glob, tl, o0, anynan, accA); break;
          default: bin_compact_pass<3, kLock, false>(a, v, Xs, txn, f0, f1, glob, tl, o0, anynan, accA); break;
        }
      } else if (valid) {
#pragma unroll
        for (int kk = 0; kk < 16; kk += kLock) {
          const int fb = fq + kk;
          if (fb + kLock - 1 < f0 || fb >= f1) continue;  // wave-uniform
          float vv[kLock];
          int o[kLock], cnt[kLock], pos[kLock];
          bool act[kLock];
          int steps = 0;
#pragma unroll
          for (int k = 0; k < kLock; ++k) {
            const int f = fb + k;
            act[k] = f >= f0 && f < f1;
            vv[k] = act[k] ? v[kk + k] : 0.f;
            o[k] = act[k] ? a.thr_off[f] : o0;
            cnt[k] = act[k] ? a.thr_off[f + 1] - o[k] : 0;
            pos[k] = 0;
            steps = max(steps, lift_steps(cnt[k]));
          }
          // bin = #{t <= v} by binary lifting, as bin_of; branch-free (clamped index + select), so the four
          // reads of a step issue back to back
          if (!glob) {
            for (int st = steps; st > 0; st >>= 1) {
              float t[kLock];
#pragma unroll
              for (int k = 0; k < kLock; ++k) {
                const int np = pos[k] + st;
                const int idx = np <= cnt[k] ? np - 1 : 0;
                t[k] = lds_load<float>(tl + (uint32_t)thr_pad(o[k] - o0 + idx) * 4u);
              }
#pragma unroll
              for (int k = 0; k < kLock; ++k) {
                const int np = pos[k] + st;
                pos[k] = (np <= cnt[k] && t[k] <= vv[k]) ? np : pos[k];
              }
            }
          } else {
            for (int st = steps; st > 0; st >>= 1) {
              float t[kLock];
#pragma unroll
              for (int k = 0; k < kLock; ++k) {
                const int np = pos[k] + st;
                t[k] = a.thr[o[k] + (np <= cnt[k] ? np - 1 : 0)];
              }
#pragma unroll
              for (int k = 0; k < kLock; ++k) {
                const int np = pos[k] + st;
                pos[k] = (np <= cnt[k] && t[k] <= vv[k]) ? np : pos[k];
              }
            }
          }
#pragma unroll
          for (int k = 0; k < kLock; ++k) {
            const int f = fb + k;
            if (act[k]) {
              const bool nan = vv[k] != vv[k];
              anynan |= nan ? 1 : 0;
              Xs[(f >> 1) * 512 + txn * 2 + (f & 1)] = nan ? (uint16_t)0xFFFFu : (uint16_t)pos[k];
            }
          }
        }
      }
      __syncthreads();  // the staged tables are overwritten by the next pass / chunk 1
#ifdef FD_FOREST_PROFILE
      if (p < 3) pr_st[2 + 2 * p] = __builtin_amdgcn_s_memtime();
#endif
    }
  }
  if (G > 0 && !early0)  // chunk 0 (the tables are dead): forest A's first, or B's when A is absent
    stage_pieces(nA > 0 ? a.nodes[0] : a.nodes[1], bufA, nA > 0 ? a.stride[0] : a.stride[1], kEnsWG / 64, wave);
  if (gg == 0) {
    lds_store<float>(accA + txn * 4, a.base_margin);
    lds_store<double>(accB + txn * 8, 0.0);
  }
  if (tid == 0) lds_store<uint32_t>(owner_cnt, 0u);
  dma_wait();  // chunk 0 (published by tile_any's barrier)
  const bool tile_nan = tile_any(anynan, reinterpret_cast<uint32_t*>(lbase + (flags - s0)), kEnsWG / 64);

  // Iteration g: the owner tree group (0, or (g - 1) & 3 with the rotating schedule) sums chunk g-1 (leaf indices from tile[(g-1)&1], values
  // from its LDS buffer), waits until all four of its waves are done reading that buffer (LDS counter),
  // then stages chunk g+1 into it; every wave walks chunk g and stores its packed leaf indices to
  // tile[g&1]; the owners complete their DMA; the barrier publishes chunk g+1 and tile[g&1].
  FD_ESTAMP(pr_t1);
  for (int g = 0; g < G; ++g) {
    FD_ESTAMP(q0);
    const bool owner = gg == (a.owner_fixed ? 0 : ((g - 1) & 3));
    if (owner) {
      if (g > 0) {
        const int c = g - 1;
        const uint32_t bp = (c & 1) ? bufB : bufA, tp = (c & 1) ? tile1 : tile0;
        if (c < nA) owner_sum<D, TPGA, kCHA, float>(bp, tp, accA, txn);
        else owner_sum<D, TPGB, kCHB, double>(bp, tp, accB, txn);
        // the leaf reads of all four owner waves are complete before any of them overwrites the buffer
        if (lane == 0)
          __hip_atomic_fetch_add(reinterpret_cast<uint32_t*>(lbase + (owner_cnt - s0)), 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
        while (__hip_atomic_load(reinterpret_cast<uint32_t*>(lbase + (owner_cnt - s0)), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP) < 4u * (uint32_t)g)
          __builtin_amdgcn_s_sleep(1);
      }
      if (g + 1 < G) {
        const int h = g + 1, fb = h >= nA ? 1 : 0;
        stage_pieces(a.nodes[fb] + (size_t)(fb ? h - nA : h) * a.stride[fb], (g & 1) ? bufA : bufB, a.stride[fb], 4,
                  wave & 3);
      }
    }
    const uint32_t cur = (g & 1) ? bufB : bufA, tw = (g & 1) ? tile1 : tile0;
    FD_ESTAMP(q1);
    const unsigned long long w =
        g < nA ? walk_pack<D, TPGA>(cur, gg, lane4, tile_nan) : walk_pack<D, TPGB>(cur, gg, lane4, tile_nan);
    lds_store<unsigned long long>(tw + (uint32_t)(gg * kTile + txn) * 8u, w);
    FD_ESTAMP(q2);
    if (owner) dma_wait();
#ifdef FD_FOREST_PROFILE
    const unsigned long long q2d = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();
#ifdef FD_FOREST_PROFILE
    const unsigned long long q3 = __builtin_amdgcn_s_memtime();
    pr_top += q1 - q0;
    pr_walk += q2 - q1;
    pr_dma += q2d - q2;
    pr_sync += q3 - q2;
#endif
  }
  if (G > 0 && gg == (a.owner_fixed ? 0 : ((G - 1) & 3))) {
    const int c = G - 1;
    const uint32_t bp = (c & 1) ? bufB : bufA, tp = (c & 1) ? tile1 : tile0;
    if (c < nA) owner_sum<D, TPGA, kCHA, float>(bp, tp, accA, txn);
    else owner_sum<D, TPGB, kCHB, double>(bp, tp, accB, txn);
  }
  __syncthreads();
#ifdef FD_FOREST_PROFILE
  if (lane == 0 && blockIdx.x < 256) {
    unsigned long long* o = g_eprof + (size_t)a.prof_slot * 256 * 16 * 16 + ((size_t)blockIdx.x * 16 + wave) * 16;
    for (int k = 0; k < 7; ++k) o[6 + k] = pr_st[k] ? pr_st[k] - pr_t0 : 0;
    o[0] = pr_t1 - pr_t0;
    o[1] = pr_top;
    o[2] = pr_walk;
    o[3] = pr_sync;
    o[13] = pr_dma;  // of pr_sync: the owner waves' wait for their chunk DMA (0 for the other waves)
    o[4] = pr_t0;
    o[5] = __builtin_amdgcn_s_memtime();
    o[14] = pr_rt0;
    o[15] = __builtin_amdgcn_s_memrealtime();
    if (wave == 0 && (blockIdx.x & 63) == 0) {
      unsigned long long* c = g_eclk + ((size_t)a.clk_slot * 4 + (blockIdx.x >> 6)) * 4;
      c[0] = pr_t0;
      c[1] = o[5];
      c[2] = pr_rt0;
      c[3] = o[15];
    }
  }
#endif
  if (gg != 0 || !valid) return;

  // epilogue: the two models' probabilities, then the blend (blend_row.h)
  double pa, pb;
  {
    const float mg = lds_load<float>(accA + txn * 4);  // XGBoost common::Sigmoid in f32
    const float xm = fminf(-mg, 88.7f);
    const float denom = expf(xm) + 1.0f + 1e-16f;
    pa = (double)(1.0f / denom);
  }
  {
    const double d = lds_load<double>(accB + txn * 8);  // sklearn score -> decision -> 1/(1+exp(s))
    const double qd = (a.if_denom != 0.0) ? d / a.if_denom : 1.0;
    const double score = pow(2.0, -qd);
    const double decision = -score - a.if_offset;
    pb = 1.0 / (1.0 + exp(decision));
  }
  if (OUT == 2) {  // one forest: its probability (forest_predict semantics) and, when asked, its raw score
    a.fp[row] = nA > 0 ? pa : pb;
    if (a.mp) a.mp[row] = nA > 0 ? (double)lds_load<float>(accA + txn * 4) : lds_load<double>(accB + txn * 8);
    return;
  }
  double raw[FD_MAX_MODELS];  // the two present models at their blend positions (selects: no scratch)
#pragma unroll
  for (int m = 0; m < FD_MAX_MODELS; ++m) raw[m] = m == a.pos[0] ? pa : (m == a.pos[1] ? pb : 0.0);
  if (a.mp) {
    a.mp[(size_t)a.mcol[0] * a.n + row] = pa;
    a.mp[(size_t)a.mcol[1] * a.n + row] = pb;
  }
  double fp, conf;
  uint8_t dec, risk;
  blend_row(a.blend, raw, fp, conf, dec, risk);
  if (OUT == 0) {
    a.fp[row] = fp;
    if (a.conf) a.conf[row] = conf;
    if (a.dec) a.dec[row] = dec;
    if (a.risk) a.risk[row] = risk;
  } else {
    ResultRecord r;
    r.fraud_prob = fp;
    r.confidence = conf;
    r.seq = a.rec[row].seq;
    r.decision = dec;
    r.risk = risk;
    r.pad = 0;
    a.res[row] = r;
  }
}

template <int OUT, bool WIDE>
const void* pick_ensemble(int D) {
  switch (D) {
    case 1: return (const void*)ensemble_kernel<1, OUT, WIDE>;
    case 2: return (const void*)ensemble_kernel<2, OUT, WIDE>;
    case 3: return (const void*)ensemble_kernel<3, OUT, WIDE>;
    case 4: return (const void*)ensemble_kernel<4, OUT, WIDE>;
    case 5: return (const void*)ensemble_kernel<5, OUT, WIDE>;
    case 6: return (const void*)ensemble_kernel<6, OUT, WIDE>;
    case 7: return (const void*)ensemble_kernel<7, OUT, WIDE>;
    case 8: return (const void*)ensemble_kernel<8, OUT, WIDE>;
    default: return nullptr;
  }
}

// (the instantiations without the small-integer table, round 5's A/B, were removed with the option: DESIGN §3)
const void* pick_ensemble(int out, bool wide, int D) {
  if (wide) return out == 1 ? pick_ensemble<1, true>(D) : out == 2 ? pick_ensemble<2, true>(D) : pick_ensemble<0, true>(D);
  return out == 1 ? pick_ensemble<1, false>(D) : out == 2 ? pick_ensemble<2, false>(D) : pick_ensemble<0, false>(D);
}

fd_tree_arrays arrays_of(const PackedForest& f) {
  fd_tree_arrays t{};
  t.n_trees = f.n_trees;
  t.tree_offsets = f.t_off.data();
  t.left = f.t_left.data();
  t.right = f.t_right.data();
  t.feature = f.t_feature.data();
  t.threshold = f.t_threshold.data();
  t.default_left = f.t_dleft.data();
  t.leaf_value = f.t_leaf.data();
  return t;
}

// Binning passes over the tables (thr, off): consecutive features whose padded tables fit the staging area (bufA +
// bufB + the tiles), a larger table alone, searched in global memory; each staged pass's image (element g of the
// pass at word thr_pad(g), 1 KiB pieces) appended to img
void plan_passes(const std::vector<float>& thr, const std::vector<int32_t>& off, int nf, bool wide, EnsPassSet& ps,
                 std::vector<float>& img) {
  const size_t stage_floats = (2 * (size_t)ens_buf(wide) + 2 * (size_t)kEnsTile) / 4;
  ps = EnsPassSet{};
  ps.f.push_back(0);
  ps.img_off.push_back((int)(img.size() * 4));
  int f = 0;
  while (f < nf) {
    int g = f;
    while (g < nf && (size_t)(off[g + 1] - off[f]) + (size_t)(off[g + 1] - off[f]) / 32 + 1 <= stage_floats) ++g;
    const int np = (int)ps.f.size() - 1;
    FD_REQUIRE(np < kMaxPass, FD_ERR_UNSUPPORTED, "ensemble binning plan too long");
    if (g == f) {  // one feature's table exceeds the LDS space
      ps.glob |= 1ull << np;
      g = f + 1;
    } else {
      const int cnt = off[g] - off[f];
      const size_t words = cnt > 0 ? (size_t)thr_pad(cnt - 1) + 1 : 0;
      const size_t base = img.size();
      img.resize(base + (words + 255) / 256 * 256, 0.f);
      for (int i = 0; i < cnt; ++i) img[base + (size_t)thr_pad(i)] = thr[(size_t)off[f] + i];
    }
    ps.f.push_back(g);
    ps.img_off.push_back((int)(img.size() * 4));
    f = g;
  }
}

// joint repack of forest A (XGBoost, slot sa) and B (IsolationForest, slot sb) into plan P; either slot may be -1
// (a single forest: the kernel walks only the other one); false when not possible (the per-model path runs)
bool build_plan(Engine& e, EnsemblePlan& P, int sa, int sb, bool wide) {
  P.valid = false;
  const PackedForest* F[2] = {sa >= 0 ? &e.forests[sa] : nullptr, sb >= 0 ? &e.forests[sb] : nullptr};
  if (!F[0] && !F[1]) return false;
  int D = 0, nf = -1;
  for (const PackedForest* f : F) {
    if (!f) continue;
    if (!f->binned || f->t_off.empty() || (nf >= 0 && f->num_feature != nf)) return false;
    nf = f->num_feature;
    D = std::max(D, f->depth);
  }
  if (D > 8) return false;
  if (ens_lds(nf, wide) > kLdsBudget) return false;
  HostPack hp[2];
  for (int k = 0; k < 2; ++k) {
    if (!F[k]) continue;
    hp[k] = pack_forest_host(F[k]->params, arrays_of(*F[k]), D);
    if (!hp[k].binned || hp[k].depth != D) return false;
  }
  // merged per-feature tables
  std::vector<std::vector<float>> merged(nf);
  for (int f = 0; f < nf; ++f) {
    for (int k = 0; k < 2; ++k) {
      if (!F[k]) continue;
      const HostPack& h = hp[k];
      merged[f].insert(merged[f].end(), h.b_thr.begin() + h.b_thr_off[f], h.b_thr.begin() + h.b_thr_off[f + 1]);
    }
    std::sort(merged[f].begin(), merged[f].end());
    merged[f].erase(std::unique(merged[f].begin(), merged[f].end()), merged[f].end());
    if (merged[f].size() > (size_t)kMaxBins) return false;
  }
  std::vector<float> thr;
  std::vector<int32_t> off(nf + 1, 0);
  int maxc = 0;
  for (int f = 0; f < nf; ++f) {
    thr.insert(thr.end(), merged[f].begin(), merged[f].end());
    off[f + 1] = (int32_t)thr.size();
    maxc = std::max(maxc, (int)merged[f].size());
  }
  const int NL = 1 << D;
  const int CH[2] = {wide ? EnsCfg<true>::CHA : EnsCfg<false>::CHA, wide ? EnsCfg<true>::CHB : EnsCfg<false>::CHB};
  const size_t leaf_sz[2] = {sizeof(float), sizeof(double)};
  for (int k = 0; k < 2; ++k) {
    if (!F[k]) {
      P.n_trees[k] = P.n_chunks[k] = 0;
      P.CH[k] = CH[k];
      P.stride[k] = 0;
      continue;
    }
    const HostPack& h = hp[k];
    const int T = h.n_trees, nc = (T + CH[k] - 1) / CH[k];
    // chunk: CH node blocks of 1 KiB (walk_ens link addressing), then the CH trees' leaf values [CH][NL];
    // padding trees (a partial last chunk) keep zero nodes and zero leaves
    const size_t leaf_bytes = (size_t)CH[k] * NL * leaf_sz[k];
    const size_t stride = ((size_t)CH[k] * 1024 + leaf_bytes + 1023) / 1024 * 1024;
    FD_REQUIRE(stride <= ens_buf(wide), FD_ERR_UNSUPPORTED, "ensemble chunk exceeds its LDS buffer");
    std::vector<char> blob((size_t)nc * stride, 0);
    for (int i = 0; i < T; ++i) {
      const char* src = h.b_blob.data() + (size_t)(i / h.b_chunk) * h.b_chunk_stride + (size_t)(i % h.b_chunk) *
                                                                                          h.b_tree_bytes;
      char* chunk = blob.data() + (size_t)(i / CH[k]) * stride;
      uint32_t* dst = reinterpret_cast<uint32_t*>(chunk + (size_t)(i % CH[k]) * 1024);
      for (int s = 1; s < NL; ++s) {
        uint32_t w;
        std::memcpy(&w, src + (size_t)s * 4, 4);
        const uint32_t f = (w >> 10) & 63u;
        if (!h.pad[(size_t)i * NL + s]) {  // real split: its threshold's index in the merged table
          const int j = (int)(w >> 16);
          const float t = h.b_thr[h.b_thr_off[f] + j];
          const uint32_t jm = (uint32_t)(std::lower_bound(merged[f].begin(), merged[f].end(), t) - merged[f].begin());
          w = (jm << 16) | (w & 0xFFFFu);
        }
        const uint32_t link = s < (NL >> 1) ? (uint32_t)s : (uint32_t)(s - (NL >> 1));
        // walk_ens node word: the pair-row of the u16 bin tile in bits [15:10], the feature's half in bit 1
        dst[s] = (w & 0xFFFF0001u) | ((f >> 1) << 10) | (link << 3) | ((f & 1u) << 1);
      }
      std::memcpy(chunk + (size_t)CH[k] * 1024 + (size_t)(i % CH[k]) * NL * leaf_sz[k], src + (size_t)NL * 4,
                  (size_t)NL * leaf_sz[k]);
    }
    P.nodes[k].ensure(blob.size());
    FD_HIP(hipMemcpy(P.nodes[k].ptr, blob.data(), blob.size(), hipMemcpyHostToDevice));
    P.n_trees[k] = T;
    P.CH[k] = CH[k];
    P.n_chunks[k] = nc;
    P.stride[k] = stride;
  }
  P.thr.ensure(std::max<size_t>(4, thr.size() * sizeof(float)));
  if (!thr.empty()) FD_HIP(hipMemcpy(P.thr.ptr, thr.data(), thr.size() * sizeof(float), hipMemcpyHostToDevice));
  P.h_thr_off = off;
  // the bins of the compact vector's constant slots (0 or 0.5): #{t <= value} in the feature's merged table
  P.h_cbin.assign(kMaxFeatures, 0);
  for (int f = 0; f < nf && f < kMaxFeatures; ++f) {
    const int src = compact_src(f);
    if (src >= 0) continue;
    const float val = src == -2 ? 0.5f : 0.0f;
    P.h_cbin[f] = (uint16_t)(std::upper_bound(merged[f].begin(), merged[f].end(), val) - merged[f].begin());
  }
  {  // the small-integer compact slots: bins of the values 0 .. kLutN - 1
    std::vector<uint16_t> lut((size_t)kIntSlots * kLutN, 0);
    for (int k = 0; k < kIntSlots; ++k) {
      const int f = kCompactSlot[kIntCompact[k]];
      if (f >= nf) continue;
      for (int x = 0; x < kLutN; ++x)
        lut[(size_t)k * kLutN + x] =
            (uint16_t)(std::upper_bound(merged[f].begin(), merged[f].end(), (float)x) - merged[f].begin());
    }
    P.h_lut = lut;
  }
  {  // the binning passes and their table images
    std::vector<float> img;
    plan_passes(thr, off, nf, wide, P.passes, img);
    P.img.ensure(std::max<size_t>(1024, img.size() * sizeof(float)));
    if (!img.empty()) FD_HIP(hipMemcpy(P.img.ptr, img.data(), img.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  P.max_feature_thr = maxc;
  P.slot[0] = sa;
  P.slot[1] = sb;
  P.gen[0] = F[0] ? F[0]->gen : 0;
  P.gen[1] = F[1] ? F[1]->gen : 0;
  P.n_forests = (F[0] ? 1 : 0) + (F[1] ? 1 : 0);
  P.D = D;
  P.nf = nf;
  P.wide = wide;
  P.kind[0] = FD_FOREST_XGB_BINARY_LOGISTIC;
  P.kind[1] = FD_FOREST_SKLEARN_IFOREST;
  P.base_margin = F[0] ? hp[0].base_margin : 0.f;
  P.if_offset = F[1] ? F[1]->if_offset : 0.0;
  P.if_denominator = F[1] ? F[1]->if_denominator : 0.0;
  P.valid = true;
  return true;
}

bool plan_current(const Engine& e, const EnsemblePlan& P, int sa, int sb, bool wide) {
  return P.valid && P.wide == wide && P.slot[0] == sa && P.slot[1] == sb &&
         P.gen[0] == (sa >= 0 ? e.forests[sa].gen : 0) && P.gen[1] == (sb >= 0 ? e.forests[sb].gen : 0);
}

// the chunk layout for this engine: option "ensemble_chunks" 1 wide / 2 compact, 0 (auto) compact once the engine
// has RCCL communicators (its sharded step's exchanges co-run with the scoring), else wide
bool want_wide(const Engine& e) { return e.ens_chunks == 1 || (e.ens_chunks == 0 && !e.comm.ready); }

}  // namespace

#ifdef FD_FOREST_PROFILE
// n words from the start of the buffers: slot k's profile at word k * 256 * 16 * 16; *next_slot (if given) = the slot
// the next launch writes (so the most recent launch wrote (next_slot + kEprofSlots - 1) % kEprofSlots)
extern "C" __attribute__((visibility("default"))) int fd_debug_ens_profile(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_eprof), sizeof(unsigned long long) * (size_t)n);
}
extern "C" __attribute__((visibility("default"))) int fd_debug_ens_profile_next(void) { return g_eprof_next; }
extern "C" __attribute__((visibility("default"))) int fd_debug_ens_clock(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_eclk), sizeof(unsigned long long) * (size_t)n);
}
extern "C" __attribute__((visibility("default"))) int fd_debug_ens_clock_next(void) { return g_eclk_next; }
#endif

namespace {
struct Pair {
  int sa = -1, sb = -1, pa = -1, pb = -1, ma = -1, mb = -1;
};

// The fused kernel applies (and its joint plan is built) when the batch is large and the present models are
// exactly one XGBoost and one IsolationForest in engine slots.
bool select_pair(Engine& e, const fd_blend_params& p, const int32_t* slots, const uint8_t* present, int64_t n,
                 Pair& q) {
  if (!e.ensemble_on || e.forest_variant != 0 || n <= 0) return false;
  if ((n + kTile - 1) / kTile < kSplitTiles) return false;  // latency batches: the tree-split path
  int k = 0;
  for (int m = 0; m < p.n_models; ++m) {
    if (present && !present[m]) continue;
    const int s = slots[m];
    if (s < 0 || s >= kMaxSlots || !e.forests[s].loaded) return false;
    const int kind = e.forests[s].kind;
    if (kind == FD_FOREST_XGB_BINARY_LOGISTIC && q.sa < 0) {
      q.sa = s;
      q.pa = k;
      q.ma = m;
    } else if (kind == FD_FOREST_SKLEARN_IFOREST && q.sb < 0) {
      q.sb = s;
      q.pb = k;
      q.mb = m;
    } else {
      return false;
    }
    ++k;
  }
  if (q.sa < 0 || q.sb < 0) return false;
  const bool wide = want_wide(e);
  if (!plan_current(e, e.ens, q.sa, q.sb, wide) && !build_plan(e, e.ens, q.sa, q.sb, wide)) return false;
  return true;
}
}  // namespace

namespace {
void plan_args(const EnsemblePlan& P, const float* dX, int64_t n, int32_t ld, bool owner_fixed, EnsArgs& a) {
  a.X = dX;
  a.n = n;
  a.ld = ld;
  a.nf = P.nf;
  a.thr = P.thr.as<const float>();
  FD_REQUIRE(P.nf <= kMaxFeatures, FD_ERR_UNSUPPORTED, "ensemble: more than 64 features");
  for (int f = 0; f <= P.nf; ++f) a.thr_off[f] = P.h_thr_off[f];
  a.owner_fixed = owner_fixed ? 1 : 0;
  for (int f = 0; f < kMaxFeatures; ++f) a.cbin[f] = f < (int)P.h_cbin.size() ? P.h_cbin[f] : 0;
  for (size_t k = 0; k < P.h_lut.size() && k < sizeof(a.lut) / sizeof(a.lut[0]); ++k) a.lut[k] = P.h_lut[k];
  a.vec4 = (ld % 4 == 0 && (reinterpret_cast<uintptr_t>(dX) & 15u) == 0) ? 1 : 0;
  const EnsPassSet& ps = P.passes;  // plan_passes
  a.n_pass = (int)ps.f.size() - 1;
  for (int p = 0; p <= a.n_pass; ++p) {
    a.pass_f[p] = ps.f[p];
    a.img_off[p] = ps.img_off[p];
  }
  a.pass_global = ps.glob;
  a.img = P.img.as<const char>();
  for (int q = 0; q < 2; ++q) {
    a.nodes[q] = P.nodes[q].as<const char>();
    a.n_chunks[q] = P.n_chunks[q];
    a.stride[q] = (int)P.stride[q];
  }
  a.base_margin = P.base_margin;
  a.if_offset = P.if_offset;
  a.if_denom = P.if_denominator;
}

// out: 0 blended columns, 1 route result records, 2 the single forest's probability column (a.fp)
bool run_plan(Engine& e, const EnsemblePlan& P, EnsArgs& a, int out, int timing_kind) {
  const void* fn = pick_ensemble(out, P.wide, P.D);
  if (!fn) return false;
  const size_t lds = ens_lds(P.nf, P.wide);
  FD_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int64_t blocks = (a.n + kTile - 1) / kTile;
  Engine::Timed* ev = e.timing ? e.next_event_pair(timing_kind) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, e.stream));
#ifdef FD_FOREST_PROFILE
  a.prof_slot = g_eprof_next;
  g_eprof_next = (g_eprof_next + 1) % kEprofSlots;
  a.clk_slot = g_eclk_next;
  g_eclk_next = (g_eclk_next + 1) % kEclkSlots;
#endif
  void* args[] = {&a};
  FD_HIP(hipLaunchKernel(fn, dim3((unsigned)blocks), dim3(kEnsWG), args, lds, e.stream));
  if (ev) FD_HIP(hipEventRecord(ev->b, e.stream));
  return true;
}
}  // namespace

bool ensemble_applies(Engine& e, const fd_blend_params& p, const int32_t* slots, const uint8_t* present, int64_t n) {
  Pair q;
  return select_pair(e, p, slots, present, n, q);
}

bool launch_ensemble(Engine& e, const fd_blend_params& p, const int32_t* slots, const uint8_t* present,
                     const float* dX, int64_t n, int32_t ld, double* dMP, double* dfp, double* dconf, uint8_t* ddec,
                     uint8_t* drisk, const RouteRecord* records, ResultRecord* results, int compact) {
  Pair q;
  if (!select_pair(e, p, slots, present, n, q)) return false;
  const int pa = q.pa, pb = q.pb, ma = q.ma, mb = q.mb;
  EnsArgs a{};
  plan_args(e.ens, dX, n, compact ? kCompactWidth : ld, e.ens_owner_fixed, a);
  a.compact = compact;
  if (compact && e.ens_bin_global) {  // one pass, every table searched where it lies (L2), nothing staged
    a.n_pass = 1;
    a.pass_f[0] = 0;
    a.pass_f[1] = e.ens.nf;
    a.pass_global = 1ull;
  }
  a.prio = e.ens_prio ? 1 : 0;
  a.pos[0] = pa;
  a.pos[1] = pb;
  a.mcol[0] = ma;
  a.mcol[1] = mb;
  a.blend = blend_consts(p, present);
  a.mp = dMP;
  a.fp = dfp;
  a.conf = dconf;
  a.dec = ddec;
  a.risk = drisk;
  a.rec = records;
  a.res = results;
  const int out = results ? 1 : 0;
  FD_REQUIRE(out == 1 || dfp != nullptr, FD_ERR_INVALID_ARG, "null output");
  return run_plan(e, e.ens, a, out, FD_TIMING_ENSEMBLE);
}

bool launch_ensemble_single(Engine& e, int slot, const float* dX, int64_t n, int32_t ld, double* dprob,
                            double* draw, hipStream_t stream) {
  if (!e.ensemble_on || e.forest_variant != 0 || n <= 0) return false;
  if ((n + kTile - 1) / kTile < kSplitTiles) return false;
  if (slot < 0 || slot >= kMaxSlots || !e.forests[slot].loaded) return false;
  const bool xgb = e.forests[slot].kind == FD_FOREST_XGB_BINARY_LOGISTIC;
  const int sa = xgb ? slot : -1, sb = xgb ? -1 : slot;
  EnsemblePlan& P = e.ens1[slot];
  const bool wide = want_wide(e);
  if (!plan_current(e, P, sa, sb, wide) && !build_plan(e, P, sa, sb, wide)) return false;
  EnsArgs a{};
  plan_args(P, dX, n, ld, e.ens_owner_fixed, a);
  a.prio = e.ens_prio ? 1 : 0;
  a.fp = dprob;
  a.mp = draw;  // one forest: its raw score (XGBoost f32 margin, IsolationForest f64 path-length sum) or null
  const hipStream_t saved = e.stream;
  if (stream) e.stream = stream;
  bool ok = false;
  try {
    ok = run_plan(e, P, a, 2, xgb ? FD_TIMING_XGB : FD_TIMING_IFOREST);
  } catch (...) {
    e.stream = saved;
    throw;
  }
  e.stream = saved;
  if (ok) ++e.ens_single_total;
  return ok;
}


}  // namespace fd
