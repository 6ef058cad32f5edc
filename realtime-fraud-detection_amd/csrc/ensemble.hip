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
// the merged table is staged in LDS in feature ranges (passes) that fit the space of chunk buffer B + the
// leaf tiles (dead until chunk 1), each transaction's 64-wide vector is binned into the [f][256] u32 tile.
// Then the chunk stream is XGBoost's CHA-tree chunks followed by the IsolationForest's CHB-tree chunks
// (node-only, double-buffered by LDS-DMA); per chunk each wave walks its TPG trees for its 64 transactions
// (walk_common.h walk4), stores the leaf values to the chunk's LDS leaf tile, and a rotating owner tree
// group adds the previous chunk's values in tree order into the f32 margin (XGBoost) or the f64 path-length
// sum (IsolationForest): both the reference's sequential sums, bit for bit. Epilogue (tree group 0, one
// thread per transaction): sigmoid / IsolationForest transform, blend_row, outputs (columns, or the 24-B
// route result records of the owner GPU).
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
constexpr int kCHA = 16;  // XGBoost trees per chunk (TPG 4)
constexpr int kCHB = 12;  // IsolationForest trees per chunk (TPG 3; f64 leaf tiles)
constexpr int kMaxPass = 64;

size_t round1k_e(size_t b) { return (b + 1023) / 1024 * 1024; }

constexpr uint32_t ens_cs(int D) { return (uint32_t)((kCHA * (4 << D) + 1023) / 1024 * 1024); }
constexpr uint32_t kEnsLV = (uint32_t)(kCHA * kTile * 4 > kCHB * kTile * 8 ? kCHA * kTile * 4 : kCHB * kTile * 8);

// LDS bytes of the kernel: Xs | bufA | bufB | lvA | lvB | accA (f32) | accB (f64) | flags, + 1 KiB alignment
size_t ens_lds(int nf, int D) {
  return (size_t)nf * 1024 + 2 * ens_cs(D) + 2 * (size_t)kEnsLV + kTile * 4 + kTile * 8 + 64 + 1024;
}

struct EnsArgs {
  const float* X;
  int64_t n;
  int ld, nf;
  const float* thr;
  const int32_t* thr_off;
  int n_pass;
  int pass_f[kMaxPass + 1];
  unsigned long long pass_global;  // bit p: pass p bins from global memory (its table does not fit LDS)
  const char* nodes[2];
  int n_chunks[2];
  int stride[2];
  const float* leaves_a;   // XGBoost [tree][2^D] f32
  const double* leaves_b;  // IsolationForest [tree][2^D] f64
  float base_margin;
  double if_offset, if_denom;
  int pos[2];   // blend position (present-model order) of forest A / B
  int mcol[2];  // model-probability column (caller's model index) of forest A / B
  BlendConsts blend;
  double* mp;
  double* fp;
  double* conf;
  uint8_t* dec;
  uint8_t* risk;
  const RouteRecord* rec;
  ResultRecord* res;
};

template <int D, int TPG, int CH, typename LeafT>
__device__ __forceinline__ void walk_chunk(uint32_t cur, int gg, uint32_t lane4, bool tile_nan,
                                           const LeafT* __restrict__ leaves, int k, uint32_t lv, int txn) {
  constexpr int NL = 1 << D;
  uint32_t slots[TPG];
  if (tile_nan)
    walk4<D, TPG, LeafT, true, true>(cur, gg, lane4, slots);
  else
    walk4<D, TPG, LeafT, false, true>(cur, gg, lane4, slots);
  LeafT lval[TPG];  // leaf values from global memory (L2-resident), all TPG loads in flight together
#pragma unroll
  for (int j = 0; j < TPG; ++j) lval[j] = leaves[((size_t)k * CH + gg * TPG + j) * NL + slots[j]];
#pragma unroll
  for (int j = 0; j < TPG; ++j) lds_store<LeafT>(lv + ((gg * TPG + j) * kTile + txn) * sizeof(LeafT), lval[j]);
}

// chunk c's leaf values added, in tree order, to its forest's running sum (one transaction)
__device__ __forceinline__ void owner_add(int c, int nA, uint32_t lvA, uint32_t lvB, uint32_t accA, uint32_t accB,
                                          int txn) {
  const uint32_t lv = (c & 1) ? lvB : lvA;
  if (c < nA) {
    float acc = lds_load<float>(accA + txn * 4);
#pragma unroll
    for (int t = 0; t < kCHA; ++t) acc += lds_load<float>(lv + (t * kTile + txn) * 4);
    lds_store<float>(accA + txn * 4, acc);
  } else {
    double acc = lds_load<double>(accB + txn * 8);
#pragma unroll
    for (int t = 0; t < kCHB; ++t) acc += lds_load<double>(lv + (t * kTile + txn) * 8);
    lds_store<double>(accB + txn * 8, acc);
  }
}

template <int D, int OUT>
__global__ void __launch_bounds__(kEnsWG) ensemble_kernel(EnsArgs a) {
  constexpr int TPGA = kCHA / 4, TPGB = kCHB / 4;
  constexpr uint32_t CS = ens_cs(D);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t sdyn = (uint32_t)(size_t)((lds_char*)smem);
  const uint32_t s0 = (sdyn + 1023u) & ~1023u;
  char* const lbase = smem + (s0 - sdyn);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int gg = wave >> 2;
  const int txn = ((wave & 3) << 6) + lane;
  const uint32_t lane4 = s0 + (uint32_t)txn * 4u;
  const uint32_t bufA = s0 + (uint32_t)a.nf * 1024u, bufB = bufA + CS;
  const uint32_t lvA = bufB + CS, lvB = lvA + kEnsLV;
  const uint32_t accA = lvB + kEnsLV, accB = accA + kTile * 4;
  const uint32_t flags = accB + kTile * 8;
  const int64_t row = (int64_t)blockIdx.x * kTile + txn;
  const bool valid = row < a.n;
  const int nA = a.n_chunks[0], G = nA + a.n_chunks[1];

  stage_chunk_asm(a.nodes[0], bufA, a.stride[0], kEnsWG / 64);  // chunk 0 lands while the tile is binned
  int anynan = 0;
  {
    uint32_t* Xs = reinterpret_cast<uint32_t*>(lbase);
    const float* xr = a.X + row * (int64_t)a.ld;
    const int ncopy = a.ld < a.nf ? a.ld : a.nf;
    const int q = tid >> 8;  // the four threads sharing `txn` bin every 4th feature of a pass
    for (int p = 0; p < a.n_pass; ++p) {
      const int f0 = a.pass_f[p], f1 = a.pass_f[p + 1];
      const bool glob = (a.pass_global >> p) & 1ull;
      const int o0 = a.thr_off[f0];
      if (!glob) {  // this pass's tables into bufB + lvA + lvB (dead until chunk 1 / the first leaf store)
        float* tl = reinterpret_cast<float*>(lbase + (bufB - s0));
        const int cnt = a.thr_off[f1] - o0;
        for (int i = tid; i < cnt; i += kEnsWG) tl[i] = a.thr[o0 + i];
        __syncthreads();
      }
      for (int f = f0 + q; f < f1; f += 4) {
        uint32_t w = 0;
        if (valid) {
          const float v = f < ncopy ? xr[f] : __builtin_nanf("");  // DMatrix: missing column = NaN
          if (v != v) {
            w = 0xFFFF0000u;
            anynan = 1;
          } else {
            const int o = a.thr_off[f], cnt = a.thr_off[f + 1] - o;
            const uint32_t b = glob ? bin_of<false>(v, a.thr + o, 0u, cnt, lift_steps(cnt))
                                    : bin_of<true>(v, nullptr, bufB + (uint32_t)(o - o0) * 4u, cnt, lift_steps(cnt));
            w = b << 16;
          }
        }
        Xs[f * kTile + txn] = w;
      }
      __syncthreads();  // the staged tables are overwritten by the next pass / chunk 1
    }
  }
  if (gg == 0) {
    lds_store<float>(accA + txn * 4, a.base_margin);
    lds_store<double>(accB + txn * 8, 0.0);
  }
  dma_wait();  // chunk 0 (published by tile_any's barrier)
  const bool tile_nan = tile_any(anynan, reinterpret_cast<uint32_t*>(lbase + (flags - s0)), kEnsWG / 64);

  for (int g = 0; g < G; ++g) {
    const uint32_t cur = (g & 1) ? bufB : bufA;
    if (g + 1 < G) {
      const int h = g + 1, fb = h >= nA ? 1 : 0;
      stage_chunk_asm(a.nodes[fb] + (size_t)(fb ? h - nA : h) * a.stride[fb], (g & 1) ? bufA : bufB, a.stride[fb],
                      kEnsWG / 64);
    }
    if (g > 0 && gg == ((g - 1) & 3)) owner_add(g - 1, nA, lvA, lvB, accA, accB, txn);
    const uint32_t lv = (g & 1) ? lvB : lvA;
    if (g < nA)
      walk_chunk<D, TPGA, kCHA, float>(cur, gg, lane4, tile_nan, a.leaves_a, g, lv, txn);
    else
      walk_chunk<D, TPGB, kCHB, double>(cur, gg, lane4, tile_nan, a.leaves_b, g - nA, lv, txn);
    dma_wait();
    __syncthreads();  // chunk g+1 landed; lv[g&1] complete; owner of g-1 done with lv[(g-1)&1]
  }
  if (G > 0 && gg == ((G - 1) & 3)) owner_add(G - 1, nA, lvA, lvB, accA, accB, txn);
  __syncthreads();
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

template <int OUT>
const void* pick_ensemble(int D) {
  switch (D) {
    case 1: return (const void*)ensemble_kernel<1, OUT>;
    case 2: return (const void*)ensemble_kernel<2, OUT>;
    case 3: return (const void*)ensemble_kernel<3, OUT>;
    case 4: return (const void*)ensemble_kernel<4, OUT>;
    case 5: return (const void*)ensemble_kernel<5, OUT>;
    case 6: return (const void*)ensemble_kernel<6, OUT>;
    case 7: return (const void*)ensemble_kernel<7, OUT>;
    case 8: return (const void*)ensemble_kernel<8, OUT>;
    default: return nullptr;
  }
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

// joint repack of forest A (XGBoost) and B (IsolationForest); false when not possible (the per-model path runs)
bool build_plan(Engine& e, int sa, int sb) {
  EnsemblePlan& P = e.ens;
  P.valid = false;
  const PackedForest& A = e.forests[sa];
  const PackedForest& B = e.forests[sb];
  if (!A.binned || !B.binned || A.num_feature != B.num_feature || A.t_off.empty() || B.t_off.empty()) return false;
  const int D = std::max(A.depth, B.depth);
  if (D > 8) return false;
  const int nf = A.num_feature;
  if (ens_lds(nf, D) > kLdsBudget) return false;
  HostPack hp[2] = {pack_forest_host(A.params, arrays_of(A), D), pack_forest_host(B.params, arrays_of(B), D)};
  if (!hp[0].binned || !hp[1].binned || hp[0].depth != D || hp[1].depth != D) return false;
  // merged per-feature tables
  std::vector<std::vector<float>> merged(nf);
  for (int f = 0; f < nf; ++f) {
    for (const HostPack& h : hp)
      merged[f].insert(merged[f].end(), h.b_thr.begin() + h.b_thr_off[f], h.b_thr.begin() + h.b_thr_off[f + 1]);
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
  const int CH[2] = {kCHA, kCHB};
  const size_t leaf_sz[2] = {sizeof(float), sizeof(double)};
  for (int k = 0; k < 2; ++k) {
    const HostPack& h = hp[k];
    const int T = h.n_trees, nc = (T + CH[k] - 1) / CH[k];
    const size_t stride = round1k_e((size_t)CH[k] * NL * 4);
    std::vector<char> nodes((size_t)nc * stride, 0);
    std::vector<char> leaves((size_t)nc * CH[k] * NL * leaf_sz[k], 0);  // padding trees: zero leaves
    for (int i = 0; i < T; ++i) {
      const char* src = h.b_blob.data() + (size_t)(i / h.b_chunk) * h.b_chunk_stride + (size_t)(i % h.b_chunk) *
                                                                                          h.b_tree_bytes;
      uint32_t* dst = reinterpret_cast<uint32_t*>(nodes.data() + (size_t)(i / CH[k]) * stride +
                                                  (size_t)(i % CH[k]) * NL * 4);
      for (int s = 1; s < NL; ++s) {
        uint32_t w;
        std::memcpy(&w, src + (size_t)s * 4, 4);
        if (!h.pad[(size_t)i * NL + s]) {  // real split: its threshold's index in the merged table
          const int f = (int)((w >> 10) & 63u), j = (int)(w >> 16);
          const float t = h.b_thr[h.b_thr_off[f] + j];
          const uint32_t jm = (uint32_t)(std::lower_bound(merged[f].begin(), merged[f].end(), t) - merged[f].begin());
          w = (jm << 16) | (w & 0xFFFFu);
        }
        dst[s] = w;
      }
      std::memcpy(leaves.data() + (size_t)i * NL * leaf_sz[k], src + (size_t)NL * 4, (size_t)NL * leaf_sz[k]);
    }
    P.nodes[k].ensure(nodes.size());
    FD_HIP(hipMemcpy(P.nodes[k].ptr, nodes.data(), nodes.size(), hipMemcpyHostToDevice));
    P.leaves[k].ensure(leaves.size());
    FD_HIP(hipMemcpy(P.leaves[k].ptr, leaves.data(), leaves.size(), hipMemcpyHostToDevice));
    P.n_trees[k] = T;
    P.CH[k] = CH[k];
    P.n_chunks[k] = nc;
    P.stride[k] = stride;
  }
  P.thr.ensure(std::max<size_t>(4, thr.size() * sizeof(float)));
  if (!thr.empty()) FD_HIP(hipMemcpy(P.thr.ptr, thr.data(), thr.size() * sizeof(float), hipMemcpyHostToDevice));
  P.thr_off.ensure(off.size() * sizeof(int32_t));
  FD_HIP(hipMemcpy(P.thr_off.ptr, off.data(), off.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  P.h_thr_off = off;
  P.max_feature_thr = maxc;
  P.slot[0] = sa;
  P.slot[1] = sb;
  P.gen[0] = A.gen;
  P.gen[1] = B.gen;
  P.n_forests = 2;
  P.D = D;
  P.nf = nf;
  P.kind[0] = FD_FOREST_XGB_BINARY_LOGISTIC;
  P.kind[1] = FD_FOREST_SKLEARN_IFOREST;
  P.base_margin = hp[0].base_margin;
  P.if_offset = B.if_offset;
  P.if_denominator = B.if_denominator;
  P.valid = true;
  return true;
}

}  // namespace

bool launch_ensemble(Engine& e, const fd_blend_params& p, const int32_t* slots, const uint8_t* present,
                     const float* dX, int64_t n, int32_t ld, double* dMP, double* dfp, double* dconf, uint8_t* ddec,
                     uint8_t* drisk, const RouteRecord* records, ResultRecord* results) {
  if (!e.ensemble_on || e.forest_variant != 0 || n <= 0) return false;
  if ((n + kTile - 1) / kTile < kSplitTiles) return false;  // latency batches: the tree-split path
  // the present models must be exactly one XGBoost and one IsolationForest in engine slots
  int sa = -1, sb = -1, pa = -1, pb = -1, ma = -1, mb = -1, k = 0;
  for (int m = 0; m < p.n_models; ++m) {
    if (present && !present[m]) continue;
    const int s = slots[m];
    if (s < 0 || s >= kMaxSlots || !e.forests[s].loaded) return false;
    const int kind = e.forests[s].kind;
    if (kind == FD_FOREST_XGB_BINARY_LOGISTIC && sa < 0) {
      sa = s;
      pa = k;
      ma = m;
    } else if (kind == FD_FOREST_SKLEARN_IFOREST && sb < 0) {
      sb = s;
      pb = k;
      mb = m;
    } else {
      return false;
    }
    ++k;
  }
  if (sa < 0 || sb < 0) return false;
  EnsemblePlan& P = e.ens;
  if (!P.valid || P.slot[0] != sa || P.slot[1] != sb || P.gen[0] != e.forests[sa].gen ||
      P.gen[1] != e.forests[sb].gen) {
    if (!build_plan(e, sa, sb)) return false;
  }
  EnsArgs a{};
  a.X = dX;
  a.n = n;
  a.ld = ld;
  a.nf = P.nf;
  a.thr = P.thr.as<const float>();
  a.thr_off = P.thr_off.as<const int32_t>();
  // binning passes: consecutive features whose tables fit bufB + the leaf tiles; a larger table alone,
  // searched in global memory
  const size_t stage_floats = (ens_cs(P.D) + 2 * (size_t)kEnsLV) / 4;
  int np = 0, f = 0;
  a.pass_f[0] = 0;
  while (f < P.nf) {
    const int32_t* o = P.h_thr_off.data();
    int g = f;
    while (g < P.nf && (size_t)(o[g + 1] - o[f]) <= stage_floats) ++g;
    if (g == f) {  // one feature's table exceeds the LDS space
      a.pass_global |= 1ull << np;
      g = f + 1;
    }
    FD_REQUIRE(np < kMaxPass, FD_ERR_UNSUPPORTED, "ensemble binning plan too long");
    a.pass_f[++np] = g;
    f = g;
  }
  a.n_pass = np;
  for (int q = 0; q < 2; ++q) {
    a.nodes[q] = P.nodes[q].as<const char>();
    a.n_chunks[q] = P.n_chunks[q];
    a.stride[q] = (int)P.stride[q];
  }
  a.leaves_a = P.leaves[0].as<const float>();
  a.leaves_b = P.leaves[1].as<const double>();
  a.base_margin = P.base_margin;
  a.if_offset = P.if_offset;
  a.if_denom = P.if_denominator;
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
  const void* fn = out ? pick_ensemble<1>(P.D) : pick_ensemble<0>(P.D);
  if (!fn) return false;
  const size_t lds = ens_lds(P.nf, P.D);
  FD_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int64_t blocks = (n + kTile - 1) / kTile;
  Engine::Timed* ev = e.timing ? e.next_event_pair(FD_TIMING_ENSEMBLE) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, e.stream));
  void* args[] = {&a};
  FD_HIP(hipLaunchKernel(fn, dim3((unsigned)blocks), dim3(kEnsWG), args, lds, e.stream));
  if (ev) FD_HIP(hipEventRecord(ev->b, e.stream));
  return true;
}

}  // namespace fd
