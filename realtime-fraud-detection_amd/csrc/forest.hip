// forest.hip — repacking and batched inference of the two tree ensembles on the hot path:
//   * XGBoost 2.0.3 gbtree / binary:logistic  (reference: ml/models/model_manager.py:157-161, 309-311)
//   * scikit-learn IsolationForest            (reference: ml/models/model_manager.py:197-200, 338-346;
//                                              sklearn/ensemble/_iforest.py _compute_score_samples)
//
// Packed layout (pack_forest_host): every tree padded to a PERFECT depth-D tree stored as a 1-based
// heap — node i's children are 2i and 2i+1, so a node's two children are one 16 B-aligned pair —
// 2^D node records {f32 thr, u32 meta} (slot 0 unused) followed by 2^D leaf values (f32 XGBoost,
// f64 IsolationForest). meta = feature*1024 (byte offset of the feature's row in the LDS feature
// tile) | default_left << 31. Trees are grouped in chunks of CH trees (1 KiB-aligned stride) that
// are staged into LDS by LDS-DMA.
//
// forest_kernel3 (depth <= 8, the configurations on the path): 1024-thread workgroup per tile of 256
// transactions. The feature tile lives in LDS as [f][256] f32, so a lane reading ANY feature hits
// bank (lane mod 32): feature gathers are conflict-free. Wave w walks, for the 64 transactions of
// txn group w&3, TPG = CH/4 trees of each staged chunk. Each level issues the feature read of the
// selected node AND the 16 B read of its two children together (speculative children): one LDS
// round trip per level instead of two. Leaf values go to LDS and a rotating owner tree-group adds a
// chunk's CH values per transaction in tree order, so the sum is the reference's sequential order:
// XGBoost's f32 margin and sklearn's f64 path-length sum are reproduced bit for bit.
// forest_kernel1: 256 threads, thread per transaction (deep trees D = 9..10; A/B reference).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "blend_row.h"
#include "fd_internal.h"
#include "walk_common.h"

namespace fd {

// ------------------------------------------------------------------------------------------------
// host-side repack

namespace {

int tree_depth(const int32_t* L, const int32_t* R, int64_t m) {
  // iterative DFS with explicit stack; validates child ids
  std::vector<std::pair<int32_t, int>> st;
  st.push_back({0, 0});
  int maxd = 0;
  int64_t visited = 0;
  while (!st.empty()) {
    auto [o, d] = st.back();
    st.pop_back();
    FD_REQUIRE(o >= 0 && o < m, FD_ERR_INVALID_ARG, "tree child index out of range");
    FD_REQUIRE(++visited <= m, FD_ERR_INVALID_ARG, "tree is not a tree (node visited twice)");
    FD_REQUIRE(d <= kMaxDepth, FD_ERR_UNSUPPORTED,
               "tree deeper than " + std::to_string(kMaxDepth) + " levels is not supported");
    if (L[o] < 0) {
      maxd = std::max(maxd, d);
    } else {
      st.push_back({L[o], d + 1});
      st.push_back({R[o], d + 1});
    }
  }
  return maxd;
}

// sklearn compares (double)x_f32 <= thr_f64 (sklearn/tree/_tree.pyx _apply_dense). For an f32 x this
// is x <= floor32(thr), i.e. x < next_up(floor32(thr)): rewrite it as the engine's single x < t form.
float sklearn_threshold_to_lt(double thr) {
  float f = (float)thr;
  if ((double)f > thr) f = std::nextafter(f, -INFINITY);
  return std::nextafter(f, INFINITY);
}

size_t round1k(size_t b) { return (b + 1023) / 1024 * 1024; }

}  // namespace

size_t lds_bytes_kernel3(int nf, size_t chunk_stride, int ch, size_t leaf_sz) {
  // Xs + 2 chunk buffers + 2 leaf-value buffers + accumulator + 16 wave flags + 1 KiB alignment slack
  return (size_t)nf * kTile * 4 + 2 * chunk_stride + 2 * (size_t)ch * kTile * leaf_sz + kTile * leaf_sz + 64 + 1024;
}

size_t lds_bytes_kernel1(int nf, size_t chunk_stride) { return (size_t)nf * kTile * 4 + 2 * chunk_stride + 64; }

// forest_kernel4 has kernel 3's LDS map (bins are u32 words, nodes 4 B)
size_t lds_bytes_kernel4(int nf, size_t chunk_stride, int ch, size_t leaf_sz) {
  return lds_bytes_kernel3(nf, chunk_stride, ch, leaf_sz);
}

namespace {

// Trees per staged chunk: for depth <= 8 the largest multiple of 4 (one tree per wave of each of the
// four tree groups, x TPG) whose LDS image fits forest_kernel3/4's 160 KiB; deeper trees: kernel 1.
int choose_chunk(int D, int nf, size_t tree_bytes, size_t leaf_sz) {
  if (D <= 8) {
    for (int ch = 16; ch >= 4; ch -= 4)
      if (lds_bytes_kernel3(nf, round1k(ch * tree_bytes), ch, leaf_sz) <= kLdsBudget) return ch;
  }
  for (int ch = 8; ch >= 1; ch /= 2)
    if (lds_bytes_kernel1(nf, round1k(ch * tree_bytes)) <= kLdsBudget) return ch;
  return 0;
}

}  // namespace

HostPack pack_forest_host(const fd_forest_params& p, const fd_tree_arrays& t, int min_depth) {
  FD_REQUIRE(p.kind == FD_FOREST_XGB_BINARY_LOGISTIC || p.kind == FD_FOREST_SKLEARN_IFOREST,
             FD_ERR_INVALID_ARG, "unknown forest kind");
  FD_REQUIRE(t.n_trees > 0 && t.tree_offsets && t.left && t.right && t.feature && t.threshold &&
                 t.leaf_value,
             FD_ERR_INVALID_ARG, "incomplete tree arrays");
  FD_REQUIRE(p.num_feature > 0 && p.num_feature <= kMaxFeatures, FD_ERR_UNSUPPORTED,
             "num_feature must be in [1, 64]");
  const bool xgb = p.kind == FD_FOREST_XGB_BINARY_LOGISTIC;
  const int T = t.n_trees, nf = p.num_feature;
  int D = 1;
  for (int i = 0; i < T; ++i) {
    const int64_t a = t.tree_offsets[i], b = t.tree_offsets[i + 1];
    FD_REQUIRE(b > a, FD_ERR_INVALID_ARG, "empty tree");
    D = std::max(D, tree_depth(t.left + a, t.right + a, b - a));
  }
  FD_REQUIRE(min_depth <= kMaxDepth, FD_ERR_UNSUPPORTED, "min_depth beyond the supported depth");
  D = std::max(D, min_depth);
  // engine threshold of an internal node: the f32 t with "go left <=> x < t"
  auto engine_thr = [&](int64_t g) { return xgb ? (float)t.threshold[g] : sklearn_threshold_to_lt(t.threshold[g]); };

  // distinct thresholds per feature (binned layout)
  HostPack hp;
  std::vector<std::vector<float>> tf(nf);
  bool binnable = true;
  for (int64_t g = 0; g < t.tree_offsets[T]; ++g) {
    if (t.left[g] < 0) continue;
    FD_REQUIRE(t.feature[g] >= 0 && t.feature[g] < nf, FD_ERR_INVALID_ARG, "split feature outside [0, num_feature)");
    const float v = engine_thr(g);
    if (v != v) binnable = false;
    tf[t.feature[g]].push_back(v);
  }
  size_t max_cnt = 0;
  for (auto& v : tf) {
    if (!binnable) break;
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());  // == merges -0.0 / 0.0: same comparisons
    max_cnt = std::max(max_cnt, v.size());
  }
  binnable = binnable && max_cnt <= (size_t)kMaxBins;

  const int NL = 1 << D;  // heap slots 1..NL-1 internal, NL..2NL-1 leaves
  const size_t leaf_sz = xgb ? sizeof(float) : sizeof(double);
  const size_t tree_bytes = (size_t)NL * 8 + (size_t)NL * leaf_sz;
  const int CH = choose_chunk(D, nf, tree_bytes, leaf_sz);
  FD_REQUIRE(CH > 0, FD_ERR_UNSUPPORTED, "forest does not fit the LDS budget");
  const size_t chunk_stride = round1k(CH * tree_bytes);
  const int n_chunks = (T + CH - 1) / CH;
  hp.blob.assign(n_chunks * chunk_stride, 0);  // padding trees: all-zero nodes/leaves
  hp.leaf_ids.assign((size_t)n_chunks * CH * NL, -1);

  const size_t b_tree_bytes = (size_t)NL * 4 + (size_t)NL * leaf_sz;
  int BCH = 0;
  if (binnable && D <= 8)
    for (int ch = 16; ch >= 4 && !BCH; ch -= 4)
      if (lds_bytes_kernel4(nf, round1k(ch * b_tree_bytes), ch, leaf_sz) <= kLdsBudget) BCH = ch;
  binnable = binnable && BCH > 0;
  if (binnable) {
    hp.binned = true;
    hp.b_chunk = BCH;
    hp.b_tree_bytes = b_tree_bytes;
    hp.b_chunk_stride = round1k(BCH * b_tree_bytes);
    hp.b_n_chunks = (T + BCH - 1) / BCH;
    hp.b_blob.assign(hp.b_n_chunks * hp.b_chunk_stride, 0);
    hp.b_thr_off.assign(nf + 1, 0);
    for (int f = 0; f < nf; ++f) {
      hp.b_thr_off[f + 1] = hp.b_thr_off[f] + (int32_t)tf[f].size();
      hp.b_thr.insert(hp.b_thr.end(), tf[f].begin(), tf[f].end());
    }
    int st = 1;
    while ((size_t)st * 2 <= max_cnt) st *= 2;
    hp.bin_steps = max_cnt ? st : 0;  // largest power of two <= max_cnt
  }

  std::vector<int32_t> cur(2 * NL);
  hp.pad.assign((size_t)T * NL, 0);
  for (int i = 0; i < T; ++i) {
    const int64_t a = t.tree_offsets[i], m = t.tree_offsets[i + 1] - a;
    const int32_t* L = t.left + a;
    const int32_t* R = t.right + a;
    const int32_t* F = t.feature + a;
    const uint8_t* DL = t.default_left ? t.default_left + a : nullptr;
    const double* LV = t.leaf_value + a;
    char* tb = hp.blob.data() + (size_t)(i / CH) * chunk_stride + (size_t)(i % CH) * tree_bytes;
    uint32_t* nodes = reinterpret_cast<uint32_t*>(tb);
    char* leaves = tb + (size_t)NL * 8;
    char* btb = binnable ? hp.b_blob.data() + (size_t)(i / BCH) * hp.b_chunk_stride + (size_t)(i % BCH) * b_tree_bytes
                         : nullptr;
    uint32_t* bnodes = reinterpret_cast<uint32_t*>(btb);
    char* bleaves = binnable ? btb + (size_t)NL * 4 : nullptr;
    cur[1] = 0;
    for (int s = 1; s < NL; ++s) {
      const int32_t o = cur[s];
      if (L[o] < 0) {  // leaf above depth D: pad node, both subtrees resolve to the same leaf
        hp.pad[(size_t)i * NL + s] = 1;
        nodes[2 * s] = 0;
        nodes[2 * s + 1] = 0;
        if (binnable) bnodes[s] = 0;
        cur[2 * s] = o;
        cur[2 * s + 1] = o;
      } else {
        FD_REQUIRE(R[o] >= 0 && R[o] < m && L[o] < m, FD_ERR_INVALID_ARG, "bad child index");
        const float thr = engine_thr(a + o);
        uint32_t tb32;
        std::memcpy(&tb32, &thr, 4);
        const uint32_t dl = (DL && DL[o]) ? 1u : 0u;
        nodes[2 * s] = tb32;
        nodes[2 * s + 1] = (uint32_t)F[o] * (uint32_t)(kTile * 4) | (dl << 31);
        if (binnable) {
          const auto& v = tf[F[o]];
          const uint32_t j = (uint32_t)(std::lower_bound(v.begin(), v.end(), thr) - v.begin());
          bnodes[s] = j << 16 | (uint32_t)F[o] * (uint32_t)(kTile * 4) | dl;
        }
        cur[2 * s] = L[o];
        cur[2 * s + 1] = R[o];
      }
    }
    for (int s = 0; s < NL; ++s) {
      const int32_t o = cur[NL + s];
      FD_REQUIRE(L[o] < 0, FD_ERR_INVALID_ARG, "internal node at maximum depth");
      if (xgb) {
        const float v = (float)LV[o];
        std::memcpy(leaves + s * 4, &v, 4);
        if (binnable) std::memcpy(bleaves + s * 4, &v, 4);
      } else {
        const double v = LV[o];
        std::memcpy(leaves + s * 8, &v, 8);
        if (binnable) std::memcpy(bleaves + s * 8, &v, 8);
      }
      hp.leaf_ids[(size_t)i * NL + s] = o;
    }
  }
  if (binnable) {  // node-only chunks for forest_kernel6: the largest supported CH whose LDS image fits
    for (int ch : {32, 24, 16})
      if (lds_bytes_kernel3(nf, round1k((size_t)ch * NL * 4), ch, leaf_sz) <= kLdsBudget) {
        hp.n_chunk = ch;
        break;
      }
    if (hp.n_chunk) {
      const int NC = hp.n_chunk;
      hp.n_chunk_stride = round1k((size_t)NC * NL * 4);
      hp.n_n_chunks = (T + NC - 1) / NC;
      hp.n_blob.assign((size_t)hp.n_n_chunks * hp.n_chunk_stride, 0);
      hp.n_leaves.assign((size_t)hp.n_n_chunks * NC * NL * leaf_sz, 0);  // padding trees: zero leaves
      for (int i = 0; i < T; ++i) {
        const char* btb = hp.b_blob.data() + (size_t)(i / BCH) * hp.b_chunk_stride + (size_t)(i % BCH) * b_tree_bytes;
        std::memcpy(hp.n_blob.data() + (size_t)(i / NC) * hp.n_chunk_stride + (size_t)(i % NC) * NL * 4, btb,
                    (size_t)NL * 4);
        std::memcpy(hp.n_leaves.data() + (size_t)i * NL * leaf_sz, btb + (size_t)NL * 4, (size_t)NL * leaf_sz);
      }
    }
  }
  hp.kind = p.kind;
  hp.n_trees = T;
  hp.n_chunks = n_chunks;
  hp.chunk = CH;
  hp.depth = D;
  hp.num_feature = nf;
  hp.tree_bytes = tree_bytes;
  hp.chunk_stride = chunk_stride;
  if (xgb) {
    // learner_model_param.base_score is stored in probability space; the margin it seeds is
    // RegLossObj::ProbToMargin = -logf(1/base_score - 1) evaluated in f32.
    const float bs = (float)p.base_score;
    hp.base_margin = -logf(1.0f / bs - 1.0f);
  }
  return hp;
}

namespace {
template <typename T>
void upload(DeviceBuffer& d, const std::vector<T>& h) {
  d.ensure(std::max<size_t>(h.size() * sizeof(T), 4));
  if (!h.empty()) FD_HIP(hipMemcpy(d.ptr, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
}
}  // namespace

void repack_forest(PackedForest& pf, const fd_forest_params& p, const fd_tree_arrays& t) {
  const HostPack hp = pack_forest_host(p, t);
  forest_loaded(pf, p, t);
  upload(pf.blob, hp.blob);
  upload(pf.leaf_ids, hp.leaf_ids);
  pf.kind = hp.kind;
  pf.n_trees = hp.n_trees;
  pf.n_chunks = hp.n_chunks;
  pf.chunk = hp.chunk;
  pf.depth = hp.depth;
  pf.num_feature = hp.num_feature;
  pf.tree_bytes = hp.tree_bytes;
  pf.chunk_stride = hp.chunk_stride;
  pf.base_margin = hp.base_margin;
  pf.if_offset = p.if_offset;
  pf.if_denominator = p.if_denominator;
  pf.binned = hp.binned;
  if (hp.binned) {
    upload(pf.b_blob, hp.b_blob);
    upload(pf.b_thr, hp.b_thr);
    upload(pf.b_thr_off, hp.b_thr_off);
    pf.b_chunk = hp.b_chunk;
    pf.b_n_chunks = hp.b_n_chunks;
    pf.b_tree_bytes = hp.b_tree_bytes;
    pf.b_chunk_stride = hp.b_chunk_stride;
    pf.bin_steps = hp.bin_steps;
    pf.b_n_thr = (int)hp.b_thr.size();
    pf.n_chunk = hp.n_chunk;
    pf.n_n_chunks = hp.n_n_chunks;
    pf.n_chunk_stride = hp.n_chunk_stride;
    if (hp.n_chunk) {
      upload(pf.n_blob, hp.n_blob);
      upload(pf.n_leaves, hp.n_leaves);
    }
  }
  pf.loaded = true;
}

// ------------------------------------------------------------------------------------------------
// device side

namespace {

// ------------------------------------------------------------------------------------------------
// forest_kernel1: 256 threads = 256 transactions, thread per transaction, CH trees interleaved.

template <int D, int CH, typename LeafT, bool NAN_AWARE>
__device__ __forceinline__ void walk1(const char* cb, const char* xlane, uint32_t (&idx)[CH]) {
  constexpr int TB = (8 + (int)sizeof(LeafT)) << D;
#pragma unroll
  for (int c = 0; c < CH; ++c) idx[c] = 1;
#pragma unroll
  for (int l = 0; l < D; ++l) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const uint2 nd = *reinterpret_cast<const uint2*>(cb + c * TB + idx[c] * 8);
      const float x = *reinterpret_cast<const float*>(xlane + (nd.y & 0x7fffffffu));
      uint32_t right = (x < __uint_as_float(nd.x)) ? 0u : 1u;
      if (NAN_AWARE) {
        if (x != x) right = (nd.y >> 31) ^ 1u;  // missing value: default direction
      }
      idx[c] = 2u * idx[c] + right;
    }
  }
}

template <int D, int CH, typename LeafT, int KIND>
__global__ void __launch_bounds__(kTile)
forest_kernel1(const float* __restrict__ X, int64_t n, int ld, int nf, const char* __restrict__ blob,
               int n_chunks, int chunk_stride, const int32_t* __restrict__ leaf_ids, int n_trees,
               float base_margin, double if_offset, double if_denom, double* __restrict__ out_prob,
               double* __restrict__ out_raw, int32_t* __restrict__ out_leaf) {
  constexpr int NL = 1 << D;
  constexpr int TB = (8 + (int)sizeof(LeafT)) << D;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Xs = reinterpret_cast<float*>(smem);  // [nf][kTile]
  char* bufs = smem + nf * kTile * 4;          // 2 x chunk_stride
  const int t = threadIdx.x;
  const int64_t row = (int64_t)blockIdx.x * kTile + t;
  const bool valid = row < n;

  stage_chunk(blob, bufs, chunk_stride, kTile / 64);  // chunk 0 lands while the tile loads
  int anynan = 0;
  const int ncopy = ld < nf ? ld : nf;
  if (valid) {
    const float* xr = X + row * (int64_t)ld;
    for (int f = 0; f < ncopy; ++f) {
      const float v = xr[f];
      Xs[f * kTile + t] = v;
      anynan |= (v != v);
    }
    for (int f = ncopy; f < nf; ++f) Xs[f * kTile + t] = __builtin_nanf("");  // DMatrix: missing
    anynan |= (ncopy < nf);
  } else {
    for (int f = 0; f < nf; ++f) Xs[f * kTile + t] = 0.f;
  }
  const bool tile_nan = tile_any(anynan, reinterpret_cast<uint32_t*>(bufs + 2 * chunk_stride), kTile / 64);

  const char* xlane = reinterpret_cast<const char*>(Xs + t);
  LeafT acc = (KIND == FD_FOREST_XGB_BINARY_LOGISTIC) ? (LeafT)base_margin : (LeafT)0;
  for (int k = 0; k < n_chunks; ++k) {
    if (k + 1 < n_chunks)
      stage_chunk(blob + (size_t)(k + 1) * chunk_stride, bufs + ((k + 1) & 1) * chunk_stride, chunk_stride,
                  kTile / 64);
    const char* cb = bufs + (k & 1) * chunk_stride;
    uint32_t idx[CH];
    if (tile_nan)
      walk1<D, CH, LeafT, true>(cb, xlane, idx);
    else
      walk1<D, CH, LeafT, false>(cb, xlane, idx);
#pragma unroll
    for (int c = 0; c < CH; ++c)  // tree order: bit-exact sequential accumulation
      acc += *reinterpret_cast<const LeafT*>(cb + c * TB + NL * 8 + (idx[c] - NL) * sizeof(LeafT));
    if (out_leaf != nullptr && valid) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int tg = k * CH + c;
        if (tg < n_trees) out_leaf[row * n_trees + tg] = leaf_ids[(size_t)tg * NL + (idx[c] - NL)];
      }
    }
    __syncthreads();  // chunk k+1 landed (vmcnt drain) and everyone is done with buffer k&1
  }
  if (valid) write_outputs<KIND, LeafT>(acc, row, if_offset, if_denom, out_prob, out_raw);
}

// ------------------------------------------------------------------------------------------------
// forest_kernel3 (depth <= 8): 1024 threads on a 256-transaction tile, speculative children.
//
// LDS (absolute byte addresses; the kernel has no static LDS, the base is 1 KiB aligned):
//   [0, nf*1024)      Xs[f][256] f32     x address = (meta & 0x7fffffff) | txn*4 (one v_and_or)
//   bufA, bufB        2 x chunk_stride   staged trees (LDS-DMA, one chunk ahead)
//   lvA, lvB          2 x [CH][256]      leaf values of the chunk being summed / being walked
//   accL              [256]              running sum per transaction (LeafT)
//   flags             16 words           tile_any

constexpr int kWG3 = 1024;

#ifdef FD_FOREST_PROFILE
// Phase-cycle instrumentation (s_memtime), built only into the profiling variant of the library:
// per wave of the first 256 workgroups {prologue, walk, leaf store, owner sum, barrier, total}.
__device__ unsigned long long g_prof[256 * 16 * 8];
FD_TL_BUF(g_tl_forest);
#define FD_PROF_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define FD_PROF_ADD(acc, a, b) acc += (b) - (a)
#else
#define FD_PROF_T(v)
#define FD_PROF_ADD(acc, a, b)
#endif

// Opaque copy: stops LLVM from folding `c ? v.z : v.x` over one loaded vector into a variable-index
// element extract (a 4-way compare/select chain per component).
__device__ __forceinline__ void opaque4(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}

// Walks TPG trees of the staged chunk at `buf` for this lane's transaction. A[j] is the LDS address
// of the children pair of the current node (heap slot i: tb + 16 i); per level one feature read and
// one 16 B read of the chosen child's own children are in flight together. Returns leaf slots.
template <int D, int TPG, typename LeafT, bool NAN_AWARE>
__device__ __forceinline__ void walk3(uint32_t buf, int gg, uint32_t lane4, uint32_t (&slot)[TPG]) {
  constexpr uint32_t TB = (8u + (uint32_t)sizeof(LeafT)) << D;
  constexpr uint32_t NL = 1u << D;
  uint32_t tb[TPG], A[TPG], thr[TPG], meta[TPG], k0[TPG], k1[TPG], k2[TPG], k3[TPG];
  float x[TPG];
#pragma unroll
  for (int j = 0; j < TPG; ++j) {
    tb[j] = buf + (uint32_t)(gg * TPG + j) * TB;
    const u32x2 root = lds_load<u32x2>(tb[j] + 8u);  // heap slot 1
    thr[j] = root.x;
    meta[j] = root.y;
    A[j] = tb[j] + 16u;
  }
#pragma unroll
  for (int j = 0; j < TPG; ++j) {
    x[j] = lds_load<float>((meta[j] & 0x7fffffffu) | lane4);
    if (D > 1) {
      const u32x4 k = lds_load<u32x4>(A[j]);  // slots 2, 3
      k0[j] = k.x; k1[j] = k.y; k2[j] = k.z; k3[j] = k.w;
    }
  }
#pragma unroll
  for (int l = 0; l < D; ++l) {
#pragma unroll
    for (int j = 0; j < TPG; ++j) {
      bool right = !(x[j] < __uint_as_float(thr[j]));
      if (NAN_AWARE) {
        if (x[j] != x[j]) right = (int32_t)meta[j] >= 0;  // missing: default direction
      }
      A[j] = 2u * A[j] - tb[j] + (right ? 16u : 0u);  // children pair of the chosen child
      if (l + 1 < D) {
        opaque4(k0[j], k1[j], k2[j], k3[j]);
        thr[j] = right ? k2[j] : k0[j];
        meta[j] = right ? k3[j] : k1[j];
      }
    }
    if (l + 1 < D) {
#pragma unroll
      for (int j = 0; j < TPG; ++j) {
        x[j] = lds_load<float>((meta[j] & 0x7fffffffu) | lane4);
        if (l + 2 < D) {
          const u32x4 k = lds_load<u32x4>(A[j]);
          k0[j] = k.x; k1[j] = k.y; k2[j] = k.z; k3[j] = k.w;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < TPG; ++j) slot[j] = ((A[j] - tb[j]) >> 4) - NL;  // leaf heap slot - 2^D
}

template <int D, int CH, typename LeafT, int KIND>
__global__ void __launch_bounds__(kWG3)
forest_kernel3(const float* __restrict__ X, int64_t n, int ld, int nf, const char* __restrict__ blob,
               int n_chunks, int chunk_stride, const int32_t* __restrict__ leaf_ids, int n_trees,
               float base_margin, double if_offset, double if_denom, double* __restrict__ out_prob,
               double* __restrict__ out_raw, int32_t* __restrict__ out_leaf) {
  constexpr int TPG = CH / 4;
  constexpr int NL = 1 << D;
  constexpr uint32_t TB = (8u + (uint32_t)sizeof(LeafT)) << D;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // 1 KiB-aligned base: no static LDS in this kernel (so the base is 0); 1 KiB slack reserved anyway
  const uint32_t sdyn = (uint32_t)(size_t)((lds_char*)smem);
  const uint32_t s0 = (sdyn + 1023u) & ~1023u;
  char* const lbase = smem + (s0 - sdyn);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int gg = wave >> 2;                  // tree group
  const int txn = ((wave & 3) << 6) + lane;  // 0..255 within the tile
  const uint32_t lane4 = s0 + (uint32_t)txn * 4u;
  const uint32_t xbytes = (uint32_t)nf * 1024u;
  const uint32_t bufA = s0 + xbytes, bufB = bufA + (uint32_t)chunk_stride;
  const uint32_t lvA = bufB + (uint32_t)chunk_stride;
  const uint32_t lvB = lvA + CH * kTile * sizeof(LeafT);
  const uint32_t accL = lvB + CH * kTile * sizeof(LeafT);
  const int64_t row = (int64_t)blockIdx.x * kTile + txn;
  const bool valid = row < n;
#ifdef FD_FOREST_PROFILE
  unsigned long long p_walk = 0, p_leaf = 0, p_own = 0, p_sync = 0;
#endif
  FD_PROF_T(p_t0);

  stage_chunk_asm(blob, bufA, chunk_stride, kWG3 / 64);  // chunk 0 lands while the tile loads
  int anynan = 0;
  const int ncopy = ld < nf ? ld : nf;
  {
    const int q = tid >> 8;  // the four threads sharing `txn` load every 4th column
    float* Xs = reinterpret_cast<float*>(lbase);
    if (valid) {
      const float* xr = X + row * (int64_t)ld;
      for (int f = q; f < ncopy; f += 4) {
        const float v = xr[f];
        Xs[f * kTile + txn] = v;
        anynan |= (v != v);
      }
      for (int f = ncopy + q; f < nf; f += 4) Xs[f * kTile + txn] = __builtin_nanf("");
      anynan |= (ncopy < nf);
    } else {
      for (int f = q; f < nf; f += 4) Xs[f * kTile + txn] = 0.f;
    }
    if (gg == 0)
      lds_store<LeafT>(accL + txn * sizeof(LeafT),
                       (KIND == FD_FOREST_XGB_BINARY_LOGISTIC) ? (LeafT)base_margin : (LeafT)0);
  }
  dma_wait();  // chunk 0 (published by tile_any's barrier)
  const bool tile_nan =
      tile_any(anynan, reinterpret_cast<uint32_t*>(lbase + (accL - s0) + kTile * sizeof(LeafT)), kWG3 / 64);
  FD_PROF_T(p_t1);

  for (int k = 0; k < n_chunks; ++k) {
    FD_PROF_T(q0);
    const uint32_t cur = (k & 1) ? bufB : bufA;
    if (k + 1 < n_chunks)
      stage_chunk_asm(blob + (size_t)(k + 1) * chunk_stride, (k & 1) ? bufA : bufB, chunk_stride, kWG3 / 64);
    // owner of chunk k-1 adds its leaf values in tree order
    if (k > 0 && gg == ((k - 1) & 3)) {
      const uint32_t lv = ((k - 1) & 1) ? lvB : lvA;
      LeafT acc = lds_load<LeafT>(accL + txn * sizeof(LeafT));
#pragma unroll
      for (int c = 0; c < CH; ++c) acc += lds_load<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT));
      lds_store<LeafT>(accL + txn * sizeof(LeafT), acc);
    }
    FD_PROF_T(q1);
    uint32_t slots[TPG];
    if (tile_nan)
      walk3<D, TPG, LeafT, true>(cur, gg, lane4, slots);
    else
      walk3<D, TPG, LeafT, false>(cur, gg, lane4, slots);
#ifdef FD_FOREST_PROFILE
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
    FD_PROF_T(q2);
    const uint32_t lv = (k & 1) ? lvB : lvA;
#pragma unroll
    for (int j = 0; j < TPG; ++j) {
      const int c = gg * TPG + j;
      const uint32_t tb = cur + (uint32_t)c * TB;
      const uint32_t slot = slots[j];
      lds_store<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT), lds_load<LeafT>(tb + NL * 8u + slot * sizeof(LeafT)));
      if (out_leaf != nullptr && valid) {
        const int tg = k * CH + c;
        if (tg < n_trees) out_leaf[row * n_trees + tg] = leaf_ids[(size_t)tg * NL + slot];
      }
    }
    FD_PROF_T(q3);
    dma_wait();
    __syncthreads();  // chunk k+1 landed; lv[k&1] complete; owner of k-1 done with lv[(k-1)&1]
    FD_PROF_T(q4);
    FD_PROF_ADD(p_own, q0, q1);
    FD_PROF_ADD(p_walk, q1, q2);
    FD_PROF_ADD(p_leaf, q2, q3);
    FD_PROF_ADD(p_sync, q3, q4);
  }
#ifdef FD_FOREST_PROFILE
  if (lane == 0 && blockIdx.x < 256) {
    FD_PROF_T(p_t2);
    unsigned long long* o = g_prof + ((size_t)blockIdx.x * 16 + wave) * 8;
    o[0] = p_t1 - p_t0; o[1] = p_walk; o[2] = p_leaf; o[3] = p_own; o[4] = p_sync; o[5] = p_t2 - p_t0;
    o[6] = p_t0; o[7] = 0;
  }
#endif
  const int last = n_chunks - 1;
  if (gg != (last & 3)) return;
  LeafT acc = lds_load<LeafT>(accL + txn * sizeof(LeafT));
  {
    const uint32_t lv = (last & 1) ? lvB : lvA;
#pragma unroll
    for (int c = 0; c < CH; ++c) acc += lds_load<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT));
  }
  if (valid) write_outputs<KIND, LeafT>(acc, row, if_offset, if_denom, out_prob, out_raw);
}

// ------------------------------------------------------------------------------------------------
// forest_kernel4 (depth <= 8, binned layout): kernel 3's structure with 4-byte nodes.
//
// The prologue replaces every feature value by its bin: the count of the feature's distinct split
// thresholds that are <= x (branchless binary lifting over the sorted table, staged in LDS when it
// fits), stored as the u32 word bin << 16 (missing/NaN: 0xFFFF << 16). A node word is
// j << 16 | feature * 1024 | default_left, so "x < t_j" is "bin <= j" is ONE unsigned compare
// word(x) <= node, the feature-row address is (node & 0xFC00) | lane, and a node's two children are
// one 8-byte pair read: per level one ds_read_b32 (feature) and one ds_read_b64 (children).

template <int D, int CH, typename LeafT, int KIND>
__global__ void __launch_bounds__(kWG3)
forest_kernel4(const float* __restrict__ X, int64_t n, int ld, int nf, const char* __restrict__ blob,
               int n_chunks, int chunk_stride, const int32_t* __restrict__ leaf_ids, int n_trees,
               const float* __restrict__ thr, const int32_t* __restrict__ thr_off, int bin_steps,
               float base_margin, double if_offset, double if_denom, double* __restrict__ out_prob,
               double* __restrict__ out_raw, int32_t* __restrict__ out_leaf) {
  constexpr int TPG = CH / 4;
  constexpr int NL = 1 << D;
  constexpr uint32_t TB = (4u + (uint32_t)sizeof(LeafT)) << D;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t sdyn = (uint32_t)(size_t)((lds_char*)smem);
  const uint32_t s0 = (sdyn + 1023u) & ~1023u;
  char* const lbase = smem + (s0 - sdyn);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int gg = wave >> 2;
  const int txn = ((wave & 3) << 6) + lane;
  const uint32_t lane4 = s0 + (uint32_t)txn * 4u;
  const uint32_t xbytes = (uint32_t)nf * 1024u;
  const uint32_t bufA = s0 + xbytes, bufB = bufA + (uint32_t)chunk_stride;
  const uint32_t lvA = bufB + (uint32_t)chunk_stride;
  const uint32_t lvB = lvA + CH * kTile * sizeof(LeafT);
  const uint32_t accL = lvB + CH * kTile * sizeof(LeafT);
  const int64_t row = (int64_t)blockIdx.x * kTile + txn;
  const bool valid = row < n;
#ifdef FD_FOREST_PROFILE
  unsigned long long p_walk = 0, p_leaf = 0, p_own = 0, p_sync = 0;
#endif
  FD_PROF_T(p_t0);

  stage_chunk_asm(blob, bufA, chunk_stride, kWG3 / 64);  // chunk 0 lands while the tile is binned
  // threshold tables: into LDS over bufB + lv (dead until chunk 1 / the first leaf store) if they fit
  const int n_thr = thr_off[nf];
  const bool tbl_lds = (uint32_t)n_thr * 4u <= accL - bufB;
  if (tbl_lds) {
    float* tl = reinterpret_cast<float*>(lbase + (bufB - s0));
    for (int i = tid; i < n_thr; i += kWG3) tl[i] = thr[i];
    __syncthreads();
  }
  int anynan = 0;
  const int ncopy = ld < nf ? ld : nf;
  {
    const int q = tid >> 8;  // the four threads sharing `txn` bin every 4th column
    uint32_t* Xs = reinterpret_cast<uint32_t*>(lbase);
    const float* xr = X + row * (int64_t)ld;
    for (int f = q; f < nf; f += 4) {
      uint32_t w = 0;
      if (valid) {
        const float v = f < ncopy ? xr[f] : __builtin_nanf("");  // DMatrix: missing column = NaN
        if (v != v) {
          w = 0xFFFF0000u;
          anynan = 1;
        } else {
          const int o = thr_off[f], cnt = thr_off[f + 1] - o;
          const uint32_t b = tbl_lds ? bin_of<true>(v, nullptr, bufB + (uint32_t)o * 4u, cnt, lift_steps(cnt))
                                     : bin_of<false>(v, thr + o, 0u, cnt, lift_steps(cnt));
          w = b << 16;
        }
      }
      Xs[f * kTile + txn] = w;
    }
    if (gg == 0)
      lds_store<LeafT>(accL + txn * sizeof(LeafT),
                       (KIND == FD_FOREST_XGB_BINARY_LOGISTIC) ? (LeafT)base_margin : (LeafT)0);
  }
  dma_wait();  // chunk 0 (published by tile_any's barrier)
  const bool tile_nan =
      tile_any(anynan, reinterpret_cast<uint32_t*>(lbase + (accL - s0) + kTile * sizeof(LeafT)), kWG3 / 64);
  FD_PROF_T(p_t1);

  for (int k = 0; k < n_chunks; ++k) {
    FD_PROF_T(q0);
    const uint32_t cur = (k & 1) ? bufB : bufA;
    if (k + 1 < n_chunks)
      stage_chunk_asm(blob + (size_t)(k + 1) * chunk_stride, (k & 1) ? bufA : bufB, chunk_stride, kWG3 / 64);
    if (k > 0 && gg == ((k - 1) & 3)) {  // owner of chunk k-1 adds its leaf values in tree order
      const uint32_t lv = ((k - 1) & 1) ? lvB : lvA;
      LeafT acc = lds_load<LeafT>(accL + txn * sizeof(LeafT));
#pragma unroll
      for (int c = 0; c < CH; ++c) acc += lds_load<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT));
      lds_store<LeafT>(accL + txn * sizeof(LeafT), acc);
    }
    FD_PROF_T(q1);
    uint32_t slots[TPG];
    if (tile_nan)
      walk4<D, TPG, LeafT, true>(cur, gg, lane4, slots);
    else
      walk4<D, TPG, LeafT, false>(cur, gg, lane4, slots);
#ifdef FD_FOREST_PROFILE
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
    FD_PROF_T(q2);
    const uint32_t lv = (k & 1) ? lvB : lvA;
#pragma unroll
    for (int j = 0; j < TPG; ++j) {
      const int c = gg * TPG + j;
      const uint32_t tb = cur + (uint32_t)c * TB;
      lds_store<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT),
                       lds_load<LeafT>(tb + NL * 4u + slots[j] * sizeof(LeafT)));
      if (out_leaf != nullptr && valid) {
        const int tg = k * CH + c;
        if (tg < n_trees) out_leaf[row * n_trees + tg] = leaf_ids[(size_t)tg * NL + slots[j]];
      }
    }
    FD_PROF_T(q3);
    dma_wait();
    __syncthreads();  // chunk k+1 landed; lv[k&1] complete; owner of k-1 done with lv[(k-1)&1]
    FD_PROF_T(q4);
    FD_PROF_ADD(p_own, q0, q1);
    FD_PROF_ADD(p_walk, q1, q2);
    FD_PROF_ADD(p_leaf, q2, q3);
    FD_PROF_ADD(p_sync, q3, q4);
  }
#ifdef FD_FOREST_PROFILE
  if (lane == 0 && blockIdx.x < 256) {
    FD_PROF_T(p_t2);
    unsigned long long* o = g_prof + ((size_t)blockIdx.x * 16 + wave) * 8;
    o[0] = p_t1 - p_t0; o[1] = p_walk; o[2] = p_leaf; o[3] = p_own; o[4] = p_sync; o[5] = p_t2 - p_t0;
    o[6] = p_t0; o[7] = 0;
  }
#endif
  const int last = n_chunks - 1;
  if (gg != (last & 3)) return;
  LeafT acc = lds_load<LeafT>(accL + txn * sizeof(LeafT));
  {
    const uint32_t lv = (last & 1) ? lvB : lvA;
#pragma unroll
    for (int c = 0; c < CH; ++c) acc += lds_load<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT));
  }
  if (valid) write_outputs<KIND, LeafT>(acc, row, if_offset, if_denom, out_prob, out_raw);
}

// ------------------------------------------------------------------------------------------------
// forest_kernel6 (depth <= 8, binned nodes): kernel 4 with node-only chunks. The staged chunk holds
// only the CH trees' node words (1 KiB per depth-8 tree instead of 2-3 KiB with the leaves), so the
// same LDS budget stages more trees per chunk: CH = 24 for XGBoost (TPG = 6 independent walks per
// wave instead of 4) and 16 for the f64-leaf IsolationForest (instead of 8). The walk is bound by the
// LDS round-trip latency of its dependent chains, not by LDS cycles (PMC: LDS array ~50 % busy, VALU
// ~35 %), so more chains per wave is the lever. After the walk each lane reads its TPG leaf values
// from the global [tree][2^D] array (L2-resident: 0.5 MiB for 500 x depth 8) with all loads in
// flight together; the owner pass and the tree-order sum are kernel 4's.
template <int D, int CH, typename LeafT, int KIND>
__global__ void __launch_bounds__(kWG3)
forest_kernel6(const float* __restrict__ X, int64_t n, int ld, int nf, const char* __restrict__ blob,
               int n_chunks, int chunk_stride, const int32_t* __restrict__ leaf_ids, int n_trees,
               const float* __restrict__ thr, const int32_t* __restrict__ thr_off, int bin_steps,
               float base_margin, double if_offset, double if_denom, double* __restrict__ out_prob,
               double* __restrict__ out_raw, int32_t* __restrict__ out_leaf, const LeafT* __restrict__ leaves) {
  constexpr int TPG = CH / 4;
  constexpr int NL = 1 << D;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t sdyn = (uint32_t)(size_t)((lds_char*)smem);
  const uint32_t s0 = (sdyn + 1023u) & ~1023u;
  char* const lbase = smem + (s0 - sdyn);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int gg = wave >> 2;
  const int txn = ((wave & 3) << 6) + lane;
  const uint32_t lane4 = s0 + (uint32_t)txn * 4u;
  const uint32_t xbytes = (uint32_t)nf * 1024u;
  const uint32_t bufA = s0 + xbytes, bufB = bufA + (uint32_t)chunk_stride;
  const uint32_t lvA = bufB + (uint32_t)chunk_stride;
  const uint32_t lvB = lvA + CH * kTile * sizeof(LeafT);
  const uint32_t accL = lvB + CH * kTile * sizeof(LeafT);
  const int64_t row = (int64_t)blockIdx.x * kTile + txn;
  const bool valid = row < n;
#ifdef FD_FOREST_PROFILE
  unsigned long long p_walk = 0, p_leaf = 0, p_own = 0, p_sync = 0;
#endif
  FD_PROF_T(p_t0);

  stage_chunk_asm(blob, bufA, chunk_stride, kWG3 / 64);  // chunk 0 lands while the tile is binned
  // threshold tables: into LDS over bufB + lv (dead until chunk 1 / the first leaf store) if they fit
  const int n_thr = thr_off[nf];
  const bool tbl_lds = (uint32_t)n_thr * 4u <= accL - bufB;
  if (tbl_lds) {
    float* tl = reinterpret_cast<float*>(lbase + (bufB - s0));
    for (int i = tid; i < n_thr; i += kWG3) tl[i] = thr[i];
    __syncthreads();
  }
  int anynan = 0;
  const int ncopy = ld < nf ? ld : nf;
  {
    const int q = tid >> 8;  // the four threads sharing `txn` bin every 4th column
    uint32_t* Xs = reinterpret_cast<uint32_t*>(lbase);
    const float* xr = X + row * (int64_t)ld;
    for (int f = q; f < nf; f += 4) {
      uint32_t w = 0;
      if (valid) {
        const float v = f < ncopy ? xr[f] : __builtin_nanf("");  // DMatrix: missing column = NaN
        if (v != v) {
          w = 0xFFFF0000u;
          anynan = 1;
        } else {
          const int o = thr_off[f], cnt = thr_off[f + 1] - o;
          const uint32_t b = tbl_lds ? bin_of<true>(v, nullptr, bufB + (uint32_t)o * 4u, cnt, lift_steps(cnt))
                                     : bin_of<false>(v, thr + o, 0u, cnt, lift_steps(cnt));
          w = b << 16;
        }
      }
      Xs[f * kTile + txn] = w;
    }
    if (gg == 0)
      lds_store<LeafT>(accL + txn * sizeof(LeafT),
                       (KIND == FD_FOREST_XGB_BINARY_LOGISTIC) ? (LeafT)base_margin : (LeafT)0);
  }
  dma_wait();  // chunk 0 (published by tile_any's barrier)
  const bool tile_nan =
      tile_any(anynan, reinterpret_cast<uint32_t*>(lbase + (accL - s0) + kTile * sizeof(LeafT)), kWG3 / 64);
  FD_PROF_T(p_t1);

  for (int k = 0; k < n_chunks; ++k) {
    FD_PROF_T(q0);
    const uint32_t cur = (k & 1) ? bufB : bufA;
    if (k + 1 < n_chunks)
      stage_chunk_asm(blob + (size_t)(k + 1) * chunk_stride, (k & 1) ? bufA : bufB, chunk_stride, kWG3 / 64);
    if (k > 0 && gg == ((k - 1) & 3)) {  // owner of chunk k-1 adds its leaf values in tree order
      const uint32_t lv = ((k - 1) & 1) ? lvB : lvA;
      LeafT acc = lds_load<LeafT>(accL + txn * sizeof(LeafT));
#pragma unroll
      for (int c = 0; c < CH; ++c) acc += lds_load<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT));
      lds_store<LeafT>(accL + txn * sizeof(LeafT), acc);
    }
    FD_PROF_T(q1);
    uint32_t slots[TPG];
    if (tile_nan)
      walk4<D, TPG, LeafT, true, true>(cur, gg, lane4, slots);
    else
      walk4<D, TPG, LeafT, false, true>(cur, gg, lane4, slots);
#ifdef FD_FOREST_PROFILE
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
    const uint32_t lv = (k & 1) ? lvB : lvA;
    LeafT lval[TPG];  // leaf values from global memory (L2-resident), all TPG loads in flight together
#pragma unroll
    for (int j = 0; j < TPG; ++j) lval[j] = leaves[((size_t)k * CH + gg * TPG + j) * NL + slots[j]];
#pragma unroll
    for (int j = 0; j < TPG; ++j) {
      const int c = gg * TPG + j;
      lds_store<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT), lval[j]);
      if (out_leaf != nullptr && valid) {
        const int tg = k * CH + c;
        if (tg < n_trees) out_leaf[row * n_trees + tg] = leaf_ids[(size_t)tg * NL + slots[j]];
      }
    }
    FD_PROF_T(q2);
    FD_PROF_T(q3);
    dma_wait();
    __syncthreads();  // chunk k+1 landed; lv[k&1] complete; owner of k-1 done with lv[(k-1)&1]
    FD_PROF_T(q4);
    FD_PROF_ADD(p_own, q0, q1);
    FD_PROF_ADD(p_walk, q1, q2);
    FD_PROF_ADD(p_leaf, q2, q3);
    FD_PROF_ADD(p_sync, q3, q4);
  }
#ifdef FD_FOREST_PROFILE
  if (lane == 0 && blockIdx.x < 256) {
    FD_PROF_T(p_t2);
    unsigned long long* o = g_prof + ((size_t)blockIdx.x * 16 + wave) * 8;
    o[0] = p_t1 - p_t0; o[1] = p_walk; o[2] = p_leaf; o[3] = p_own; o[4] = p_sync; o[5] = p_t2 - p_t0;
    o[6] = p_t0; o[7] = 0;
  }
#endif
  const int last = n_chunks - 1;
  if (gg != (last & 3)) return;
  LeafT acc = lds_load<LeafT>(accL + txn * sizeof(LeafT));
  {
    const uint32_t lv = (last & 1) ? lvB : lvA;
#pragma unroll
    for (int c = 0; c < CH; ++c) acc += lds_load<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT));
  }
  if (valid) write_outputs<KIND, LeafT>(acc, row, if_offset, if_denom, out_prob, out_raw);
}

// ------------------------------------------------------------------------------------------------
// Small-batch (latency) path: tree-split over workgroups. A 1k micro-batch is 4 tiles, so the
// tile-per-workgroup kernels keep 4 CUs busy for the whole forest (~90 us for 500 x depth 8). Here
//   split_bin_kernel   : every feature value -> its bin word once, feature-major [nf][n_pad] in HBM,
//                        plus a per-tile "has NaN" flag;
//   split_walk_kernel  : grid (tiles, chunk groups): kernel 4's walk over the group's chunks; the bin
//                        rows of the tile arrive by LDS-DMA (1 KiB per feature row), every leaf value
//                        goes to a [tree][n] scratch in HBM (and the leaf id when asked);
//   split_sum_kernel   : per transaction, base margin + the leaf values in tree order (the
//                        reference's sequential f32 / f64 sum, bit for bit), then the outputs.

__global__ void __launch_bounds__(kSplitBin)
split_bin_kernel(const float* __restrict__ X, int64_t n, int64_t n_pad, int ld, int nf, const float* __restrict__ thr,
                 const int32_t* __restrict__ thr_off, int bin_steps, uint32_t* __restrict__ bins,
                 uint32_t* __restrict__ tile_nan) {
  split_bin_body(X, n, n_pad, ld, (int)blockIdx.y, (int64_t)blockIdx.x * kSplitBin + threadIdx.x, thr, thr_off, bins,
                 tile_nan);
}

// both forests of a latency batch binned in one launch: grid.y = nf_a + nf_b
__global__ void __launch_bounds__(kSplitBin)
split_bin_pair_kernel(const float* __restrict__ X, int64_t n, int64_t n_pad, int ld, SplitBinArgs a, SplitBinArgs b) {
  FD_TL(g_tl_forest, 3, 0);
  split_bin_pair_cell(X, n, n_pad, ld, a, b, (int)blockIdx.y, (int64_t)blockIdx.x * kSplitBin + threadIdx.x);
  FD_TL(g_tl_forest, 3, 3);
}

// Stage `rows` rows of 1 KiB (row r at src + r * row_stride) into LDS at dst + r * 1024 by LDS-DMA.
__device__ __forceinline__ void stage_rows_asm(const char* __restrict__ src, size_t row_stride, uint32_t dst, int rows,
                                               int nwaves) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int p = wave; p < rows; p += nwaves) {
    const char* g = src + (size_t)p * row_stride + lane * 16;
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

template <int D, int CH, typename LeafT>
__device__ __forceinline__ void split_walk_body(const uint32_t* __restrict__ bins, int64_t n, int64_t n_pad, int nf,
                                                const uint32_t* __restrict__ tile_nan, const char* __restrict__ blob,
                                                int n_chunks, int chunk_stride, int chunks_per_group,
                                                const int32_t* __restrict__ leaf_ids, int n_trees,
                                                LeafT* __restrict__ leaves, int32_t* __restrict__ out_leaf, int gy) {
  constexpr int TPG = CH / 4;
  constexpr int NL = 1 << D;
  constexpr uint32_t TB = (4u + (uint32_t)sizeof(LeafT)) << D;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t sdyn = (uint32_t)(size_t)((lds_char*)smem);
  const uint32_t s0 = (sdyn + 1023u) & ~1023u;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int gg = wave >> 2;
  const int txn = ((wave & 3) << 6) + lane;
  const uint32_t lane4 = s0 + (uint32_t)txn * 4u;
  const uint32_t bufA = s0 + (uint32_t)nf * 1024u, bufB = bufA + (uint32_t)chunk_stride;
  const int tile = blockIdx.x;
  const int64_t row = (int64_t)tile * kTile + txn;
  const int k0 = gy * chunks_per_group;
  const int k1 = min(n_chunks, k0 + chunks_per_group);
  if (k0 >= k1) return;  // uniform per workgroup
  stage_rows_asm(reinterpret_cast<const char*>(bins + (size_t)tile * kTile), (size_t)n_pad * 4u, s0, nf, kWG3 / 64);
  stage_chunk_asm(blob + (size_t)k0 * chunk_stride, bufA, chunk_stride, kWG3 / 64);
  const bool tile_has_nan = tile_nan[tile] != 0u;
  dma_wait();
  __syncthreads();
  for (int k = k0; k < k1; ++k) {
    const uint32_t cur = ((k - k0) & 1) ? bufB : bufA;
    if (k + 1 < k1)
      stage_chunk_asm(blob + (size_t)(k + 1) * chunk_stride, ((k - k0) & 1) ? bufA : bufB, chunk_stride, kWG3 / 64);
    uint32_t slots[TPG];
    if (tile_has_nan)
      walk4<D, TPG, LeafT, true>(cur, gg, lane4, slots);
    else
      walk4<D, TPG, LeafT, false>(cur, gg, lane4, slots);
#pragma unroll
    for (int j = 0; j < TPG; ++j) {
      const int c = gg * TPG + j;
      const int tg = k * CH + c;
      const uint32_t tb = cur + (uint32_t)c * TB;
      if (row < n && tg < n_trees) {
        leaves[(size_t)tg * n + row] = lds_load<LeafT>(tb + NL * 4u + slots[j] * sizeof(LeafT));
        if (out_leaf != nullptr) out_leaf[row * n_trees + tg] = leaf_ids[(size_t)tg * NL + slots[j]];
      }
    }
    dma_wait();
    __syncthreads();
  }
}

template <int D, int CH, typename LeafT>
__global__ void __launch_bounds__(kWG3)
split_walk_kernel(const uint32_t* __restrict__ bins, int64_t n, int64_t n_pad, int nf,
                  const uint32_t* __restrict__ tile_nan, const char* __restrict__ blob, int n_chunks,
                  int chunk_stride, int chunks_per_group, const int32_t* __restrict__ leaf_ids, int n_trees,
                  LeafT* __restrict__ leaves, int32_t* __restrict__ out_leaf) {
  split_walk_body<D, CH, LeafT>(bins, n, n_pad, nf, tile_nan, blob, n_chunks, chunk_stride, chunks_per_group, leaf_ids,
                                n_trees, leaves, out_leaf, (int)blockIdx.y);
}

constexpr int kSumRows = 8;  // transactions per workgroup of the sum kernels (below)

// one forest's side of the latency pair (split_walk_pair_kernel / split_sum_pair_blend_kernel)
struct SplitWalkArgs {
  const uint32_t* bins;
  const uint32_t* tile_nan;
  const char* blob;
  int n_chunks, chunk_stride, cpg, groups;
  const int32_t* leaf_ids;
  int n_trees;
  void* leaves;
};

// Both forests of a latency batch walked in ONE launch (grid.y = XGBoost's chunk groups, then the
// IsolationForest's): the launch and the queue gap between two walks saved, and the two walks' workgroups share the
// CUs instead of running one after the other
template <int DX, int CHX, int DI, int CHI>
__global__ void __launch_bounds__(kWG3) split_walk_pair_kernel(int64_t n, int64_t n_pad, int nf, SplitWalkArgs x,
                                                               SplitWalkArgs f) {
  FD_TL(g_tl_forest, 4, 0);
  const int gy = (int)blockIdx.y;
  if (gy < x.groups)
    split_walk_body<DX, CHX, float>(x.bins, n, n_pad, nf, x.tile_nan, x.blob, x.n_chunks, x.chunk_stride, x.cpg,
                                    x.leaf_ids, x.n_trees, static_cast<float*>(x.leaves), nullptr, gy);
  else
    split_walk_body<DI, CHI, double>(f.bins, n, n_pad, nf, f.tile_nan, f.blob, f.n_chunks, f.chunk_stride, f.cpg,
                                     f.leaf_ids, f.n_trees, static_cast<double*>(f.leaves), nullptr, gy - x.groups);
  FD_TL(g_tl_forest, 4, 3);
}

// The latency pair's epilogue in ONE launch: per transaction the XGBoost margin (base + f32 leaves in tree order)
// and the IsolationForest path-length sum (f64, tree order) — split_sum_kernel's sequential sums, bit for bit —
// their probabilities (into the model-probability columns), then blend_row over every present model (the others'
// columns, e.g. the LSTM head's, read from memory) -> fraud probability, confidence, decision, risk. Replaces two
// sum launches and the blend launch.
struct PairBlendArgs {
  BlendConsts blend;
  Cols cols;      // present models' columns (present order); the two forests' entries are written here
  int pos_x, pos_f;  // present-order positions of the XGBoost / IsolationForest
  float base_margin;
  double if_offset, if_denom;
  double *fp, *conf;
  uint8_t *dec, *risk;
};

constexpr int kPairRows = 4;    // transactions per workgroup of the pair epilogue (256 workgroups for a 1 k batch)
static_assert(kPairRows == 4, "the pair epilogue stages a tree's rows as one 16-B (f32) / 32-B (f64) load");
constexpr int kPairTcX = 2048;  // XGBoost trees per LDS block (f32: 32 KiB)
constexpr int kPairTcF = 1024;  // IsolationForest trees per LDS block (f64: 32 KiB)
constexpr int kPairLoads = 4;   // trees (16 / 32-B leaf loads) in flight per thread per staging round

// One dependent global round trip for the whole epilogue: the other models' columns (e.g. the LSTM head's) and
// both forests' [trees][rows] leaf blocks are loaded together (a tree's 4 rows per 16 / 32-B load), then one wave adds
// the f32 margins and another wave the f64 path lengths, each in tree order (the sequential sums, bit for bit),
// and the probabilities go straight into blend_row (not written and read back).
__global__ void __launch_bounds__(256)
split_sum_pair_blend_kernel(const float* __restrict__ lx, int tx, const double* __restrict__ lf, int tf, int64_t n,
                            PairBlendArgs a, uint32_t* __restrict__ nan_x, uint32_t* __restrict__ nan_f) {
  constexpr int R = kPairRows;
  // row-major blocks (a row's trees contiguous: the sums read 4 / 2 leaves per ds_read_b128); the row strides are
  // 16 mod 64 banks, so the staging stores of a wave ((tree, row) = (i / 4, i % 4)) hit distinct banks
  constexpr int kSX = kPairTcX + 16, kSF = kPairTcF + 16;
  __shared__ __attribute__((aligned(16))) float bx[R * kSX];
  __shared__ __attribute__((aligned(16))) double bfl[R * kSF];
  __shared__ double fsum[R];
  FD_TL(g_tl_forest, 5, 0);
  const int tid = threadIdx.x;
  // XCD-aware rows: workgroups b and b + 8 run on the same XCD (round-robin dispatch), so give each XCD a
  // contiguous run of row blocks — the 128-B lines of a tree's leaves are then fetched into one L2, not eight
  const unsigned G = gridDim.x, xq = G / 8u, xr = G % 8u, x = blockIdx.x % 8u, k = blockIdx.x / 8u;
  const unsigned lb = (x < xr ? x * (xq + 1u) : xr * (xq + 1u) + (x - xr) * xq) + k;
  const int64_t r0 = (int64_t)lb * R;
  const int rows = (int)min<int64_t>(R, n - r0);
  const bool xrow = tid < rows;                  // wave 0: the XGBoost margin and the blend of row tid
  const bool frow = tid >= 64 && tid < 64 + rows;  // wave 1: the IsolationForest sum of row tid - 64
  double other[FD_MAX_MODELS];
#pragma unroll
  for (int m = 0; m < FD_MAX_MODELS; ++m)
    other[m] = (xrow && m < a.blend.n_models && m != a.pos_x && m != a.pos_f) ? a.cols.p[m][r0 + tid] : 0.0;
  float accx = a.base_margin;
  double accf = 0.0;
  for (int t0x = 0, t0f = 0; t0x < tx || t0f < tf; t0x += kPairTcX, t0f += kPairTcF) {
    const int tcx = max(0, min(kPairTcX, tx - t0x)), tcf = max(0, min(kPairTcF, tf - t0f));
    // one tree's R leaves per item (16 B of f32 / 32 B of f64 when the rows are aligned and complete)
    const int items = tcx + tcf;
    const bool vec = rows == R && (n % R) == 0;
    for (int base = 0; base < items; base += 256 * kPairLoads) {
      uint4 v[kPairLoads][2];
#pragma unroll
      for (int u = 0; u < kPairLoads; ++u) {
        const int i = base + u * 256 + tid;
        v[u][0] = v[u][1] = make_uint4(0u, 0u, 0u, 0u);
        if (i < tcx) {
          const float* src = lx + (size_t)(t0x + i) * n + r0;
          if (vec) {
            v[u][0] = *reinterpret_cast<const uint4*>(src);
          } else {
            unsigned w[R];
#pragma unroll
            for (int r = 0; r < R; ++r) w[r] = r < rows ? __float_as_uint(src[r]) : 0u;
            v[u][0] = make_uint4(w[0], w[1], w[2], w[3]);
          }
        } else if (i < items) {
          const double* src = lf + (size_t)(t0f + i - tcx) * n + r0;
          if (vec) {
            v[u][0] = reinterpret_cast<const uint4*>(src)[0];
            v[u][1] = reinterpret_cast<const uint4*>(src)[1];
          } else {
            unsigned long long w[R];
#pragma unroll
            for (int r = 0; r < R; ++r) w[r] = r < rows ? (unsigned long long)__double_as_longlong(src[r]) : 0ull;
            v[u][0] = make_uint4((unsigned)w[0], (unsigned)(w[0] >> 32), (unsigned)w[1], (unsigned)(w[1] >> 32));
            v[u][1] = make_uint4((unsigned)w[2], (unsigned)(w[2] >> 32), (unsigned)w[3], (unsigned)(w[3] >> 32));
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kPairLoads; ++u) {
        const int i = base + u * 256 + tid;
        if (i < tcx) {
          bx[0 * kSX + i] = __uint_as_float(v[u][0].x);
          bx[1 * kSX + i] = __uint_as_float(v[u][0].y);
          bx[2 * kSX + i] = __uint_as_float(v[u][0].z);
          bx[3 * kSX + i] = __uint_as_float(v[u][0].w);
        } else if (i < items) {
          const int t = i - tcx;
          bfl[0 * kSF + t] = __longlong_as_double((long long)(((unsigned long long)v[u][0].y << 32) | v[u][0].x));
          bfl[1 * kSF + t] = __longlong_as_double((long long)(((unsigned long long)v[u][0].w << 32) | v[u][0].z));
          bfl[2 * kSF + t] = __longlong_as_double((long long)(((unsigned long long)v[u][1].y << 32) | v[u][1].x));
          bfl[3 * kSF + t] = __longlong_as_double((long long)(((unsigned long long)v[u][1].w << 32) | v[u][1].z));
        }
      }
    }
    __syncthreads();
    if (t0x == 0) FD_TL(g_tl_forest, 5, 1);
    if (xrow) {  // tree order: 64 leaves per batch of 16 ds_read_b128
      const float4* q = reinterpret_cast<const float4*>(&bx[tid * kSX]);
      int t = 0;
      for (; t + 64 <= tcx; t += 64) {
        float4 w[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) w[u] = q[t / 4 + u];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          accx += w[u].x;
          accx += w[u].y;
          accx += w[u].z;
          accx += w[u].w;
        }
      }
      for (; t < tcx; ++t) accx += bx[tid * kSX + t];
    } else if (frow) {
      const int r = tid - 64;
      const double2* q = reinterpret_cast<const double2*>(&bfl[r * kSF]);
      int t = 0;
      for (; t + 32 <= tcf; t += 32) {
        double2 w[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) w[u] = q[t / 2 + u];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          accf += w[u].x;
          accf += w[u].y;
        }
      }
      for (; t < tcf; ++t) accf += bfl[r * kSF + t];
    }
    __syncthreads();
    if (t0x == 0) FD_TL(g_tl_forest, 5, 2);
  }
  if (frow) fsum[tid - 64] = accf;
  if (tid == 0 && r0 % kTile == 0) {  // every walk of the tile is done (stream order): clear the NaN flags
    nan_x[r0 / kTile] = 0u;
    nan_f[r0 / kTile] = 0u;
  }
  __syncthreads();
  if (!xrow) return;
  const int64_t row = r0 + tid;
  const double px = forest_prob<FD_FOREST_XGB_BINARY_LOGISTIC, float>(accx, 0.0, 0.0);
  const double pf = forest_prob<FD_FOREST_SKLEARN_IFOREST, double>(fsum[tid], a.if_offset, a.if_denom);
  const_cast<double*>(a.cols.p[a.pos_x])[row] = px;
  const_cast<double*>(a.cols.p[a.pos_f])[row] = pf;
  double raw[FD_MAX_MODELS];
#pragma unroll
  for (int m = 0; m < FD_MAX_MODELS; ++m) raw[m] = m == a.pos_x ? px : (m == a.pos_f ? pf : other[m]);
  double fp, conf;
  uint8_t dec, risk;
  blend_row(a.blend, raw, fp, conf, dec, risk);
  a.fp[row] = fp;
  if (a.conf) a.conf[row] = conf;
  if (a.dec) a.dec[row] = dec;
  if (a.risk) a.risk[row] = risk;
  FD_TL(g_tl_forest, 5, 3);
}

// 8 transactions per workgroup (128 workgroups for a 1 k batch): all 256 threads stream a [trees][8] block of
// leaf values into LDS (independent 32-B row loads), then 8 threads add them in tree order (the sequential sum)

template <int KIND, typename LeafT>
__global__ void __launch_bounds__(256)
split_sum_kernel(const LeafT* __restrict__ leaves, int64_t n, int n_trees, float base_margin, double if_offset,
                 double if_denom, double* __restrict__ out_prob, double* __restrict__ out_raw,
                 uint32_t* __restrict__ tile_nan) {
  constexpr int kTc = 65536 / (kSumRows * (int)sizeof(LeafT));  // trees per LDS block (64 KiB)
  __shared__ LeafT blk[kTc * kSumRows];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * kSumRows;
  const int rows = (int)min<int64_t>(kSumRows, n - r0);
  LeafT acc = (KIND == FD_FOREST_XGB_BINARY_LOGISTIC) ? (LeafT)base_margin : (LeafT)0;
  for (int t0 = 0; t0 < n_trees; t0 += kTc) {
    const int tc = min(kTc, n_trees - t0);
    const int total = tc * kSumRows;
    for (int base = 0; base < total; base += 256 * 16) {  // 16 independent loads in flight per thread
      LeafT v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int i = base + u * 256 + tid;
        const int t = i / kSumRows, r = i - t * kSumRows;
        v[u] = (i < total && r < rows) ? leaves[(size_t)(t0 + t) * n + r0 + r] : (LeafT)0;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int i = base + u * 256 + tid;
        if (i < total) blk[i] = v[u];
      }
    }
    __syncthreads();
    if (tid < rows) {
      int t = 0;
      for (; t + 16 <= tc; t += 16) {
        LeafT v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = blk[(t + u) * kSumRows + tid];
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += v[u];
      }
      for (; t < tc; ++t) acc += blk[t * kSumRows + tid];
    }
    __syncthreads();
  }
  if (tid < rows) write_outputs<KIND, LeafT>(acc, r0 + tid, if_offset, if_denom, out_prob, out_raw);
  if (tid == 0 && r0 % kTile == 0) tile_nan[r0 / kTile] = 0u;  // every walk of the tile is done (stream order)
}

// ------------------------------------------------------------------------------------------------
// dispatch

using KernelFn = void (*)(const float*, int64_t, int, int, const char*, int, int, const int32_t*, int,
                          float, double, double, double*, double*, int32_t*);

template <typename LeafT, int KIND, int CH>
KernelFn pick1_ch(int D) {
  switch (D) {
    case 1: return forest_kernel1<1, CH, LeafT, KIND>;
    case 2: return forest_kernel1<2, CH, LeafT, KIND>;
    case 3: return forest_kernel1<3, CH, LeafT, KIND>;
    case 4: return forest_kernel1<4, CH, LeafT, KIND>;
    case 5: return forest_kernel1<5, CH, LeafT, KIND>;
    case 6: return forest_kernel1<6, CH, LeafT, KIND>;
    case 7: return forest_kernel1<7, CH, LeafT, KIND>;
    case 8: return forest_kernel1<8, CH, LeafT, KIND>;
    case 9: return forest_kernel1<9, CH, LeafT, KIND>;
    case 10: return forest_kernel1<10, CH, LeafT, KIND>;
    default: return nullptr;
  }
}

template <typename LeafT, int KIND>
KernelFn pick1(int D, int CH) {
  switch (CH) {
    case 1: return pick1_ch<LeafT, KIND, 1>(D);
    case 2: return pick1_ch<LeafT, KIND, 2>(D);
    case 4: return pick1_ch<LeafT, KIND, 4>(D);
    case 8: return pick1_ch<LeafT, KIND, 8>(D);
    case 12: return pick1_ch<LeafT, KIND, 12>(D);
    case 16: return pick1_ch<LeafT, KIND, 16>(D);
    default: return nullptr;
  }
}

template <typename LeafT, int KIND, int CH>
KernelFn pick3_ch(int D) {
  switch (D) {
    case 1: return forest_kernel3<1, CH, LeafT, KIND>;
    case 2: return forest_kernel3<2, CH, LeafT, KIND>;
    case 3: return forest_kernel3<3, CH, LeafT, KIND>;
    case 4: return forest_kernel3<4, CH, LeafT, KIND>;
    case 5: return forest_kernel3<5, CH, LeafT, KIND>;
    case 6: return forest_kernel3<6, CH, LeafT, KIND>;
    case 7: return forest_kernel3<7, CH, LeafT, KIND>;
    case 8: return forest_kernel3<8, CH, LeafT, KIND>;
    default: return nullptr;
  }
}

template <typename LeafT, int KIND>
KernelFn pick3(int D, int CH) {
  switch (CH) {
    case 4: return pick3_ch<LeafT, KIND, 4>(D);
    case 8: return pick3_ch<LeafT, KIND, 8>(D);
    case 12: return pick3_ch<LeafT, KIND, 12>(D);
    case 16: return pick3_ch<LeafT, KIND, 16>(D);
    default: return nullptr;
  }
}

using KernelFn4 = void (*)(const float*, int64_t, int, int, const char*, int, int, const int32_t*, int,
                           const float*, const int32_t*, int, float, double, double, double*, double*, int32_t*);

template <typename LeafT, int KIND, int CH>
KernelFn4 pick4_ch(int D) {
  switch (D) {
    case 1: return forest_kernel4<1, CH, LeafT, KIND>;
    case 2: return forest_kernel4<2, CH, LeafT, KIND>;
    case 3: return forest_kernel4<3, CH, LeafT, KIND>;
    case 4: return forest_kernel4<4, CH, LeafT, KIND>;
    case 5: return forest_kernel4<5, CH, LeafT, KIND>;
    case 6: return forest_kernel4<6, CH, LeafT, KIND>;
    case 7: return forest_kernel4<7, CH, LeafT, KIND>;
    case 8: return forest_kernel4<8, CH, LeafT, KIND>;
    default: return nullptr;
  }
}

template <typename LeafT, int KIND>
KernelFn4 pick4(int D, int CH) {
  switch (CH) {
    case 4: return pick4_ch<LeafT, KIND, 4>(D);
    case 8: return pick4_ch<LeafT, KIND, 8>(D);
    case 12: return pick4_ch<LeafT, KIND, 12>(D);
    case 16: return pick4_ch<LeafT, KIND, 16>(D);
    default: return nullptr;
  }
}

template <int D, typename LeafT>
void* pick_split_ch(int CH) {
  switch (CH) {
    case 4: return (void*)split_walk_kernel<D, 4, LeafT>;
    case 8: return (void*)split_walk_kernel<D, 8, LeafT>;
    case 12: return (void*)split_walk_kernel<D, 12, LeafT>;
    case 16: return (void*)split_walk_kernel<D, 16, LeafT>;
    default: return nullptr;
  }
}

template <typename LeafT>
void* pick_split(int D, int CH) {
  switch (D) {
    case 1: return pick_split_ch<1, LeafT>(CH);
    case 2: return pick_split_ch<2, LeafT>(CH);
    case 3: return pick_split_ch<3, LeafT>(CH);
    case 4: return pick_split_ch<4, LeafT>(CH);
    case 5: return pick_split_ch<5, LeafT>(CH);
    case 6: return pick_split_ch<6, LeafT>(CH);
    case 7: return pick_split_ch<7, LeafT>(CH);
    case 8: return pick_split_ch<8, LeafT>(CH);
    default: return nullptr;
  }
}

using KernelFn6 = void (*)(const float*, int64_t, int, int, const char*, int, int, const int32_t*, int,
                           const float*, const int32_t*, int, float, double, double, double*, double*, int32_t*,
                           const void*);

template <typename LeafT, int KIND, int CH>
KernelFn6 pick6_ch(int D) {
  switch (D) {
    case 1: return (KernelFn6)forest_kernel6<1, CH, LeafT, KIND>;
    case 2: return (KernelFn6)forest_kernel6<2, CH, LeafT, KIND>;
    case 3: return (KernelFn6)forest_kernel6<3, CH, LeafT, KIND>;
    case 4: return (KernelFn6)forest_kernel6<4, CH, LeafT, KIND>;
    case 5: return (KernelFn6)forest_kernel6<5, CH, LeafT, KIND>;
    case 6: return (KernelFn6)forest_kernel6<6, CH, LeafT, KIND>;
    case 7: return (KernelFn6)forest_kernel6<7, CH, LeafT, KIND>;
    case 8: return (KernelFn6)forest_kernel6<8, CH, LeafT, KIND>;
    default: return nullptr;
  }
}

template <typename LeafT, int KIND>
KernelFn6 pick6(int D, int CH) {
  switch (CH) {
    case 16: return pick6_ch<LeafT, KIND, 16>(D);
    case 24: return pick6_ch<LeafT, KIND, 24>(D);
    case 32: return pick6_ch<LeafT, KIND, 32>(D);
    default: return nullptr;
  }
}

// small-batch launch: bin once, walk (tiles x chunk groups), sequential sum
// stage 1: the forest's scratch for this batch (NaN tile flags zeroed when allocated, cleared after each use)
template <typename LeafT>
SplitBinArgs split_prepare(const PackedForest& pf, int64_t n, int64_t tiles, hipStream_t stream) {
  const int64_t n_pad = tiles * kTile;
  SplitScratch& sc = pf.split;  // per forest: two forests may run concurrently on different streams
  sc.bins.ensure((size_t)pf.num_feature * n_pad * 4);
  if (sc.nan.bytes < (size_t)tiles * 4) {
    sc.nan.ensure((size_t)tiles * 4);
    FD_HIP(hipMemsetAsync(sc.nan.ptr, 0, sc.nan.bytes, stream));
  }
  sc.leaves.ensure((size_t)pf.n_trees * n * sizeof(LeafT));
  return SplitBinArgs{pf.b_thr.as<const float>(), pf.b_thr_off.as<const int32_t>(), sc.bins.as<uint32_t>(),
                      sc.nan.as<uint32_t>(), pf.num_feature};
}

// stage 3: walk (tiles x chunk groups) over the binned rows, then the sequential sum
template <typename LeafT, int KIND>
void split_walk_sum(const PackedForest& pf, int64_t n, double* d_prob, double* d_raw, int32_t* d_leaf, int64_t tiles,
                    hipStream_t stream) {
  const int64_t n_pad = tiles * kTile;
  SplitScratch& sc = pf.split;
  // chunk groups: enough workgroups to cover the CUs (tiles x groups >= 256)
  const int want = (int)std::max<int64_t>(1, (256 + tiles - 1) / tiles);
  const int cpg = std::max(1, (pf.b_n_chunks + want - 1) / want);
  const int groups = (pf.b_n_chunks + cpg - 1) / cpg;
  void* fn = pick_split<LeafT>(pf.depth, pf.b_chunk);
  FD_REQUIRE(fn != nullptr, FD_ERR_UNSUPPORTED, "no split forest kernel for this depth/chunk");
  const size_t lds = (size_t)pf.num_feature * 1024 + 2 * pf.b_chunk_stride + 1024;
  FD_REQUIRE(lds <= kLdsBudget, FD_ERR_UNSUPPORTED, "split forest kernel exceeds the LDS budget");
  FD_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  using WalkFn = void (*)(const uint32_t*, int64_t, int64_t, int, const uint32_t*, const char*, int, int, int,
                          const int32_t*, int, LeafT*, int32_t*);
  hipLaunchKernelGGL((WalkFn)fn, dim3((unsigned)tiles, (unsigned)groups), dim3(kWG3), lds, stream,
                     sc.bins.as<const uint32_t>(), n, n_pad, pf.num_feature, sc.nan.as<const uint32_t>(),
                     pf.b_blob.as<const char>(), pf.b_n_chunks, (int)pf.b_chunk_stride, cpg,
                     pf.leaf_ids.as<const int32_t>(), pf.n_trees, sc.leaves.as<LeafT>(), d_leaf);
  FD_HIP(hipGetLastError());
  hipLaunchKernelGGL((split_sum_kernel<KIND, LeafT>), dim3((unsigned)((n + kSumRows - 1) / kSumRows)), dim3(256), 0,
                     stream, sc.leaves.as<const LeafT>(), n, pf.n_trees, pf.base_margin, pf.if_offset,
                     pf.if_denominator, d_prob, d_raw, sc.nan.as<uint32_t>());
  FD_HIP(hipGetLastError());
}

template <typename LeafT, int KIND>
void launch_split(Engine& e, const PackedForest& pf, const float* d_X, int64_t n, int32_t ld, double* d_prob,
                  double* d_raw, int32_t* d_leaf, int64_t tiles, hipStream_t stream) {
  (void)e;
  const SplitBinArgs a = split_prepare<LeafT>(pf, n, tiles, stream);
  hipLaunchKernelGGL(split_bin_kernel, dim3((unsigned)(tiles * kTile / kSplitBin), (unsigned)pf.num_feature),
                     dim3(kSplitBin), 0, stream, d_X, n, tiles * kTile, (int)ld, pf.num_feature, a.thr, a.thr_off,
                     pf.bin_steps, a.bins, a.tile_nan);
  FD_HIP(hipGetLastError());
  split_walk_sum<LeafT, KIND>(pf, n, d_prob, d_raw, d_leaf, tiles, stream);
}

bool split_path(const Engine& e, const PackedForest& pf, int64_t n) {
  const int64_t blocks = (n + kTile - 1) / kTile;
  const bool ok_split = pf.binned && pf.depth <= 8 && pf.b_chunk % 4 == 0;
  return ok_split && (e.forest_variant == 6 || (e.forest_variant == 0 && blocks < kSplitTiles));
}

}  // namespace

#ifdef FD_FOREST_PROFILE
extern "C" __attribute__((visibility("default"))) int fd_debug_forest_profile(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * (size_t)n);
}
extern "C" __attribute__((visibility("default"))) int fd_debug_tl_forest(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(fd::g_tl_forest), sizeof(fd::g_tl_forest));
}
#endif

// Kernel choice (option "forest_kernel"): 0 auto = kernel 6 when the binned node-only layout exists
// (depth <= 8, <= 65534 distinct thresholds per feature; config 2: 84.1 vs kernel 4's 88.2 us, config-3
// IsolationForest 38.1 vs 38.7 us, tools/forest_sweep.py), else kernel 4 (binned), else kernel 3
// (depth <= 8), else kernel 1; 8 forces kernel 6; 1/2/3 force kernel 1/3/4; 6 forces the tree-split
// small-batch path, which auto also takes below kSplitTiles tiles (FD_ERR_UNSUPPORTED when the forest
// cannot use it).
// Two forests of a latency batch on one stream (score_matrix, small_streams 0): one binning launch for both,
// then each forest's walk and sum. false: not applicable (a forest off the split path); nothing launched.
bool launch_forest_pair(Engine& e, const PackedForest& pa, const PackedForest& pb, const float* d_X, int64_t n,
                        int32_t ld, double* d_prob_a, double* d_prob_b) {
  if (n == 0 || !split_path(e, pa, n) || !split_path(e, pb, n) || &pa == &pb) return false;
  FD_REQUIRE(d_X && d_prob_a && d_prob_b && ld > 0, FD_ERR_INVALID_ARG, "null buffer or bad ld");
  const int64_t tiles = (n + kTile - 1) / kTile;
  const hipStream_t st = e.stream;
  const bool xa = pa.kind == FD_FOREST_XGB_BINARY_LOGISTIC, xb = pb.kind == FD_FOREST_XGB_BINARY_LOGISTIC;
  Engine::Timed* ev = e.timing ? e.next_event_pair(xa ? FD_TIMING_XGB : FD_TIMING_IFOREST) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, st));  // the first forest's time includes the shared binning
  const SplitBinArgs a = xa ? split_prepare<float>(pa, n, tiles, st) : split_prepare<double>(pa, n, tiles, st);
  const SplitBinArgs b = xb ? split_prepare<float>(pb, n, tiles, st) : split_prepare<double>(pb, n, tiles, st);
  hipLaunchKernelGGL(split_bin_pair_kernel, dim3((unsigned)(tiles * kTile / kSplitBin), (unsigned)(a.nf + b.nf)),
                     dim3(kSplitBin), 0, st, d_X, n, tiles * kTile, (int)ld, a, b);
  FD_HIP(hipGetLastError());
  if (xa)
    split_walk_sum<float, FD_FOREST_XGB_BINARY_LOGISTIC>(pa, n, d_prob_a, nullptr, nullptr, tiles, st);
  else
    split_walk_sum<double, FD_FOREST_SKLEARN_IFOREST>(pa, n, d_prob_a, nullptr, nullptr, tiles, st);
  if (ev) FD_HIP(hipEventRecord(ev->b, st));
  ev = e.timing ? e.next_event_pair(xb ? FD_TIMING_XGB : FD_TIMING_IFOREST) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, st));
  if (xb)
    split_walk_sum<float, FD_FOREST_XGB_BINARY_LOGISTIC>(pb, n, d_prob_b, nullptr, nullptr, tiles, st);
  else
    split_walk_sum<double, FD_FOREST_SKLEARN_IFOREST>(pb, n, d_prob_b, nullptr, nullptr, tiles, st);
  if (ev) FD_HIP(hipEventRecord(ev->b, st));
  return true;
}

namespace {
template <int CHX>
const void* pick_walk_pair_i(int chi) {
  switch (chi) {
    case 4: return (const void*)split_walk_pair_kernel<8, CHX, 8, 4>;
    case 8: return (const void*)split_walk_pair_kernel<8, CHX, 8, 8>;
    case 12: return (const void*)split_walk_pair_kernel<8, CHX, 8, 12>;
    case 16: return (const void*)split_walk_pair_kernel<8, CHX, 8, 16>;
    default: return nullptr;
  }
}
const void* pick_walk_pair(int chx, int chi) {
  switch (chx) {
    case 4: return pick_walk_pair_i<4>(chi);
    case 8: return pick_walk_pair_i<8>(chi);
    case 12: return pick_walk_pair_i<12>(chi);
    case 16: return pick_walk_pair_i<16>(chi);
    default: return nullptr;
  }
}

// chunk groups of one forest's walk over `tiles` tiles: enough workgroups to cover the CUs (as split_walk_sum)
void walk_groups(const PackedForest& pf, int64_t tiles, int& cpg, int& groups) {
  const int want = (int)std::max<int64_t>(1, (256 + tiles - 1) / tiles);
  cpg = std::max(1, (pf.b_n_chunks + want - 1) / want);
  groups = (pf.b_n_chunks + cpg - 1) / cpg;
}

// The pair path's forests (XGBoost first) and its walk kernel, or false when it does not apply
bool pair_blend_plan(const Engine& e, const PackedForest& p1, const PackedForest& p2, int64_t n,
                     const PackedForest*& xf, const PackedForest*& ff, const void*& walk, size_t& lds) {
  if (n == 0 || &p1 == &p2 || !split_path(e, p1, n) || !split_path(e, p2, n)) return false;
  const bool x1 = p1.kind == FD_FOREST_XGB_BINARY_LOGISTIC, x2 = p2.kind == FD_FOREST_XGB_BINARY_LOGISTIC;
  if (x1 == x2) return false;  // one XGBoost and one IsolationForest
  const PackedForest& X = x1 ? p1 : p2;
  const PackedForest& F = x1 ? p2 : p1;
  if (X.depth != 8 || F.depth != 8 || X.num_feature != F.num_feature) return false;
  walk = pick_walk_pair(X.b_chunk, F.b_chunk);
  if (!walk) return false;
  lds = (size_t)X.num_feature * 1024 + 2 * std::max(X.b_chunk_stride, F.b_chunk_stride) + 1024;
  if (lds > kLdsBudget) return false;
  xf = &X;
  ff = &F;
  return true;
}
}  // namespace

bool forest_pair_prebin(Engine& e, const PackedForest& p1, const PackedForest& p2, const float* d_X, int64_t n,
                        int32_t ld) {
  PreBin& pb = e.prebin;
  pb.want = pb.done = false;
  const PackedForest *xf = nullptr, *ff = nullptr;
  const void* walk = nullptr;
  size_t lds = 0;
  if (!e.latency_prebin || !pair_blend_plan(e, p1, p2, n, xf, ff, walk, lds)) return false;
  const int64_t tiles = (n + kTile - 1) / kTile;
  const SplitBinArgs a = split_prepare<float>(*xf, n, tiles, e.stream);
  const SplitBinArgs b = split_prepare<double>(*ff, n, tiles, e.stream);
  pb.thr[0] = a.thr, pb.thr[1] = b.thr;
  pb.thr_off[0] = a.thr_off, pb.thr_off[1] = b.thr_off;
  pb.bins[0] = a.bins, pb.bins[1] = b.bins;
  pb.nan[0] = a.tile_nan, pb.nan[1] = b.tile_nan;
  pb.nf[0] = a.nf, pb.nf[1] = b.nf;
  pb.steps[0] = xf->bin_steps, pb.steps[1] = ff->bin_steps;
  pb.thr_nonempty = xf->b_thr.bytes >= sizeof(float) && ff->b_thr.bytes >= sizeof(float) && xf->bin_steps > 0 &&
                    ff->bin_steps > 0;
  pb.n = n;
  pb.n_pad = tiles * kTile;
  pb.ld = ld;
  pb.fx = xf;
  pb.ff = ff;
  pb.X = d_X;
  pb.want = true;
  return true;
}

bool launch_forest_pair_blend(Engine& e, const PackedForest& p1, const PackedForest& p2, const float* d_X, int64_t n,
                              int32_t ld, const BlendConsts& bc, const double* const* cols, int pos1, int pos2,
                              double* dfp, double* dconf, uint8_t* ddec, uint8_t* drisk, hipEvent_t before_blend) {
  const PackedForest *xf = nullptr, *ff = nullptr;
  const void* walk = nullptr;
  size_t lds = 0;
  // the bins of an LSTM launch that binned these vectors for this pair (PreBin), consumed here
  const bool prebinned = e.prebin.done && e.prebin.X == d_X && e.prebin.n == n && e.prebin.ld == ld;
  const void* pre_fx = e.prebin.fx;
  const void* pre_ff = e.prebin.ff;
  e.prebin.want = e.prebin.done = false;
  if (!pair_blend_plan(e, p1, p2, n, xf, ff, walk, lds)) return false;
  const PackedForest& X = *xf;
  const PackedForest& F = *ff;
  const int nf = X.num_feature;
  FD_REQUIRE(d_X && dfp && cols && ld > 0, FD_ERR_INVALID_ARG, "null buffer or bad ld");
  const int64_t tiles = (n + kTile - 1) / kTile, n_pad = tiles * kTile;
  const hipStream_t st = e.stream;
  Engine::Timed* ev = e.timing ? e.next_event_pair(FD_TIMING_XGB) : nullptr;  // the pair's launches
  if (ev) FD_HIP(hipEventRecord(ev->a, st));
  const SplitBinArgs a = split_prepare<float>(X, n, tiles, st);
  const SplitBinArgs b = split_prepare<double>(F, n, tiles, st);
  if (prebinned && pre_fx == &X && pre_ff == &F) {
    ++e.prebin_total;
  } else {
    hipLaunchKernelGGL(split_bin_pair_kernel, dim3((unsigned)(tiles * kTile / kSplitBin), (unsigned)(a.nf + b.nf)),
                       dim3(kSplitBin), 0, st, d_X, n, n_pad, (int)ld, a, b);
    FD_HIP(hipGetLastError());
  }
  SplitWalkArgs wx{}, wf{};
  wx.bins = a.bins;
  wx.tile_nan = a.tile_nan;
  wx.blob = X.b_blob.as<const char>();
  wx.n_chunks = X.b_n_chunks;
  wx.chunk_stride = (int)X.b_chunk_stride;
  walk_groups(X, tiles, wx.cpg, wx.groups);
  wx.leaf_ids = X.leaf_ids.as<const int32_t>();
  wx.n_trees = X.n_trees;
  wx.leaves = X.split.leaves.ptr;
  wf.bins = b.bins;
  wf.tile_nan = b.tile_nan;
  wf.blob = F.b_blob.as<const char>();
  wf.n_chunks = F.b_n_chunks;
  wf.chunk_stride = (int)F.b_chunk_stride;
  walk_groups(F, tiles, wf.cpg, wf.groups);
  wf.leaf_ids = F.leaf_ids.as<const int32_t>();
  wf.n_trees = F.n_trees;
  wf.leaves = F.split.leaves.ptr;
  FD_HIP(hipFuncSetAttribute(walk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  void* wargs[] = {&n, const_cast<int64_t*>(&n_pad), const_cast<int*>(&nf), &wx, &wf};
  FD_HIP(hipLaunchKernel(walk, dim3((unsigned)tiles, (unsigned)(wx.groups + wf.groups)), dim3(kWG3), wargs, lds, st));
  PairBlendArgs pa{};
  pa.blend = bc;
  for (int m = 0; m < bc.n_models; ++m) pa.cols.p[m] = cols[m];
  const bool x1 = &X == &p1;
  pa.pos_x = x1 ? pos1 : pos2;
  pa.pos_f = x1 ? pos2 : pos1;
  pa.base_margin = X.base_margin;
  pa.if_offset = F.if_offset;
  pa.if_denom = F.if_denominator;
  pa.fp = dfp;
  pa.conf = dconf;
  pa.dec = ddec;
  pa.risk = drisk;
  if (before_blend) FD_HIP(hipStreamWaitEvent(st, before_blend, 0));  // e.g. the LSTM head on a side stream
  hipLaunchKernelGGL(split_sum_pair_blend_kernel, dim3((unsigned)((n + kPairRows - 1) / kPairRows)), dim3(256), 0, st,
                     X.split.leaves.as<const float>(), X.n_trees, F.split.leaves.as<const double>(), F.n_trees, n, pa,
                     a.tile_nan, b.tile_nan);
  FD_HIP(hipGetLastError());
  if (ev) FD_HIP(hipEventRecord(ev->b, st));
  return true;
}

void launch_forest(Engine& e, const PackedForest& pf, const float* d_X, int64_t n, int32_t ld,
                   double* d_prob, double* d_raw, int32_t* d_leaf, hipStream_t stream) {
  FD_REQUIRE(d_X && d_prob && ld > 0, FD_ERR_INVALID_ARG, "null buffer or bad ld");
  if (n == 0) return;
  const bool xgb = pf.kind == FD_FOREST_XGB_BINARY_LOGISTIC;
  const size_t leaf_sz = xgb ? sizeof(float) : sizeof(double);
  const int64_t blocks = (n + kTile - 1) / kTile;
  FD_REQUIRE(blocks < (1ll << 31), FD_ERR_INVALID_ARG, "batch too large");
  const int v = e.forest_variant;
  FD_REQUIRE(v == 0 || v == 1 || v == 2 || v == 3 || v == 6 || v == 8, FD_ERR_INVALID_ARG,
             "forest_kernel option must be 0, 1, 2, 3, 6 or 8");
  Engine::Timed* ev = nullptr;

  // small batches: tree-split latency path (option 6 forces it; auto below 128 tiles)
  const bool ok_split = pf.binned && pf.depth <= 8 && pf.b_chunk % 4 == 0;
  if (v == 6) FD_REQUIRE(ok_split, FD_ERR_UNSUPPORTED, "the split forest path needs the binned layout (depth <= 8)");
  if ((v == 6 || (v == 0 && blocks < kSplitTiles)) && ok_split) {
    const hipStream_t st = stream ? stream : e.stream;
    ev = e.timing ? e.next_event_pair(xgb ? FD_TIMING_XGB : FD_TIMING_IFOREST) : nullptr;
    if (ev) FD_HIP(hipEventRecord(ev->a, st));
    if (xgb)
      launch_split<float, FD_FOREST_XGB_BINARY_LOGISTIC>(e, pf, d_X, n, ld, d_prob, d_raw, d_leaf, blocks, st);
    else
      launch_split<double, FD_FOREST_SKLEARN_IFOREST>(e, pf, d_X, n, ld, d_prob, d_raw, d_leaf, blocks, st);
    if (ev) FD_HIP(hipEventRecord(ev->b, st));
    return;
  }

  // large batches without leaf ids: the fused ensemble kernel over this one forest (its u16 merged-bin tile,
  // link-encoded nodes and LDS-staged leaves; the same f32 margin / f64 path-length sums in tree order)
  if (v == 0 && !d_leaf) {
    const int slot = (int)(&pf - e.forests);
    if (slot >= 0 && slot < kMaxSlots && launch_ensemble_single(e, slot, d_X, n, ld, d_prob, d_raw, stream)) return;
  }

  // + 64 B: kernel 6's two item counters after the tile_any flags
  const size_t lds6 = pf.n_chunk ? lds_bytes_kernel3(pf.num_feature, pf.n_chunk_stride, pf.n_chunk, leaf_sz) + 64 : 0;
  const bool ok6 = pf.binned && pf.n_chunk > 0 && pf.depth <= 8 && lds6 <= kLdsBudget;
  if (v == 8)
    FD_REQUIRE(ok6, FD_ERR_UNSUPPORTED, "forest kernel 6 needs the binned node-only layout (depth <= 8)");
  if ((v == 0 || v == 8) && ok6) {
    KernelFn6 fn = xgb ? pick6<float, FD_FOREST_XGB_BINARY_LOGISTIC>(pf.depth, pf.n_chunk)
                       : pick6<double, FD_FOREST_SKLEARN_IFOREST>(pf.depth, pf.n_chunk);
    FD_REQUIRE(fn != nullptr, FD_ERR_UNSUPPORTED, "no forest kernel 6 for this depth/chunk");
    FD_HIP(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds6));
    ev = e.timing ? e.next_event_pair(xgb ? FD_TIMING_XGB : FD_TIMING_IFOREST) : nullptr;
    if (ev) FD_HIP(hipEventRecord(ev->a, e.stream));
    hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(kWG3), lds6, e.stream, d_X, n, (int)ld, pf.num_feature,
                       pf.n_blob.as<const char>(), pf.n_n_chunks, (int)pf.n_chunk_stride,
                       pf.leaf_ids.as<const int32_t>(), pf.n_trees, pf.b_thr.as<const float>(),
                       pf.b_thr_off.as<const int32_t>(), pf.bin_steps, pf.base_margin, pf.if_offset,
                       pf.if_denominator, d_prob, d_raw, d_leaf, (const void*)pf.n_leaves.ptr);
    FD_HIP(hipGetLastError());
    if (ev) FD_HIP(hipEventRecord(ev->b, e.stream));
    return;
  }

  const size_t lds4 = pf.binned ? lds_bytes_kernel4(pf.num_feature, pf.b_chunk_stride, pf.b_chunk, leaf_sz) : 0;
  const bool ok4 = pf.binned && pf.depth <= 8 && pf.b_chunk % 4 == 0 && lds4 <= kLdsBudget;
  if (v == 3) FD_REQUIRE(ok4, FD_ERR_UNSUPPORTED, "forest kernel 4 needs the binned layout (depth <= 8)");
  if ((v == 0 || v == 3) && ok4) {
    KernelFn4 fn = xgb ? pick4<float, FD_FOREST_XGB_BINARY_LOGISTIC>(pf.depth, pf.b_chunk)
                       : pick4<double, FD_FOREST_SKLEARN_IFOREST>(pf.depth, pf.b_chunk);
    FD_REQUIRE(fn != nullptr, FD_ERR_UNSUPPORTED, "no forest kernel 4 for this depth/chunk");
    FD_HIP(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds4));
    ev = e.timing ? e.next_event_pair(xgb ? FD_TIMING_XGB : FD_TIMING_IFOREST) : nullptr;
    if (ev) FD_HIP(hipEventRecord(ev->a, e.stream));
    hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(kWG3), lds4, e.stream, d_X, n, (int)ld, pf.num_feature,
                       pf.b_blob.as<const char>(), pf.b_n_chunks, (int)pf.b_chunk_stride,
                       pf.leaf_ids.as<const int32_t>(), pf.n_trees, pf.b_thr.as<const float>(),
                       pf.b_thr_off.as<const int32_t>(), pf.bin_steps, pf.base_margin, pf.if_offset,
                       pf.if_denominator, d_prob, d_raw, d_leaf);
    FD_HIP(hipGetLastError());
    if (ev) FD_HIP(hipEventRecord(ev->b, e.stream));
    return;
  }

  KernelFn fn = nullptr;
  int threads = kTile;
  size_t lds = 0;
  const size_t lds3 = lds_bytes_kernel3(pf.num_feature, pf.chunk_stride, pf.chunk, leaf_sz);
  const bool ok3 = pf.depth <= 8 && pf.chunk % 4 == 0 && lds3 <= kLdsBudget;
  if (v == 2) FD_REQUIRE(ok3, FD_ERR_UNSUPPORTED, "forest kernel 3 does not fit this forest");
  if (v != 1 && ok3) {
    fn = xgb ? pick3<float, FD_FOREST_XGB_BINARY_LOGISTIC>(pf.depth, pf.chunk)
             : pick3<double, FD_FOREST_SKLEARN_IFOREST>(pf.depth, pf.chunk);
    threads = kWG3;
    lds = lds3;
  }
  if (!fn) {
    fn = xgb ? pick1<float, FD_FOREST_XGB_BINARY_LOGISTIC>(pf.depth, pf.chunk)
             : pick1<double, FD_FOREST_SKLEARN_IFOREST>(pf.depth, pf.chunk);
    lds = lds_bytes_kernel1(pf.num_feature, pf.chunk_stride);
  }
  FD_REQUIRE(fn != nullptr, FD_ERR_UNSUPPORTED, "no forest kernel for this depth/chunk");
  FD_REQUIRE(lds <= kLdsBudget, FD_ERR_UNSUPPORTED, "LDS budget exceeded");
  FD_HIP(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  ev = e.timing ? e.next_event_pair(xgb ? FD_TIMING_XGB : FD_TIMING_IFOREST) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, e.stream));
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(threads), lds, e.stream, d_X, n, (int)ld, pf.num_feature,
                     pf.blob.as<const char>(), pf.n_chunks, (int)pf.chunk_stride, pf.leaf_ids.as<const int32_t>(),
                     pf.n_trees, pf.base_margin, pf.if_offset, pf.if_denominator, d_prob, d_raw, d_leaf);
  FD_HIP(hipGetLastError());
  if (ev) FD_HIP(hipEventRecord(ev->b, e.stream));
}

}  // namespace fd
