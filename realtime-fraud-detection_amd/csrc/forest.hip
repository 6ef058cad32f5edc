// forest.hip — repacking and batched inference of the two tree ensembles on the hot path:
//   * XGBoost 2.0.3 gbtree / binary:logistic  (reference: ml/models/model_manager.py:157-161, 309-311)
//   * scikit-learn IsolationForest            (reference: ml/models/model_manager.py:197-200, 338-346;
//                                              sklearn/ensemble/_iforest.py _compute_score_samples)
//
// Kernel shape (gfx950):
//   one workgroup = 256 threads = a tile of 256 transactions, one transaction per lane;
//   the tile's features live in LDS as [feature][256] f32, so a lane reading ANY feature hits bank
//   (lane mod 32): every feature gather is conflict-free whatever split feature each lane is at;
//   trees stream through two LDS buffers of CH trees each by LDS-DMA (global_load_lds_dwordx4), the
//   next chunk landing while the current one is walked;
//   every lane walks the CH trees of a chunk together (CH independent dependency chains = the ILP
//   that hides LDS latency), one level per step, branch-free on a perfect depth-D layout;
//   leaf values are added in tree order, so the XGBoost margin is the same f32 sequence the
//   reference's CPU predictor sums (bit-exact), and the IF path-length sum the same f64 sequence
//   sklearn's `depths +=` loop sums.
#include <cmath>
#include <cstring>
#include <algorithm>

#include "fd_internal.h"

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

int chunk_for_depth(int D) { return D <= 8 ? 8 : (D == 9 ? 4 : 2); }

}  // namespace

HostPack pack_forest_host(const fd_forest_params& p, const fd_tree_arrays& t) {
  FD_REQUIRE(p.kind == FD_FOREST_XGB_BINARY_LOGISTIC || p.kind == FD_FOREST_SKLEARN_IFOREST,
             FD_ERR_INVALID_ARG, "unknown forest kind");
  FD_REQUIRE(t.n_trees > 0 && t.tree_offsets && t.left && t.right && t.feature && t.threshold &&
                 t.leaf_value,
             FD_ERR_INVALID_ARG, "incomplete tree arrays");
  FD_REQUIRE(p.num_feature > 0 && p.num_feature <= kMaxFeatures, FD_ERR_UNSUPPORTED,
             "num_feature must be in [1, 64]");
  const bool xgb = p.kind == FD_FOREST_XGB_BINARY_LOGISTIC;
  const int T = t.n_trees;
  int D = 1;
  for (int i = 0; i < T; ++i) {
    const int64_t a = t.tree_offsets[i], b = t.tree_offsets[i + 1];
    FD_REQUIRE(b > a, FD_ERR_INVALID_ARG, "empty tree");
    D = std::max(D, tree_depth(t.left + a, t.right + a, b - a));
  }
  const int NI = (1 << D) - 1, NL = 1 << D;
  const int CH = chunk_for_depth(D);
  const size_t leaf_sz = xgb ? sizeof(float) : sizeof(double);
  const size_t tree_bytes = (size_t)NI * 8 + (size_t)NL * leaf_sz;
  const size_t chunk_stride = ((CH * tree_bytes) + 1023) / 1024 * 1024;
  const int n_chunks = (T + CH - 1) / CH;
  HostPack hp;
  hp.blob.assign(n_chunks * chunk_stride, 0);  // padding trees: all-zero nodes/leaves
  hp.leaf_ids.assign((size_t)n_chunks * CH * NL, -1);
  std::vector<int32_t> cur(NI + NL);

  for (int i = 0; i < T; ++i) {
    const int64_t a = t.tree_offsets[i], m = t.tree_offsets[i + 1] - a;
    const int32_t* L = t.left + a;
    const int32_t* R = t.right + a;
    const int32_t* F = t.feature + a;
    const double* TH = t.threshold + a;
    const uint8_t* DL = t.default_left ? t.default_left + a : nullptr;
    const double* LV = t.leaf_value + a;
    char* tb = hp.blob.data() + (size_t)(i / CH) * chunk_stride + (size_t)(i % CH) * tree_bytes;
    uint32_t* nodes = reinterpret_cast<uint32_t*>(tb);
    char* leaves = tb + (size_t)NI * 8;
    cur[0] = 0;
    for (int s = 0; s < NI; ++s) {
      const int32_t o = cur[s];
      if (L[o] < 0) {  // leaf above depth D: pad node, both subtrees resolve to the same leaf
        nodes[2 * s] = 0;
        nodes[2 * s + 1] = 0;
        cur[2 * s + 1] = o;
        cur[2 * s + 2] = o;
      } else {
        FD_REQUIRE(R[o] >= 0 && R[o] < m && L[o] < m, FD_ERR_INVALID_ARG, "bad child index");
        FD_REQUIRE(F[o] >= 0 && F[o] < p.num_feature, FD_ERR_INVALID_ARG,
                   "split feature outside [0, num_feature)");
        const float thr = xgb ? (float)TH[o] : sklearn_threshold_to_lt(TH[o]);
        uint32_t tb32;
        std::memcpy(&tb32, &thr, 4);
        const uint32_t dl = (DL && DL[o]) ? 1u : 0u;
        nodes[2 * s] = tb32;
        nodes[2 * s + 1] = (uint32_t)F[o] * (uint32_t)(kTile * 4) | (dl << 31);
        cur[2 * s + 1] = L[o];
        cur[2 * s + 2] = R[o];
      }
    }
    for (int s = 0; s < NL; ++s) {
      const int32_t o = cur[NI + s];
      FD_REQUIRE(L[o] < 0, FD_ERR_INVALID_ARG, "internal node at maximum depth");
      if (xgb) {
        const float v = (float)LV[o];
        std::memcpy(leaves + s * 4, &v, 4);
      } else {
        const double v = LV[o];
        std::memcpy(leaves + s * 8, &v, 8);
      }
      hp.leaf_ids[(size_t)i * NL + s] = o;
    }
  }
  hp.kind = p.kind;
  hp.n_trees = T;
  hp.n_chunks = n_chunks;
  hp.chunk = CH;
  hp.depth = D;
  hp.num_feature = p.num_feature;
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

void repack_forest(PackedForest& pf, const fd_forest_params& p, const fd_tree_arrays& t) {
  const HostPack hp = pack_forest_host(p, t);
  pf.blob.ensure(hp.blob.size());
  FD_HIP(hipMemcpy(pf.blob.ptr, hp.blob.data(), hp.blob.size(), hipMemcpyHostToDevice));
  pf.leaf_ids.ensure(hp.leaf_ids.size() * sizeof(int32_t));
  FD_HIP(hipMemcpy(pf.leaf_ids.ptr, hp.leaf_ids.data(), hp.leaf_ids.size() * sizeof(int32_t),
                   hipMemcpyHostToDevice));
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
  pf.loaded = true;
}

// ------------------------------------------------------------------------------------------------
// device side

namespace {

template <int D, typename LeafT>
struct Geo {
  static constexpr int NI = (1 << D) - 1;
  static constexpr int NL = 1 << D;
  static constexpr int TREE_BYTES = NI * 8 + NL * (int)sizeof(LeafT);
};

using lds_ptr = __attribute__((address_space(3))) void*;

// Stage one chunk (chunk_stride bytes, a multiple of 1 KiB) global -> LDS with LDS-DMA:
// each wave-instruction moves one 1 KiB piece (64 lanes x 16 B), pieces dealt round-robin to waves.
__device__ __forceinline__ void stage_chunk(const char* __restrict__ src, char* dst, int stride) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int pieces = stride >> 10;
  for (int p = wave; p < pieces; p += kTile / 64) {
    __builtin_amdgcn_global_load_lds((const void*)(src + (p << 10) + lane * 16),
                                     (lds_ptr)(dst + (p << 10)), 16, 0, 0);
  }
}

// Tile-wide OR that is also the prologue barrier. Hand-rolled (per-wave ballot -> one LDS word per
// wave) because __syncthreads_or pulls 256 B of STATIC LDS into the kernel, which shifts the
// dynamic-LDS base and breaks the 1 KiB-aligned feature-tile addressing of forest_kernel_v2.
__device__ __forceinline__ bool tile_any(int pred, uint32_t* flags, int nwaves) {
  const unsigned long long b = __ballot(pred);
  if ((threadIdx.x & 63) == 0) flags[threadIdx.x >> 6] = (b != 0ull) ? 1u : 0u;
  __syncthreads();
  uint32_t r = 0;
  for (int i = 0; i < nwaves; ++i) r |= flags[i];
  return r != 0u;
}

// Walk CH perfect trees of one LDS chunk for this lane; returns leaf slots in idx[].
template <int D, int CH, typename LeafT, bool NAN_AWARE>
__device__ __forceinline__ void walk_chunk(const char* cb, const char* xlane, uint32_t (&idx)[CH]) {
  using G = Geo<D, LeafT>;
#pragma unroll
  for (int c = 0; c < CH; ++c) idx[c] = 0;
#pragma unroll
  for (int l = 0; l < D; ++l) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const uint2 nd = *reinterpret_cast<const uint2*>(cb + c * G::TREE_BYTES + idx[c] * 8);
      const float x = *reinterpret_cast<const float*>(xlane + (nd.y & 0x7fffffffu));
      const float thr = __uint_as_float(nd.x);
      uint32_t right = (x < thr) ? 0u : 1u;
      if (NAN_AWARE) {
        if (x != x) right = (nd.y >> 31) ^ 1u;  // missing value: default direction
      }
      idx[c] = 2u * idx[c] + 1u + right;
    }
  }
}

template <int D, int CH, typename LeafT, int KIND>
__global__ void __launch_bounds__(kTile)
forest_kernel(const float* __restrict__ X, int64_t n, int ld, int nf, const char* __restrict__ blob,
              int n_chunks, int chunk_stride, const int32_t* __restrict__ leaf_ids, int n_trees,
              float base_margin, double if_offset, double if_denom, double* __restrict__ out_prob,
              double* __restrict__ out_raw, int32_t* __restrict__ out_leaf) {
  using G = Geo<D, LeafT>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Xs = reinterpret_cast<float*>(smem);  // [nf][kTile]
  char* bufs = smem + nf * kTile * 4;          // 2 x chunk_stride
  const int t = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kTile;
  const int64_t row = row0 + t;
  const bool valid = row < n;

  // chunk 0 starts landing while the feature tile is loaded
  stage_chunk(blob, bufs, chunk_stride);

  // feature tile: lane t owns row t; LDS writes [f][t] are consecutive across lanes (conflict-free)
  int anynan = 0;
  const int ncopy = ld < nf ? ld : nf;
  if (valid) {
    const float* xr = X + row * (int64_t)ld;
    if ((ld & 1) == 0) {
      const float2* x2 = reinterpret_cast<const float2*>(xr);
      int f = 0;
      for (; f + 1 < ncopy; f += 2) {
        const float2 v = x2[f >> 1];
        Xs[f * kTile + t] = v.x;
        Xs[(f + 1) * kTile + t] = v.y;
        anynan |= (v.x != v.x) | (v.y != v.y);
      }
      for (; f < ncopy; ++f) {
        const float v = xr[f];
        Xs[f * kTile + t] = v;
        anynan |= (v != v);
      }
    } else {
      for (int f = 0; f < ncopy; ++f) {
        const float v = xr[f];
        Xs[f * kTile + t] = v;
        anynan |= (v != v);
      }
    }
    // columns the caller did not supply are missing (XGBoost DMatrix semantics)
    for (int f = ncopy; f < nf; ++f) Xs[f * kTile + t] = __builtin_nanf("");
    anynan |= (ncopy < nf);
  } else {
    for (int f = 0; f < nf; ++f) Xs[f * kTile + t] = 0.f;
  }
  // barrier: feature tile + chunk 0 visible (the barrier's vmcnt(0) drains the LDS-DMA)
  const bool tile_nan = tile_any(anynan, reinterpret_cast<uint32_t*>(bufs + 2 * chunk_stride), kTile / 64);

  const char* xlane = reinterpret_cast<const char*>(Xs + t);
  LeafT acc = (KIND == FD_FOREST_XGB_BINARY_LOGISTIC) ? (LeafT)base_margin : (LeafT)0;
  for (int k = 0; k < n_chunks; ++k) {
    if (k + 1 < n_chunks)
      stage_chunk(blob + (size_t)(k + 1) * chunk_stride, bufs + ((k + 1) & 1) * chunk_stride,
                  chunk_stride);
    const char* cb = bufs + (k & 1) * chunk_stride;
    uint32_t idx[CH];
    if (tile_nan)
      walk_chunk<D, CH, LeafT, true>(cb, xlane, idx);
    else
      walk_chunk<D, CH, LeafT, false>(cb, xlane, idx);
#pragma unroll
    for (int c = 0; c < CH; ++c) {  // tree order: bit-exact sequential accumulation
      const LeafT v = *reinterpret_cast<const LeafT*>(cb + c * G::TREE_BYTES + G::NI * 8 +
                                                      (idx[c] - G::NI) * sizeof(LeafT));
      acc += v;
    }
    if (out_leaf != nullptr && valid) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int tg = k * CH + c;
        if (tg < n_trees)
          out_leaf[row * n_trees + tg] = leaf_ids[(size_t)tg * G::NL + (idx[c] - G::NI)];
      }
    }
    __syncthreads();  // chunk k+1 landed (vmcnt drain) and everyone is done with buffer k&1
  }

  if (!valid) return;
  if (KIND == FD_FOREST_XGB_BINARY_LOGISTIC) {
    // xgboost common::Sigmoid (src/common/math.h), f32
    const float m = (float)acc;
    const float xm = fminf(-m, 88.7f);
    const float denom = expf(xm) + 1.0f + 1e-16f;
    const float p = 1.0f / denom;
    out_prob[row] = (double)p;
    if (out_raw) out_raw[row] = (double)m;
  } else {
    // sklearn: scores = 2 ** -(depths / denominator); decision = -scores - offset_;
    // reference wraps: 1 / (1 + exp(decision))   (ml/models/model_manager.py:344-346)
    const double d = (double)acc;
    const double q = (if_denom != 0.0) ? d / if_denom : 1.0;
    const double score = pow(2.0, -q);
    const double decision = -score - if_offset;
    out_prob[row] = 1.0 / (1.0 + exp(decision));
    if (out_raw) out_raw[row] = d;
  }
}

// ------------------------------------------------------------------------------------------------
// v2 (depth <= 8, the configurations on the path): 1024-thread workgroups on the same 256-txn tile.
// The 64k-txn micro-batch gives exactly 256 tiles = one workgroup per CU, so v1 (256 threads) ran
// ONE wave per SIMD and was issue/latency bound. v2 runs 16 waves: wave w walks, for the 64
// transactions of txn group (w & 3), the trees of tree group (w >> 2) of each staged chunk (2 of the
// chunk's 8 trees) and stores the leaf values in LDS; one rotating "owner" tree group per chunk then
// adds the chunk's 8 values per transaction in tree order into the LDS accumulator, so the sum is
// still the reference's sequential order (bit-exact) while the walking is spread over 16 waves.
//
// LDS layout (absolute byte addresses, dynamic LDS starts at 0):
//   [0, nf*1024)            Xs[f][256] f32     -> x address = (meta & 0x7fffffff) | txn*4 (one v_and_or)
//   buf0, buf1              2 x chunk_stride   staged trees (LDS-DMA)
//   lv0, lv1                2 x [8][256] LeafT leaf values of the chunk being summed / being walked
//   accL                    [256] LeafT        running sum per transaction
// A node address a walks as a' = 2a - tb + 8 + 8*right (tb = tree base), i.e. breadth-first slots.

typedef __attribute__((address_space(3))) char lds_char;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <typename T>
__device__ __forceinline__ T lds_load(uint32_t addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) T*>((size_t)addr);
}
template <typename T>
__device__ __forceinline__ void lds_store(uint32_t addr, T v) {
  *reinterpret_cast<__attribute__((address_space(3))) T*>((size_t)addr) = v;
}

constexpr int kWG2 = 1024;
constexpr int kTreeGroups2 = kWG2 / kTile;  // 4
constexpr int kCH2 = 8;                     // trees per staged chunk
constexpr int kTPG2 = kCH2 / kTreeGroups2;  // trees per wave per chunk

template <int D, typename LeafT, bool NAN_AWARE>
__device__ __forceinline__ void walk2(uint32_t buf, int gg, uint32_t lane4, uint32_t (&a)[kTPG2]) {
  using G = Geo<D, LeafT>;
  uint32_t tb[kTPG2], k0[kTPG2], k1[kTPG2];
#pragma unroll
  for (int j = 0; j < kTPG2; ++j) {
    tb[j] = buf + (uint32_t)((gg * kTPG2 + j) * G::TREE_BYTES);
    k0[j] = 8u - tb[j];
    k1[j] = 16u - tb[j];
    a[j] = tb[j];
  }
#pragma unroll
  for (int l = 0; l < D; ++l) {
#pragma unroll
    for (int j = 0; j < kTPG2; ++j) {
      const u32x2 nd = lds_load<u32x2>(a[j]);
      const float x = lds_load<float>((nd.y & 0x7fffffffu) | lane4);
      bool right = !(x < __uint_as_float(nd.x));
      if (NAN_AWARE) {
        if (x != x) right = (nd.y >> 31) == 0u;
      }
      a[j] = 2u * a[j] + (right ? k1[j] : k0[j]);
    }
  }
}

template <int D, typename LeafT, int KIND>
__global__ void __launch_bounds__(kWG2)
forest_kernel_v2(const float* __restrict__ X, int64_t n, int ld, int nf, const char* __restrict__ blob,
                 int n_chunks, int chunk_stride, const int32_t* __restrict__ leaf_ids, int n_trees,
                 float base_margin, double if_offset, double if_denom, double* __restrict__ out_prob,
                 double* __restrict__ out_raw, int32_t* __restrict__ out_leaf) {
  using G = Geo<D, LeafT>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // Feature-tile addressing needs a 1 KiB-aligned base: (meta & 0x7fffffff) | txn*4. The kernel uses
  // no static LDS, so the dynamic base is 0; the host reserves 1 KiB of slack in case it is not.
  const uint32_t sdyn = (uint32_t)(size_t)((lds_char*)smem);
  const uint32_t s0 = (sdyn + 1023u) & ~1023u;
  char* const lbase = smem + (s0 - sdyn);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int gg = wave >> 2;                // tree group
  const int txn = ((wave & 3) << 6) + lane;  // 0..255 within the tile
  const uint32_t lane4 = s0 + (uint32_t)txn * 4u;
  const uint32_t xbytes = (uint32_t)nf * 1024u;
  const uint32_t bufA = s0 + xbytes, bufB = bufA + (uint32_t)chunk_stride;
  const uint32_t lvA = bufB + (uint32_t)chunk_stride;
  const uint32_t lvB = lvA + kCH2 * kTile * sizeof(LeafT);
  const uint32_t accL = lvB + kCH2 * kTile * sizeof(LeafT);
  const int64_t row = (int64_t)blockIdx.x * kTile + txn;
  const bool valid = row < n;

  // chunk 0 lands while the feature tile loads (16 waves issue its 1 KiB pieces)
  {
    const int pieces = chunk_stride >> 10;
    for (int p = wave; p < pieces; p += kWG2 / 64)
      __builtin_amdgcn_global_load_lds((const void*)(blob + (p << 10) + lane * 16),
                                       (lds_ptr)(lbase + xbytes + (p << 10)), 16, 0, 0);
  }
  // feature tile: 4 threads per transaction, each a strided subset of the columns
  int anynan = 0;
  const int ncopy = ld < nf ? ld : nf;
  {
    const int q = tid >> 8;  // 0..3 (the four threads sharing `txn` have q = tree group)
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
  const bool tile_nan =
      tile_any(anynan, reinterpret_cast<uint32_t*>(lbase + (accL - s0) + kTile * sizeof(LeafT)), kWG2 / 64);

  for (int k = 0; k < n_chunks; ++k) {
    const uint32_t cur = (k & 1) ? bufB : bufA;
    if (k + 1 < n_chunks) {
      const char* src = blob + (size_t)(k + 1) * chunk_stride;
      char* dst = lbase + xbytes + ((k + 1) & 1) * chunk_stride;
      const int pieces = chunk_stride >> 10;
      for (int p = wave; p < pieces; p += kWG2 / 64)
        __builtin_amdgcn_global_load_lds((const void*)(src + (p << 10) + lane * 16), (lds_ptr)(dst + (p << 10)),
                                         16, 0, 0);
    }
    // owner of chunk k-1 adds its leaf values in tree order
    if (k > 0 && gg == ((k - 1) & 3)) {
      const uint32_t lv = ((k - 1) & 1) ? lvB : lvA;
      LeafT acc = lds_load<LeafT>(accL + txn * sizeof(LeafT));
#pragma unroll
      for (int c = 0; c < kCH2; ++c) acc += lds_load<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT));
      lds_store<LeafT>(accL + txn * sizeof(LeafT), acc);
    }
    uint32_t a[kTPG2];
    if (tile_nan)
      walk2<D, LeafT, true>(cur, gg, lane4, a);
    else
      walk2<D, LeafT, false>(cur, gg, lane4, a);
    const uint32_t lv = (k & 1) ? lvB : lvA;
#pragma unroll
    for (int j = 0; j < kTPG2; ++j) {
      const int c = gg * kTPG2 + j;
      const uint32_t tb = cur + (uint32_t)(c * G::TREE_BYTES);
      const uint32_t la = (sizeof(LeafT) == 8) ? a[j] : (tb + G::NI * 4u + ((a[j] - tb) >> 1));
      lds_store<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT), lds_load<LeafT>(la));
      if (out_leaf != nullptr && valid) {
        const int tg = k * kCH2 + c;
        if (tg < n_trees)
          out_leaf[row * n_trees + tg] = leaf_ids[(size_t)tg * G::NL + ((a[j] - tb) >> 3) - G::NI];
      }
    }
    __syncthreads();  // chunk k+1 landed; lv[k&1] complete; owner of k-1 done with lv[(k-1)&1]
  }
  const int last = n_chunks - 1;
  if (gg != (last & 3)) return;
  LeafT acc = lds_load<LeafT>(accL + txn * sizeof(LeafT));
  {
    const uint32_t lv = (last & 1) ? lvB : lvA;
#pragma unroll
    for (int c = 0; c < kCH2; ++c) acc += lds_load<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT));
  }
  if (!valid) return;
  if (KIND == FD_FOREST_XGB_BINARY_LOGISTIC) {
    const float m = (float)acc;
    const float xm = fminf(-m, 88.7f);
    const float denom = expf(xm) + 1.0f + 1e-16f;
    out_prob[row] = (double)(1.0f / denom);
    if (out_raw) out_raw[row] = (double)m;
  } else {
    const double d = (double)acc;
    const double q = (if_denom != 0.0) ? d / if_denom : 1.0;
    const double score = pow(2.0, -q);
    const double decision = -score - if_offset;
    out_prob[row] = 1.0 / (1.0 + exp(decision));
    if (out_raw) out_raw[row] = d;
  }
}

using KernelFn = void (*)(const float*, int64_t, int, int, const char*, int, int, const int32_t*, int,
                          float, double, double, double*, double*, int32_t*);

template <int D, typename LeafT, int KIND>
KernelFn pick_ch() {
  constexpr int CH = D <= 8 ? 8 : (D == 9 ? 4 : 2);
  return forest_kernel<D, CH, LeafT, KIND>;
}

template <typename LeafT, int KIND>
KernelFn pick(int D) {
  switch (D) {
    case 1: return pick_ch<1, LeafT, KIND>();
    case 2: return pick_ch<2, LeafT, KIND>();
    case 3: return pick_ch<3, LeafT, KIND>();
    case 4: return pick_ch<4, LeafT, KIND>();
    case 5: return pick_ch<5, LeafT, KIND>();
    case 6: return pick_ch<6, LeafT, KIND>();
    case 7: return pick_ch<7, LeafT, KIND>();
    case 8: return pick_ch<8, LeafT, KIND>();
    case 9: return pick_ch<9, LeafT, KIND>();
    case 10: return pick_ch<10, LeafT, KIND>();
    default: throw Error(FD_ERR_UNSUPPORTED, "unsupported tree depth");
  }
}

template <typename LeafT, int KIND>
KernelFn pick_v2(int D) {
  switch (D) {
    case 1: return forest_kernel_v2<1, LeafT, KIND>;
    case 2: return forest_kernel_v2<2, LeafT, KIND>;
    case 3: return forest_kernel_v2<3, LeafT, KIND>;
    case 4: return forest_kernel_v2<4, LeafT, KIND>;
    case 5: return forest_kernel_v2<5, LeafT, KIND>;
    case 6: return forest_kernel_v2<6, LeafT, KIND>;
    case 7: return forest_kernel_v2<7, LeafT, KIND>;
    case 8: return forest_kernel_v2<8, LeafT, KIND>;
    default: return nullptr;
  }
}

}  // namespace

void launch_forest(Engine& e, const PackedForest& pf, const float* d_X, int64_t n, int32_t ld,
                   double* d_prob, double* d_raw, int32_t* d_leaf) {
  FD_REQUIRE(d_X && d_prob && ld > 0, FD_ERR_INVALID_ARG, "null buffer or bad ld");
  if (n == 0) return;
  const bool xgb = pf.kind == FD_FOREST_XGB_BINARY_LOGISTIC;
  const size_t leaf_sz = xgb ? sizeof(float) : sizeof(double);
  const size_t xbytes = (size_t)pf.num_feature * kTile * 4;
  KernelFn fn = nullptr;
  int threads = kTile;
  size_t lds = 0;
  // v2: 1024-thread tree-split kernel where it fits the 160 KiB LDS budget
  // + 16 wave flags (tile_any) + 1 KiB alignment slack for the feature tile
  const size_t lds2 = xbytes + 2 * pf.chunk_stride + 2 * (size_t)kCH2 * kTile * leaf_sz + kTile * leaf_sz + 64 + 1024;
  if (e.forest_variant != 1 && pf.depth <= 8 && pf.chunk == kCH2 && lds2 <= 160 * 1024) {
    fn = xgb ? pick_v2<float, FD_FOREST_XGB_BINARY_LOGISTIC>(pf.depth)
             : pick_v2<double, FD_FOREST_SKLEARN_IFOREST>(pf.depth);
    threads = kWG2;
    lds = lds2;
  }
  if (!fn) {
    FD_REQUIRE(e.forest_variant != 2, FD_ERR_UNSUPPORTED, "forest kernel v2 does not fit this forest");
    fn = xgb ? pick<float, FD_FOREST_XGB_BINARY_LOGISTIC>(pf.depth)
             : pick<double, FD_FOREST_SKLEARN_IFOREST>(pf.depth);
    lds = xbytes + 2 * pf.chunk_stride + 64;  // + tile_any flags
  }
  FD_REQUIRE(lds <= 160 * 1024, FD_ERR_UNSUPPORTED, "LDS budget exceeded");
  FD_HIP(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int64_t blocks = (n + kTile - 1) / kTile;
  FD_REQUIRE(blocks < (1ll << 31), FD_ERR_INVALID_ARG, "batch too large");
  Engine::Timed* ev = e.timing ? e.next_event_pair(xgb ? FD_TIMING_XGB : FD_TIMING_IFOREST) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, e.stream));
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(threads), lds, e.stream, d_X, n, (int)ld,
                     pf.num_feature, pf.blob.as<const char>(), pf.n_chunks, (int)pf.chunk_stride,
                     pf.leaf_ids.as<const int32_t>(), pf.n_trees, pf.base_margin, pf.if_offset,
                     pf.if_denominator, d_prob, d_raw, d_leaf);
  FD_HIP(hipGetLastError());
  if (ev) FD_HIP(hipEventRecord(ev->b, e.stream));
}

}  // namespace fd
