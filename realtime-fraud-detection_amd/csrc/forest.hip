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

size_t round1k(size_t b) { return (b + 1023) / 1024 * 1024; }

}  // namespace

size_t lds_bytes_kernel3(int nf, size_t chunk_stride, int ch, size_t leaf_sz) {
  // Xs + 2 chunk buffers + 2 leaf-value buffers + accumulator + 16 wave flags + 1 KiB alignment slack
  return (size_t)nf * kTile * 4 + 2 * chunk_stride + 2 * (size_t)ch * kTile * leaf_sz + kTile * leaf_sz + 64 + 1024;
}

size_t lds_bytes_kernel1(int nf, size_t chunk_stride) { return (size_t)nf * kTile * 4 + 2 * chunk_stride + 64; }

// Trees per staged chunk: for depth <= 8 the largest multiple of 4 (one tree per wave of each of the
// four tree groups, x TPG) whose LDS image fits forest_kernel3's 160 KiB; deeper trees: kernel 1.
static int choose_chunk(int D, int nf, size_t leaf_sz) {
  const size_t tb = ((size_t)8 + leaf_sz) << D;
  if (D <= 8) {
    for (int ch = 16; ch >= 4; ch -= 4)
      if (lds_bytes_kernel3(nf, round1k(ch * tb), ch, leaf_sz) <= kLdsBudget) return ch;
  }
  for (int ch = 8; ch >= 1; ch /= 2)
    if (lds_bytes_kernel1(nf, round1k(ch * tb)) <= kLdsBudget) return ch;
  throw Error(FD_ERR_UNSUPPORTED, "forest does not fit the LDS budget");
}

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
  const int NL = 1 << D;  // heap slots 1..NL-1 internal, NL..2NL-1 leaves
  const size_t leaf_sz = xgb ? sizeof(float) : sizeof(double);
  const size_t tree_bytes = (size_t)NL * 8 + (size_t)NL * leaf_sz;
  const int CH = choose_chunk(D, p.num_feature, leaf_sz);
  const size_t chunk_stride = round1k(CH * tree_bytes);
  const int n_chunks = (T + CH - 1) / CH;
  HostPack hp;
  hp.blob.assign(n_chunks * chunk_stride, 0);  // padding trees: all-zero nodes/leaves
  hp.leaf_ids.assign((size_t)n_chunks * CH * NL, -1);
  std::vector<int32_t> cur(2 * NL);

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
    char* leaves = tb + (size_t)NL * 8;
    cur[1] = 0;
    for (int s = 1; s < NL; ++s) {
      const int32_t o = cur[s];
      if (L[o] < 0) {  // leaf above depth D: pad node, both subtrees resolve to the same leaf
        nodes[2 * s] = 0;
        nodes[2 * s + 1] = 0;
        cur[2 * s] = o;
        cur[2 * s + 1] = o;
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

typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) void* lds_ptr;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ T lds_load(uint32_t addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) T*>((size_t)addr);
}
template <typename T>
__device__ __forceinline__ void lds_store(uint32_t addr, T v) {
  *reinterpret_cast<__attribute__((address_space(3))) T*>((size_t)addr) = v;
}

// Tile-wide OR that is also the prologue barrier. Hand-rolled (per-wave ballot -> one LDS word per
// wave) because __syncthreads_or pulls 256 B of STATIC LDS into the kernel, which shifts the
// dynamic-LDS base and breaks the 1 KiB-aligned feature-tile addressing of forest_kernel3.
__device__ __forceinline__ bool tile_any(int pred, uint32_t* flags, int nwaves) {
  const unsigned long long b = __ballot(pred);
  if ((threadIdx.x & 63) == 0) flags[threadIdx.x >> 6] = (b != 0ull) ? 1u : 0u;
  __syncthreads();
  uint32_t r = 0;
  for (int i = 0; i < nwaves; ++i) r |= flags[i];
  return r != 0u;
}

// Stage one chunk (stride bytes, a multiple of 1 KiB) global -> LDS with LDS-DMA: each
// wave-instruction moves one 1 KiB piece (64 lanes x 16 B), pieces dealt round-robin to waves.
__device__ __forceinline__ void stage_chunk(const char* __restrict__ src, char* dst, int stride, int nwaves) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int pieces = stride >> 10;
  for (int p = wave; p < pieces; p += nwaves)
    __builtin_amdgcn_global_load_lds((const void*)(src + (p << 10) + lane * 16), (lds_ptr)(dst + (p << 10)), 16,
                                     0, 0);
}

// XGBoost common::Sigmoid (src/common/math.h) in f32 / sklearn score -> decision -> the
// reference's 1/(1+exp(s)) in f64.
template <int KIND, typename LeafT>
__device__ __forceinline__ void write_outputs(LeafT acc, int64_t row, double if_offset, double if_denom,
                                              double* out_prob, double* out_raw) {
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

template <int D, int TPG, typename LeafT, bool NAN_AWARE>
__device__ __forceinline__ void walk3(uint32_t buf, int gg, uint32_t lane4, uint32_t (&idx)[TPG]) {
  constexpr uint32_t TB = (8u + (uint32_t)sizeof(LeafT)) << D;
  uint32_t tb[TPG];
  u32x2 nd[TPG];
  u32x4 kids[TPG];
  float x[TPG];
#pragma unroll
  for (int j = 0; j < TPG; ++j) {
    tb[j] = buf + (uint32_t)(gg * TPG + j) * TB;
    idx[j] = 1u;
    nd[j] = lds_load<u32x2>(tb[j] + 8u);  // root = heap slot 1
  }
#pragma unroll
  for (int j = 0; j < TPG; ++j) {
    x[j] = lds_load<float>((nd[j].y & 0x7fffffffu) | lane4);
    if (D > 1) kids[j] = lds_load<u32x4>(tb[j] + 16u);  // slots 2, 3
  }
#pragma unroll
  for (int l = 0; l + 1 < D; ++l) {
#pragma unroll
    for (int j = 0; j < TPG; ++j) {
      bool right = !(x[j] < __uint_as_float(nd[j].x));
      if (NAN_AWARE) {
        if (x[j] != x[j]) right = (nd[j].y >> 31) == 0u;
      }
      idx[j] = 2u * idx[j] + (right ? 1u : 0u);
      nd[j].x = right ? kids[j].z : kids[j].x;
      nd[j].y = right ? kids[j].w : kids[j].y;
    }
#pragma unroll
    for (int j = 0; j < TPG; ++j) {
      x[j] = lds_load<float>((nd[j].y & 0x7fffffffu) | lane4);
      if (l + 2 < D) kids[j] = lds_load<u32x4>(tb[j] + 16u * idx[j]);  // children of the new node
    }
  }
#pragma unroll
  for (int j = 0; j < TPG; ++j) {
    bool right = !(x[j] < __uint_as_float(nd[j].x));
    if (NAN_AWARE) {
      if (x[j] != x[j]) right = (nd[j].y >> 31) == 0u;
    }
    idx[j] = 2u * idx[j] + (right ? 1u : 0u);  // leaf heap slot in [2^D, 2^(D+1))
  }
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

  stage_chunk(blob, lbase + xbytes, chunk_stride, kWG3 / 64);  // chunk 0 lands while the tile loads
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
  const bool tile_nan =
      tile_any(anynan, reinterpret_cast<uint32_t*>(lbase + (accL - s0) + kTile * sizeof(LeafT)), kWG3 / 64);

  for (int k = 0; k < n_chunks; ++k) {
    const uint32_t cur = (k & 1) ? bufB : bufA;
    if (k + 1 < n_chunks)
      stage_chunk(blob + (size_t)(k + 1) * chunk_stride, lbase + xbytes + ((k + 1) & 1) * chunk_stride,
                  chunk_stride, kWG3 / 64);
    // owner of chunk k-1 adds its leaf values in tree order
    if (k > 0 && gg == ((k - 1) & 3)) {
      const uint32_t lv = ((k - 1) & 1) ? lvB : lvA;
      LeafT acc = lds_load<LeafT>(accL + txn * sizeof(LeafT));
#pragma unroll
      for (int c = 0; c < CH; ++c) acc += lds_load<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT));
      lds_store<LeafT>(accL + txn * sizeof(LeafT), acc);
    }
    uint32_t idx[TPG];
    if (tile_nan)
      walk3<D, TPG, LeafT, true>(cur, gg, lane4, idx);
    else
      walk3<D, TPG, LeafT, false>(cur, gg, lane4, idx);
    const uint32_t lv = (k & 1) ? lvB : lvA;
#pragma unroll
    for (int j = 0; j < TPG; ++j) {
      const int c = gg * TPG + j;
      const uint32_t tb = cur + (uint32_t)c * TB;
      const uint32_t slot = idx[j] - NL;
      lds_store<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT), lds_load<LeafT>(tb + NL * 8u + slot * sizeof(LeafT)));
      if (out_leaf != nullptr && valid) {
        const int tg = k * CH + c;
        if (tg < n_trees) out_leaf[row * n_trees + tg] = leaf_ids[(size_t)tg * NL + slot];
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
    for (int c = 0; c < CH; ++c) acc += lds_load<LeafT>(lv + (c * kTile + txn) * sizeof(LeafT));
  }
  if (valid) write_outputs<KIND, LeafT>(acc, row, if_offset, if_denom, out_prob, out_raw);
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

}  // namespace

void launch_forest(Engine& e, const PackedForest& pf, const float* d_X, int64_t n, int32_t ld,
                   double* d_prob, double* d_raw, int32_t* d_leaf) {
  FD_REQUIRE(d_X && d_prob && ld > 0, FD_ERR_INVALID_ARG, "null buffer or bad ld");
  if (n == 0) return;
  const bool xgb = pf.kind == FD_FOREST_XGB_BINARY_LOGISTIC;
  const size_t leaf_sz = xgb ? sizeof(float) : sizeof(double);
  KernelFn fn = nullptr;
  int threads = kTile;
  size_t lds = 0;
  const size_t lds3 = lds_bytes_kernel3(pf.num_feature, pf.chunk_stride, pf.chunk, leaf_sz);
  if (e.forest_variant != 1 && pf.depth <= 8 && pf.chunk % 4 == 0 && lds3 <= kLdsBudget) {
    fn = xgb ? pick3<float, FD_FOREST_XGB_BINARY_LOGISTIC>(pf.depth, pf.chunk)
             : pick3<double, FD_FOREST_SKLEARN_IFOREST>(pf.depth, pf.chunk);
    threads = kWG3;
    lds = lds3;
  }
  if (!fn) {
    FD_REQUIRE(e.forest_variant != 2, FD_ERR_UNSUPPORTED, "forest kernel 3 does not fit this forest");
    fn = xgb ? pick1<float, FD_FOREST_XGB_BINARY_LOGISTIC>(pf.depth, pf.chunk)
             : pick1<double, FD_FOREST_SKLEARN_IFOREST>(pf.depth, pf.chunk);
    lds = lds_bytes_kernel1(pf.num_feature, pf.chunk_stride);
  }
  FD_REQUIRE(fn != nullptr, FD_ERR_UNSUPPORTED, "no forest kernel for this depth/chunk");
  FD_REQUIRE(lds <= kLdsBudget, FD_ERR_UNSUPPORTED, "LDS budget exceeded");
  FD_HIP(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int64_t blocks = (n + kTile - 1) / kTile;
  FD_REQUIRE(blocks < (1ll << 31), FD_ERR_INVALID_ARG, "batch too large");
  Engine::Timed* ev = e.timing ? e.next_event_pair(xgb ? FD_TIMING_XGB : FD_TIMING_IFOREST) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, e.stream));
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(threads), lds, e.stream, d_X, n, (int)ld, pf.num_feature,
                     pf.blob.as<const char>(), pf.n_chunks, (int)pf.chunk_stride, pf.leaf_ids.as<const int32_t>(),
                     pf.n_trees, pf.base_margin, pf.if_offset, pf.if_denominator, d_prob, d_raw, d_leaf);
  FD_HIP(hipGetLastError());
  if (ev) FD_HIP(hipEventRecord(ev->b, e.stream));
}

}  // namespace fd
