// walk_common.h — device helpers shared by the forest kernels (forest.hip) and the fused ensemble kernel
// (ensemble.hip): LDS access by byte address, LDS-DMA chunk staging, the binned perfect-tree walk, feature
// binning against sorted threshold tables, and the reference's output transforms.
//
// Binned node words (see forest.hip "Binned layout"): a node is ONE u32 `j << 16 | feature * 1024 |
// default_left`, a feature value's bin word is `bin << 16` (NaN: 0xFFFF << 16) with bin = #{thresholds
// <= x}, so "x < t_j" is "bin <= j" is one unsigned compare word(x) <= node, and the feature-row address in
// the [f][256] LDS tile is (node & 0xFC00) | lane.
#pragma once

#include <cmath>
#include <cstdint>

#include "fd_internal.h"

namespace fd {
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

// Same staging, issued through inline asm. While an LDS-DMA issued by the builtin is outstanding,
// LLVM's waitcnt insertion cannot count LDS reads and emits lgkmcnt(0) before every use, which
// serialises the walk's independent chains. Hidden from the compiler, the DMA must be completed by
// the caller: dma_wait() (vmcnt(0)) before the barrier that publishes the chunk.
__device__ __forceinline__ void stage_chunk_asm(const char* __restrict__ src, uint32_t dst, int stride, int nwaves) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int pieces = stride >> 10;
  for (int p = wave; p < pieces; p += nwaves) {
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
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// XGBoost common::Sigmoid (src/common/math.h) in f32 / sklearn score -> decision -> the
// reference's 1/(1+exp(s)) in f64.
template <int KIND, typename LeafT>
__device__ __forceinline__ double forest_prob(LeafT acc, double if_offset, double if_denom) {
  if (KIND == FD_FOREST_XGB_BINARY_LOGISTIC) {
    const float m = (float)acc;
    const float xm = fminf(-m, 88.7f);
    const float denom = expf(xm) + 1.0f + 1e-16f;
    return (double)(1.0f / denom);
  } else {
    const double d = (double)acc;
    const double q = (if_denom != 0.0) ? d / if_denom : 1.0;
    const double score = pow(2.0, -q);
    const double decision = -score - if_offset;
    return 1.0 / (1.0 + exp(decision));
  }
}
template <int KIND, typename LeafT>
__device__ __forceinline__ void write_outputs(LeafT acc, int64_t row, double if_offset, double if_denom,
                                              double* out_prob, double* out_raw) {
  out_prob[row] = forest_prob<KIND, LeafT>(acc, if_offset, if_denom);
  if (out_raw) out_raw[row] = KIND == FD_FOREST_XGB_BINARY_LOGISTIC ? (double)(float)acc : (double)acc;
}


template <int D, int TPG, typename LeafT, bool NAN_AWARE, bool NODE_ONLY = false>
__device__ __forceinline__ void walk4(uint32_t buf, int gg, uint32_t lane4, uint32_t (&slot)[TPG]) {
  // tree stride in the staged chunk: node words + leaf values, or node words only (kernel 6)
  constexpr uint32_t TB = NODE_ONLY ? (4u << D) : (4u + (uint32_t)sizeof(LeafT)) << D;
  constexpr uint32_t NL = 1u << D;
  // P = LDS address of the children pair of the current node (heap slot i: tb + 8 i). Chosen child
  // c = 2i + r has its pair at tb + 8c = 2P - tb + 8r = (P << 1) + (r ? 8 - tb : -tb).
  uint32_t tb[TPG], c0[TPG], c8[TPG], P[TPG], node[TPG], kl[TPG], kr[TPG], xw[TPG];
#pragma unroll
  for (int j = 0; j < TPG; ++j) {
    tb[j] = buf + (uint32_t)(gg * TPG + j) * TB;
    c0[j] = 0u - tb[j];
    c8[j] = 8u - tb[j];
    asm volatile("" : "+v"(c0[j]), "+v"(c8[j]));  // keep the two-term form (one cndmask + one lshl_add)
    node[j] = lds_load<uint32_t>(tb[j] + 4u);     // heap slot 1
    P[j] = tb[j] + 8u;                            // slots 2, 3
  }
#pragma unroll
  for (int j = 0; j < TPG; ++j) {
    xw[j] = lds_load<uint32_t>((node[j] & 0xFC00u) | lane4);
    if (D > 1) {
      const u32x2 k = lds_load<u32x2>(P[j]);
      kl[j] = k.x;
      kr[j] = k.y;
    }
  }
  // software-pipelined over the TPG chains: chain j's next reads are issued right after its step, so
  // the wave keeps ~2 (TPG - 1) LDS reads in flight while it steps the other chains
#pragma unroll
  for (int l = 0; l < D; ++l) {
#pragma unroll
    for (int j = 0; j < TPG; ++j) {
      bool right = xw[j] > node[j];  // bin > j  <=>  !(x < t_j)
      if (NAN_AWARE) {
        if (xw[j] == 0xFFFF0000u) right = (node[j] & 1u) == 0u;  // missing: default direction
      }
      P[j] = (P[j] << 1) + (right ? c8[j] : c0[j]);
      if (l + 1 < D) {
        uint32_t a = kl[j], b = kr[j];
        asm volatile("" : "+v"(a), "+v"(b));
        node[j] = right ? b : a;
        xw[j] = lds_load<uint32_t>((node[j] & 0xFC00u) | lane4);
        if (l + 2 < D) {
          const u32x2 k = lds_load<u32x2>(P[j]);
          kl[j] = k.x;
          kr[j] = k.y;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < TPG; ++j) slot[j] = ((P[j] - tb[j]) >> 3) - NL;  // leaf heap slot - 2^D
}


// largest power of two <= cnt (0 for cnt == 0): binary lifting over cnt entries needs exactly these
// steps (a feature no split uses — the 64-wide vector's pad slots — costs none)
__device__ __forceinline__ int lift_steps(int cnt) { return cnt > 0 ? (int)(1u << (31 - __clz(cnt))) : 0; }

// ---- tree-split binning (forest.hip split_bin_kernel / split_bin_pair_kernel; lstm.hip lstm_kernel4's bin blocks)
constexpr int kSplitBin = 256;  // rows per binning workgroup (one thread each)

// one thread per (feature f, row r): the binary search's dependent loads are the only latency
__device__ __forceinline__ void split_bin_body(const float* __restrict__ X, int64_t n, int64_t n_pad, int ld, int f,
                                               int64_t r, const float* __restrict__ thr,
                                               const int32_t* __restrict__ thr_off, uint32_t* __restrict__ bins,
                                               uint32_t* __restrict__ tile_nan) {
  const bool ok = r < n;  // r within [0, n_pad)
  float v = 0.f;
  if (ok) v = f < ld ? X[r * (int64_t)ld + f] : __builtin_nanf("");  // DMatrix: missing column = NaN
  const int o = thr_off[f], cnt = thr_off[f + 1] - o;
  int pos = 0;
  for (int st = lift_steps(cnt); st > 0; st >>= 1) {
    const int np = pos + st;
    if (np <= cnt && thr[o + np - 1] <= v) pos = np;
  }
  const bool isnan_v = ok && v != v;
  bins[(size_t)f * n_pad + r] = !ok ? 0u : (isnan_v ? 0xFFFF0000u : (uint32_t)pos << 16);
  // tile flag: nonzero when the tile holds a NaN; the step's sum kernel, its last launch over this scratch, clears it
  // again, so a replayed hipGraph of the step starts from clear flags (no host-side epoch). (kTile rows per tile, a
  // multiple of the 64 rows of a wave)
  if (__ballot(isnan_v) != 0ull && (threadIdx.x & 63) == 0) tile_nan[r / kTile] = 1u;
}

// one forest's binning inputs / outputs
struct SplitBinArgs {
  const float* thr;
  const int32_t* thr_off;
  uint32_t* bins;
  uint32_t* tile_nan;
  int nf;
};

// cell y of a forest pair's binning: features 0..a.nf-1 of the first forest, then the second's
__device__ __forceinline__ void split_bin_pair_cell(const float* __restrict__ X, int64_t n, int64_t n_pad, int ld,
                                                    const SplitBinArgs& a, const SplitBinArgs& b, int y, int64_t r) {
  if (y < a.nf)
    split_bin_body(X, n, n_pad, ld, y, r, a.thr, a.thr_off, a.bins, a.tile_nan);
  else
    split_bin_body(X, n, n_pad, ld, y - a.nf, r, b.thr, b.thr_off, b.bins, b.tile_nan);
}


// bin(v) = #{t in tbl[0, cnt) : t <= v}, tbl ascending; steps = largest power of two <= cnt.
template <bool IN_LDS>
__device__ __forceinline__ uint32_t bin_of(float v, const float* __restrict__ gt, uint32_t lt, int cnt, int steps) {
  int pos = 0;
  for (int st = steps; st > 0; st >>= 1) {
    const int np = pos + st;
    if (np <= cnt) {
      const float t = IN_LDS ? lds_load<float>(lt + (uint32_t)(np - 1) * 4u) : gt[np - 1];
      if (t <= v) pos = np;
    }
  }
  return (uint32_t)pos;
}


}  // namespace
}  // namespace fd
