// lstm.hip — the LSTM sequence head of the ensemble (lstm_sequential) on the CDNA4 matrix cores.
//
// Reference: ModelManager._load_tensorflow_model / _predict_tensorflow
// (ml/models/model_manager.py:162-165, 313-319) with the registry entry lstm_sequential
// (ml/utils/config.py:145-157: sequence_length 10, hidden_units 128, weight 0.25). The reference ships
// no model file (its DummyModel raises, so the head is dropped); the build defines the head as a
// 1-layer LSTM(H = 128) over the card's last T events (per-event input = the 16 bridged raw features,
// sign*log1p-compressed, features.hip seq_input) followed by Dense(1, sigmoid) or Dense(2, softmax)[:, 1],
// i.e. what Keras' LSTM(128) + Dense computes (gate order i, f, g(c~), o, as Keras and PyTorch).
//
// Kernel: one workgroup of 8 waves per tile of 16 transactions, computing in f32 on MFMA
// (v_mfma_f32_16x16x4_f32: exact f32 fma chains, the reference model's precision — no bf16).
//   gates[16 txn x 512] = x_t[16 x 16] W_ih^T + h_{t-1}[16 x 128] W_hh^T + b
// Wave w owns hidden units 16w..16w+15: its four 16x16 accumulator tiles are the i, f, g, o gates of
// those units, so with the MFMA C/D layout (col = lane & 15 = unit, row = 4 (lane >> 4) + reg = txn)
// every lane holds all four gates of its (txn, unit) cells and the cell update is lane-local.
// W_ih / W_hh stay in VGPRs for the whole kernel (144 B-operand registers per lane, packed at load so
// the preload is coalesced); h_t goes through a double-buffered LDS tile laid out so each lane reads
// its 32 A-operand values with 8 ds_read_b128; one barrier per time step.
// Per 16-txn tile and step: 4 tiles x 36 k-steps = 144 MFMAs per wave = 2.36 MFLOP per workgroup.
//
// Small batches (the latency path, config 5's 1 k micro-batches) would leave most CUs idle with 16-row
// tiles (64 workgroups for 1 k), and the recurrence cannot be split across CUs without a per-step
// exchange of h_t. lstm_kernel4 therefore takes 4 transactions per workgroup on the 16-block form
// v_mfma_f32_4x4x1_16b_f32 (the same f32 rate per instruction-cycle, a quarter of the rows): all 16
// blocks share the A operand — the CBSZ/ABID broadcast of one block's 4 values, so a single VGPR holding
// h[txn][k0 + block] feeds 16 instructions and a lane reads all of h_t with two ds_read_b128 — and each
// block takes 4 gate columns, so one instruction is 4 txn x 64 columns x 1 k. Lane l of wave w accumulates column (gate l >> 4, unit
// 16 w + (l & 15)) for the 4 transactions (one register each); a 4 x 4 transpose across the 16-lane
// rows (two v_permlane32_swap + two v_permlane16_swap) then gives lane (q, unit) the i, f, g, o gates
// of transaction q, so each lane updates ONE cell (5 transcendentals instead of 20). The workgroup
// loops over tiles (persistent grid) with the weights resident in VGPRs.
// Software-pipelined steps (round 5): of step t+1's 144 k-steps, the 16 of x_{t+1} and the 16 of the wave's OWN
// hidden units (h_t of its lanes, moved into the A-operand order by one ds_bpermute, no LDS round trip) need nothing
// from the other waves, so they are issued before step t's barrier, while the matrix pipe would otherwise idle
// through the cell update, the h_t stores and the barrier; after the barrier only the other 7 units' blocks remain.
// Wave w's W_hh blocks are packed in the order w, w+1, ..., w+7 (mod 8) for this. Step 0's W_hh h_{-1} (h = 0) is
// skipped when every W_hh weight is finite (0 * w = 0 adds nothing; a non-finite weight keeps the products).
#include <algorithm>
#include <cmath>
#include <utility>

#include "fd_internal.h"
#include "walk_common.h"

namespace fd {
#ifdef FD_FOREST_PROFILE
FD_TL_BUF(g_tl_lstm);
#endif
namespace {

constexpr int kH = kLstmHidden;  // 128
constexpr int kI = kSeqInput;    // 16
constexpr int kRows = 16;        // transactions per workgroup
constexpr int kKS = kI / 4 + kH / 4;  // 36 k-steps of 4
constexpr int kKT = kI + kH;          // 144 k values: one 4x4x1 MFMA each

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Gate nonlinearities on the hardware transcendentals (v_exp_f32, v_rcp_f32: ~1 ulp each) instead of
// the correctly rounded libm sequences: the per-step cell update is the serial tail between two MFMA
// chains. sigm(x) = 1 / (1 + 2^(-x log2 e)) saturates to exactly 0 / 1; tanh(x) = 2 sigm(2x) - 1 has an
// absolute error of a few 1e-8 near 0. The head's probabilities stay within the 1e-5 north-star bar
// of the PyTorch fp32 forward (tests/test_gpu_lstm.py).
__device__ __forceinline__ float sigm(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.44269504088896341f));
}
__device__ __forceinline__ float tanh_g(float x) { return 2.0f * sigm(2.0f * x) - 1.0f; }

__global__ void __launch_bounds__(512) lstm_kernel(const float* __restrict__ seq, int64_t n, int T,
                                                   const float* __restrict__ wpk, const float* __restrict__ bias,
                                                   const float* __restrict__ wout, const float* __restrict__ bout,
                                                   int n_out, double* __restrict__ prob) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float hbuf[2][kRows][4][kH / 4];       // 16 KB
  __shared__ __attribute__((aligned(16))) float xs[FD_MAX_SEQ_LEN][kRows][4][kI / 4];  // 16 KB
  __shared__ float zs[kRows][2];
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63;
  const int64_t row0 = (int64_t)blockIdx.x * kRows;

  // x tile -> LDS in the A-operand order (k = 4 s + (lane >> 4) -> [k & 3][k >> 2])
  for (int idx = tid; idx < kRows * T * kI; idx += 512) {
    const int r = idx / (T * kI), rem = idx - r * (T * kI), t = rem / kI, k = rem - t * kI;
    xs[t][r][k & 3][k >> 2] = (row0 + r < n) ? seq[(size_t)(row0 + r) * T * kI + rem] : 0.f;
  }
  for (int idx = tid; idx < kRows * kH; idx += 512) (&hbuf[0][0][0][0])[idx] = 0.f;

  // B operands for the whole sequence: lane holds W[g*128 + unit][4 s + (lane >> 4)]
  float bw[4][kKS];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int s = 0; s < kKS; ++s) bw[g][s] = wpk[((size_t)(w * 4 + g) * kKS + s) * 64 + l];
  const int unit = 16 * w + (l & 15);
  float bg[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bg[g] = bias[g * kH + unit];
  float c[4] = {0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    f32x4 acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = f32x4{bg[g], bg[g], bg[g], bg[g]};
    const f32x4 xa = *reinterpret_cast<const f32x4*>(&xs[t][l & 15][l >> 4][0]);
#pragma unroll
    for (int s = 0; s < kI / 4; ++s)
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[s], bw[g][s], acc[g], 0, 0, 0);
    const float* hp = &hbuf[t & 1][l & 15][l >> 4][0];
#pragma unroll
    for (int sb = 0; sb < kH / 16; ++sb) {
      const f32x4 ha = *reinterpret_cast<const f32x4*>(hp + 4 * sb);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(ha[j], bw[g][kI / 4 + 4 * sb + j], acc[g], 0, 0, 0);
    }
    float* hn = &hbuf[(t + 1) & 1][0][0][0];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float ig = sigm(acc[0][j]), fg = sigm(acc[1][j]), gg = tanh_g(acc[2][j]), og = sigm(acc[3][j]);
      c[j] = fg * c[j] + ig * gg;
      const float hv = og * tanh_g(c[j]);
      const int r = 4 * (l >> 4) + j;
      hn[(r * 4 + (unit & 3)) * (kH / 4) + (unit >> 2)] = hv;
    }
    __syncthreads();
  }

  // dense head over h_T, summed in k order. (lstm_kernel4's head sums a wave's partials by butterfly instead, so the
  // two tile forms agree within the 1e-5 tolerance the tests hold both to, not bit for bit)
  if (tid < kRows * n_out) {
    const int r = tid / n_out, o = tid - r * n_out;
    const float* hT = &hbuf[T & 1][r][0][0];
    float z = bout[o];
    for (int k = 0; k < kH; ++k) z = z + wout[o * kH + k] * hT[(k & 3) * (kH / 4) + (k >> 2)];
    zs[r][o] = z;
  }
  __syncthreads();
  if (tid < kRows && row0 + tid < n) {
    float p;
    if (n_out == 1) {
      p = sigm(zs[tid][0]);
    } else {  // softmax([z0, z1])[1]
      const float m = fmaxf(zs[tid][0], zs[tid][1]);
      const float e0 = expf(zs[tid][0] - m), e1 = expf(zs[tid][1] - m);
      p = e1 / (e0 + e1);
    }
    prob[row0 + tid] = (double)p;
  }
}

// lane row g (16 lanes), register j holds M[j][g] -> register j holds M[g][j]
__device__ __forceinline__ void xpose_rows4(float& a0, float& a1, float& a2, float& a3) {
  const auto r02 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a0), __float_as_uint(a2), false, false);
  const auto r13 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a1), __float_as_uint(a3), false, false);
  const auto r01 = __builtin_amdgcn_permlane16_swap(r02[0], r13[0], false, false);
  const auto r23 = __builtin_amdgcn_permlane16_swap(r02[1], r13[1], false, false);
  a0 = __uint_as_float(r01[0]);
  a1 = __uint_as_float(r01[1]);
  a2 = __uint_as_float(r23[0]);
  a3 = __uint_as_float(r23[1]);
}

// acc[J & 3] += A(block J, broadcast to all 16 blocks: CBSZ 4, ABID J) x B(b[J]) for J = 0..15: lanes
// 4J..4J+3 of `a` hold the 4 transactions' values at k = k0 + J, so one VGPR feeds 16 k-steps
template <int... J>
__device__ __forceinline__ void mfma_abid16(float a, const float* b, f32x4* acc, std::integer_sequence<int, J...>) {
  ((acc[J & 3] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b[J], acc[J & 3], 4, J, 0)), ...);
}

// option latency_prebin (fd_internal.h PreBin): the XGBoost + IsolationForest pair's tree-split binning
// (split_bin_pair_kernel's cells, two per workgroup) in the first `blocks` workgroups of the LSTM launch, which the
// dispatcher places ahead of the LSTM's own: the pair's binning launch and its queue gap go
struct LstmBinArgs {
  const float* X;
  int64_t n, n_pad;
  int ld;
  SplitBinArgs a, b;
  int blocks, row_blocks;
  int last;  // the binning workgroups after the LSTM's (option latency_prebin 2) instead of ahead of them
  // option latency_prebin 3 (blocks 0): the searches inside the LSTM's own workgroups instead — thread g of the
  // launch takes searches g and g + 512 gridDim.x of the n_pad x (a.nf + b.nf) (feature-major), one binary-lifting
  // level per recurrence step of its first tile (the load in flight behind the step's MFMAs), the rest after (two
  // levels per step, the second load behind the gate tail, measured slower: the LSTM launch 22.0 -> 22.3 us)
  int inline_searches;
  int steps;  // the lifting's first step: a power of two >= every feature's largest one (higher ones are skipped)
};

// one (row, feature) search of the inline form: split_bin_body's count of the feature's ascending thresholds <= v,
// advanced one level at a time
struct InlineSearch {
  const float* thr;
  float v;
  int o, cnt, pos;
  bool act;
};

__device__ __forceinline__ void inline_search_init(const LstmBinArgs& pb, int64_t s, InlineSearch& q) {
  const int64_t total = pb.n_pad * (int64_t)(pb.a.nf + pb.b.nf);
  q.act = s < total;
  const int y = q.act ? (int)(s / pb.n_pad) : 0;
  const int64_t r = q.act ? s - (int64_t)y * pb.n_pad : 0;
  const bool fb = y >= pb.a.nf;
  const int f = fb ? y - pb.a.nf : y;
  const int32_t* to = fb ? pb.b.thr_off : pb.a.thr_off;
  q.thr = fb ? pb.b.thr : pb.a.thr;
  q.o = to[f];
  q.cnt = (q.act && r < pb.n) ? to[f + 1] - q.o : 0;
  q.v = (q.act && r < pb.n) ? (f < pb.ld ? pb.X[r * (int64_t)pb.ld + f] : __builtin_nanf("")) : 0.f;
  q.pos = 0;
}

__device__ __forceinline__ float inline_search_load(const InlineSearch& q, int st) {
  return q.thr[max(q.o + min(q.pos + st, q.cnt) - 1, 0)];
}

__device__ __forceinline__ void inline_search_step(InlineSearch& q, int st, float t) {
  const int np = q.pos + st;
  if (np <= q.cnt && t <= q.v) q.pos = np;
}

__device__ __forceinline__ void inline_search_store(const LstmBinArgs& pb, int64_t s, const InlineSearch& q) {
  if (!q.act) return;
  const int y = (int)(s / pb.n_pad);
  const int64_t r = s - (int64_t)y * pb.n_pad;
  const bool fb = y >= pb.a.nf;
  const int f = fb ? y - pb.a.nf : y;
  const SplitBinArgs& A = fb ? pb.b : pb.a;
  const bool ok = r < pb.n, isnan_v = ok && q.v != q.v;
  A.bins[(size_t)f * pb.n_pad + r] = !ok ? 0u : (isnan_v ? 0xFFFF0000u : (uint32_t)q.pos << 16);
  if (isnan_v) A.tile_nan[r / kTile] = 1u;
}

__global__ void __launch_bounds__(512) lstm_kernel4(const float* __restrict__ seq, int64_t n, int T,
                                                    const float* __restrict__ wpk4, const float* __restrict__ bias,
                                                    const float* __restrict__ wout, const float* __restrict__ bout,
                                                    int n_out, double* __restrict__ prob,
                                                    const unsigned long long* __restrict__ desc,
                                                    const float* __restrict__ ring, int h0_skip, LstmBinArgs pb) {
#pragma clang fp contract(off)
  const unsigned gx = gridDim.x - (unsigned)pb.blocks;  // the LSTM's workgroups
  const int bin_wg = pb.last ? (int)blockIdx.x - (int)gx : (int)blockIdx.x;
  if (bin_wg >= 0 && bin_wg < pb.blocks) {  // a binning workgroup: cells 2b and 2b + 1, a half-workgroup (4 waves) each
    const int cell = bin_wg * 2 + (int)(threadIdx.x >> 8);
    const int y = cell / pb.row_blocks, rb = cell - y * pb.row_blocks;
    if (y < pb.a.nf + pb.b.nf)
      split_bin_pair_cell(pb.X, pb.n, pb.n_pad, pb.ld, pb.a, pb.b, y, (int64_t)rb * kSplitBin + (threadIdx.x & 255));
    return;
  }
  const unsigned bx = pb.last ? blockIdx.x : blockIdx.x - (unsigned)pb.blocks;
  // h_t and x_t in the A-operand order: (txn i, k) at lane i + 4 (k & 15), register k >> 4. h_t is stored
  // register-major, [register][lane]: a lane's reads (one word per register) and the cell writes (a wave's 64
  // lanes cover 64 consecutive words of one register row) are both bank-conflict free. (Lane-major [lane][8],
  // read as two ds_read_b128, put a wave's 64 writes on 4 banks: PMC 74 % of LDS-active cycles in conflicts.)
  __shared__ __attribute__((aligned(16))) float hbuf[2][kH / 16][64];       // 4 KB
  __shared__ __attribute__((aligned(16))) float xs[FD_MAX_SEQ_LEN][64];     // 4 KB
  __shared__ float hT[4][kH];
  __shared__ float zs[4][2];
  FD_TL(g_tl_lstm, 2, 0);
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63;
  const int per = T * kI;  // sequence elements per transaction (<= 256: two staging elements per thread)
  const int64_t ntiles = (n + 3) / 4;
  // latency path: the first tile's sequence descriptors are loaded before the weights (vector loads retire in
  // order, so the ring gather below waits for these alone, and its own loads overlap the weights')
  unsigned long long dsc[2] = {0ull, 0ull};
  if (desc != nullptr && bx < ntiles) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int idx = tid + 512 * j, r = idx / per;
      if (idx < 4 * per && (int64_t)bx * 4 + r < n) dsc[j] = desc[(int64_t)bx * 4 + r];
    }
  }
  // latency_prebin 3: this thread's two searches, their values and table bounds loaded before the weights (so the
  // first level's wait does not wait for those)
  const bool inl = pb.inline_searches != 0;
  const int64_t s0 = (int64_t)bx * 512 + tid, s1 = s0 + (int64_t)gx * 512;
  InlineSearch is0{}, is1{};
  int ist = pb.steps;
  if (inl) {
    inline_search_init(pb, s0, is0);
    inline_search_init(pb, s1, is1);
  }
  // B operands: lane l holds W[(l >> 4) * 128 + 16 w + (l & 15)][k] for k = 0..143 (W_ih, then W_hh's unit blocks
  // in the order w, w+1, ..., w+7 mod 8: load_lstm)
  float bw[kKT];
#pragma unroll
  for (int k = 0; k < kKT; ++k) bw[k] = wpk4[((size_t)w * kKT + k) * 64 + l];
  const int q = l >> 4, unit = 16 * w + (l & 15);
  const int wq = __builtin_amdgcn_readfirstlane(w);
  // own units into the A-operand order: lane j takes h of transaction j & 3, unit 16 w + (j >> 2)
  const int own_src = (16 * (l & 3) + (l >> 2)) * 4;
  const float bcol = bias[q * kH + unit];
  // dense head: wave w computes output ho of transaction hr, lane l the products of units l and l + 64
  const int hr = w & 3, ho = w >> 2;
  const float wo0 = ho < n_out ? wout[ho * kH + l] : 0.f, wo1 = ho < n_out ? wout[ho * kH + 64 + l] : 0.f;
  const float bo = ho < n_out ? bout[ho] : 0.f;
  for (int64_t tile = bx; tile < ntiles; tile += gx) {
    const int64_t row0 = tile * 4;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int idx = tid + 512 * j;
      if (idx >= 4 * per) break;
      const int r = idx / per, rem = idx - r * per, t = rem / kI, k = rem - t * kI;
      float v = 0.f;
      if (row0 + r < n) {
        const unsigned long long d = desc == nullptr ? kSeqMaterialized : (tile == bx ? dsc[j] : desc[row0 + r]);
        if (d & kSeqMaterialized) {
          v = seq[(size_t)(row0 + r) * per + rem];
        } else {  // the card's ring: oldest -> newest, left-padded with zero events (features.hip seq_step)
          const int head = (int)((d >> 32) & 0xffu), sn = (int)((d >> 40) & 0xffu), pad = T - sn;
          if (t >= pad) {
            int src = head - sn + (t - pad);
            if (src < 0) src += T;
            v = ring[((size_t)(unsigned)d * T + src) * kI + k];
          }
        }
      }
      xs[t][r + 4 * k] = v;
    }
    (&hbuf[0][0][0])[tid] = 0.f;  // 512 threads = 4 x 128
    float c = 0.f, h = 0.f;
    __syncthreads();
    if (tile == bx) FD_TL(g_tl_lstm, 2, 1);
    f32x4 acc[4] = {f32x4{bcol, bcol, bcol, bcol}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                    f32x4{0.f, 0.f, 0.f, 0.f}};
    mfma_abid16(xs[0][l], &bw[0], acc, std::make_integer_sequence<int, 16>{});
    for (int t = 0; t < T; ++t) {
      const float xn = xs[t + 1 < T ? t + 1 : t][l];  // x_{t+1}, read early (its LDS latency off the barrier window)
      // latency_prebin 3: one lifting level of this thread's searches, its loads in flight behind the step
      const bool lvl = inl && tile == bx && ist > 0;
      float it0 = 0.f, it1 = 0.f;
      if (lvl) {
        it0 = inline_search_load(is0, ist);
        it1 = inline_search_load(is1, ist);
      }
      if (t > 0) {  // h_{t-1} of the other seven waves' units (blocks w+1 .. w+7), published by the last barrier
        float hv[kH / 16 - 1];
#pragma unroll
        for (int j = 1; j < kH / 16; ++j) hv[j - 1] = hbuf[t & 1][(wq + j) & (kH / 16 - 1)][l];
        mfma_abid16(hv[0], &bw[kI + 16], acc, std::make_integer_sequence<int, 16>{});
        mfma_abid16(hv[1], &bw[kI + 32], acc, std::make_integer_sequence<int, 16>{});
        mfma_abid16(hv[2], &bw[kI + 48], acc, std::make_integer_sequence<int, 16>{});
        mfma_abid16(hv[3], &bw[kI + 64], acc, std::make_integer_sequence<int, 16>{});
        mfma_abid16(hv[4], &bw[kI + 80], acc, std::make_integer_sequence<int, 16>{});
        mfma_abid16(hv[5], &bw[kI + 96], acc, std::make_integer_sequence<int, 16>{});
        mfma_abid16(hv[6], &bw[kI + 112], acc, std::make_integer_sequence<int, 16>{});
      } else if (!h0_skip) {  // W_hh h_{-1} with h_{-1} = 0, products kept (a non-finite weight makes them NaN)
#pragma unroll
        for (int j = 0; j < kH / 16; ++j) mfma_abid16(0.f, &bw[kI + 16 * j], acc, std::make_integer_sequence<int, 16>{});
      }
      // register r = transaction r of this lane's gate column; after the transpose register j = gate j of
      // transaction q
      float g0 = (acc[0][0] + acc[1][0]) + (acc[2][0] + acc[3][0]);
      float g1 = (acc[0][1] + acc[1][1]) + (acc[2][1] + acc[3][1]);
      float g2 = (acc[0][2] + acc[1][2]) + (acc[2][2] + acc[3][2]);
      float g3 = (acc[0][3] + acc[1][3]) + (acc[2][3] + acc[3][3]);
      xpose_rows4(g0, g1, g2, g3);
      const float ig = sigm(g0), fg = sigm(g1), gg = tanh_g(g2), og = sigm(g3);
      c = fg * c + ig * gg;
      h = og * tanh_g(c);
      hbuf[(t + 1) & 1][unit >> 4][q + 4 * (unit & 15)] = h;
      if (t + 1 < T) {  // step t+1's own k-steps before the barrier: x_{t+1}, then this wave's own units of h_t
        acc[0] = f32x4{bcol, bcol, bcol, bcol};
        acc[1] = acc[2] = acc[3] = f32x4{0.f, 0.f, 0.f, 0.f};
        mfma_abid16(xn, &bw[0], acc, std::make_integer_sequence<int, 16>{});
        const float ho = __int_as_float(__builtin_amdgcn_ds_bpermute(own_src, __float_as_int(h)));
        mfma_abid16(ho, &bw[kI], acc, std::make_integer_sequence<int, 16>{});
      }
      if (lvl) {
        inline_search_step(is0, ist, it0);
        inline_search_step(is1, ist, it1);
        ist >>= 1;
      }
      __syncthreads();
    }
    if (tile == bx) FD_TL(g_tl_lstm, 2, 2);
    hT[q][unit] = h;
    __syncthreads();
    if (ho < n_out) {  // dense head over h_T: a wave's 64 two-product partials, then a butterfly sum
      float z = wo0 * hT[hr][l] + wo1 * hT[hr][l + 64];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) z += __shfl_xor(z, off);
      if (l == 0) zs[hr][ho] = bo + z;
    }
    __syncthreads();
    if (tid < 4 && row0 + tid < n) {
      float p;
      if (n_out == 1) {
        p = sigm(zs[tid][0]);
      } else {
        const float m = fmaxf(zs[tid][0], zs[tid][1]);
        const float e0 = expf(zs[tid][0] - m), e1 = expf(zs[tid][1] - m);
        p = e1 / (e0 + e1);
      }
      prob[row0 + tid] = (double)p;
    }
    __syncthreads();  // xs / hbuf / hT / zs are rewritten by the next tile
  }
  if (inl) {  // the levels the recurrence did not cover, then the bins
    for (; ist > 0; ist >>= 1) {
      const float t0 = inline_search_load(is0, ist), t1 = inline_search_load(is1, ist);
      inline_search_step(is0, ist, t0);
      inline_search_step(is1, ist, t1);
    }
    inline_search_store(pb, s0, is0);
    inline_search_store(pb, s1, is1);
  }
  FD_TL(g_tl_lstm, 2, 3);
}

}  // namespace

void load_lstm(Engine& e, const fd_lstm_params& p) {
  FD_REQUIRE(p.hidden == kH, FD_ERR_UNSUPPORTED, "LSTM hidden size must be 128 (lstm_sequential hidden_units)");
  FD_REQUIRE(p.input_size >= 1 && p.input_size <= kI, FD_ERR_UNSUPPORTED, "LSTM input size must be in [1, 16]");
  FD_REQUIRE(p.n_out == 1 || p.n_out == 2, FD_ERR_UNSUPPORTED, "LSTM head must have 1 (sigmoid) or 2 (softmax) outputs");
  FD_REQUIRE(p.w_ih && p.w_hh && p.w_out, FD_ERR_INVALID_ARG, "null LSTM weights");
  const int I = p.input_size;
  // packed B operands: [wave][gate][k-step][lane] = W[g*128 + 16 wave + (lane & 15)][k], k = 4 s + (lane >> 4);
  // k-steps 0..3 from W_ih (zero beyond input_size), 4..35 from W_hh
  std::vector<float> pk((size_t)8 * 4 * kKS * 64);
  for (int w = 0; w < 8; ++w)
    for (int g = 0; g < 4; ++g)
      for (int s = 0; s < kKS; ++s)
        for (int l = 0; l < 64; ++l) {
          const int row = g * kH + 16 * w + (l & 15);
          float v;
          if (s < kI / 4) {
            const int k = 4 * s + (l >> 4);
            v = k < I ? p.w_ih[(size_t)row * I + k] : 0.f;
          } else {
            const int k = 4 * (s - kI / 4) + (l >> 4);
            v = p.w_hh[(size_t)row * kH + k];
          }
          pk[(((size_t)w * 4 + g) * kKS + s) * 64 + l] = v;
        }
  // 4-row kernel: [wave][k][lane] = W[(lane >> 4) * 128 + 16 wave + (lane & 15)][k'], k < 16 from W_ih (k' = k),
  // then W_hh's 16-unit blocks rotated so that the wave's own block comes first: k = 16 + 16 j + r holds
  // k' = 16 ((wave + j) mod 8) + r (lstm_kernel4's pipelined steps)
  std::vector<float> pk4((size_t)8 * kKT * 64);
  for (int w = 0; w < 8; ++w)
    for (int k = 0; k < kKT; ++k)
      for (int l = 0; l < 64; ++l) {
        const int row = (l >> 4) * kH + 16 * w + (l & 15);
        float v;
        if (k < kI) {
          v = k < I ? p.w_ih[(size_t)row * I + k] : 0.f;
        } else {
          const int j = (k - kI) >> 4, r = (k - kI) & 15;
          v = p.w_hh[(size_t)row * kH + 16 * ((w + j) & 7) + r];
        }
        pk4[((size_t)w * kKT + k) * 64 + l] = v;
      }
  bool hh_finite = true;
  for (size_t i = 0; i < (size_t)4 * kH * kH; ++i) hh_finite = hh_finite && std::isfinite(p.w_hh[i]);
  std::vector<float> b(4 * kH);
  for (int i = 0; i < 4 * kH; ++i) b[i] = (p.b_ih ? p.b_ih[i] : 0.f) + (p.b_hh ? p.b_hh[i] : 0.f);
  std::vector<float> wo((size_t)p.n_out * kH), bo(p.n_out);
  for (int i = 0; i < p.n_out * kH; ++i) wo[i] = p.w_out[i];
  for (int i = 0; i < p.n_out; ++i) bo[i] = p.b_out ? p.b_out[i] : 0.f;
  LstmModel& m = e.lstm;
  m.wpk.ensure(pk.size() * 4);
  m.wpk4.ensure(pk4.size() * 4);
  m.bias.ensure(b.size() * 4);
  m.wout.ensure(wo.size() * 4);
  m.bout.ensure(16);
  FD_HIP(hipMemcpy(m.wpk.ptr, pk.data(), pk.size() * 4, hipMemcpyHostToDevice));
  FD_HIP(hipMemcpy(m.wpk4.ptr, pk4.data(), pk4.size() * 4, hipMemcpyHostToDevice));
  FD_HIP(hipMemcpy(m.bias.ptr, b.data(), b.size() * 4, hipMemcpyHostToDevice));
  FD_HIP(hipMemcpy(m.wout.ptr, wo.data(), wo.size() * 4, hipMemcpyHostToDevice));
  FD_HIP(hipMemcpy(m.bout.ptr, bo.data(), bo.size() * 4, hipMemcpyHostToDevice));
  m.input_size = I;
  m.n_out = p.n_out;
  m.hh_finite = hh_finite;
  m.loaded = true;
}

void launch_lstm(Engine& e, hipStream_t stream, const float* d_seq, int64_t n, int T, double* d_prob,
                 const unsigned long long* d_desc) {
  const LstmModel& m = e.lstm;
  FD_REQUIRE(m.loaded, FD_ERR_NOT_LOADED, "Model lstm_sequential not loaded");
  FD_REQUIRE(T >= 1 && T <= FD_MAX_SEQ_LEN, FD_ERR_INVALID_ARG, "sequence length must be in [1, 16]");
  FD_REQUIRE(n >= 0 && n < (1ll << 31), FD_ERR_INVALID_ARG, "batch size out of range");
  if (n == 0) return;
  FD_REQUIRE(d_seq && d_prob, FD_ERR_INVALID_ARG, "null sequence / output");
  Engine::Timed* ev = e.timing ? e.next_event_pair(FD_TIMING_LSTM) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, stream));
  const int rows = e.lstm_rows ? e.lstm_rows : (n < 4096 ? 4 : 16);
  FD_REQUIRE(d_desc == nullptr || (rows == 4 && e.state.S == T && e.state.seq.ptr), FD_ERR_INVALID_ARG,
             "internal: sequence descriptors need the 4-row LSTM kernel and the engine's history ring");
  if (rows == 4) {  // one 512-thread workgroup per CU (bw[] holds 144 VGPRs), looping over 4-row tiles
    const int64_t tiles = (n + 3) / 4;
    LstmBinArgs pb{};
    PreBin& q = e.prebin;
    if (q.want && stream == e.stream) {  // the forest pair's binning ahead of the LSTM's workgroups (PreBin)
      pb.X = q.X;
      pb.n = q.n;
      pb.n_pad = q.n_pad;
      pb.ld = q.ld;
      pb.a = SplitBinArgs{q.thr[0], q.thr_off[0], q.bins[0], q.nan[0], q.nf[0]};
      pb.b = SplitBinArgs{q.thr[1], q.thr_off[1], q.bins[1], q.nan[1], q.nf[1]};
      pb.row_blocks = (int)(q.n_pad / kSplitBin);
      pb.blocks = (pb.row_blocks * (q.nf[0] + q.nf[1]) + 1) / 2;
      pb.last = e.latency_prebin_mode >= 2 ? 1 : 0;  // (3 falls back to 2 below)
      const int64_t searches = q.n_pad * (int64_t)(q.nf[0] + q.nf[1]);
      if (e.latency_prebin_mode == 3 && q.thr_nonempty && searches <= 2 * 512 * std::min<int64_t>(tiles, 256)) {
        pb.inline_searches = 1;  // two searches per LSTM thread at most; else the extra workgroups (2)
        pb.blocks = 0;
        pb.steps = std::max(q.steps[0], q.steps[1]);
      }
      q.done = true;
    }
    hipLaunchKernelGGL(lstm_kernel4, dim3((unsigned)(std::min<int64_t>(tiles, 256) + pb.blocks)), dim3(512), 0, stream,
                       d_seq, n, T, m.wpk4.as<const float>(), m.bias.as<const float>(), m.wout.as<const float>(),
                       m.bout.as<const float>(), m.n_out, d_prob, d_desc,
                       d_desc ? e.state.seq.as<const float>() : nullptr, m.hh_finite ? 1 : 0, pb);
  } else {
    hipLaunchKernelGGL(lstm_kernel, dim3((unsigned)((n + kRows - 1) / kRows)), dim3(512), 0, stream, d_seq, n, T,
                       m.wpk.as<const float>(), m.bias.as<const float>(), m.wout.as<const float>(),
                       m.bout.as<const float>(), m.n_out, d_prob);
  }
  FD_HIP(hipGetLastError());
  if (ev) FD_HIP(hipEventRecord(ev->b, stream));
}

}  // namespace fd

#ifdef FD_FOREST_PROFILE
extern "C" __attribute__((visibility("default"))) int fd_debug_tl_lstm(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(fd::g_tl_lstm), sizeof(fd::g_tl_lstm));
}
#endif
