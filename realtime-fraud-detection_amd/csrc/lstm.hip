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
#include <cmath>

#include "fd_internal.h"

namespace fd {
namespace {

constexpr int kH = kLstmHidden;  // 128
constexpr int kI = kSeqInput;    // 16
constexpr int kRows = 16;        // transactions per workgroup
constexpr int kKS = kI / 4 + kH / 4;  // 36 k-steps of 4

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

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
      const float ig = sigm(acc[0][j]), fg = sigm(acc[1][j]), gg = tanhf(acc[2][j]), og = sigm(acc[3][j]);
      c[j] = fg * c[j] + ig * gg;
      const float hv = og * tanhf(c[j]);
      const int r = 4 * (l >> 4) + j;
      hn[(r * 4 + (unit & 3)) * (kH / 4) + (unit >> 2)] = hv;
    }
    __syncthreads();
  }

  // dense head over h_T, fixed k order
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
  std::vector<float> b(4 * kH);
  for (int i = 0; i < 4 * kH; ++i) b[i] = (p.b_ih ? p.b_ih[i] : 0.f) + (p.b_hh ? p.b_hh[i] : 0.f);
  std::vector<float> wo((size_t)p.n_out * kH), bo(p.n_out);
  for (int i = 0; i < p.n_out * kH; ++i) wo[i] = p.w_out[i];
  for (int i = 0; i < p.n_out; ++i) bo[i] = p.b_out ? p.b_out[i] : 0.f;
  LstmModel& m = e.lstm;
  m.wpk.ensure(pk.size() * 4);
  m.bias.ensure(b.size() * 4);
  m.wout.ensure(wo.size() * 4);
  m.bout.ensure(16);
  FD_HIP(hipMemcpy(m.wpk.ptr, pk.data(), pk.size() * 4, hipMemcpyHostToDevice));
  FD_HIP(hipMemcpy(m.bias.ptr, b.data(), b.size() * 4, hipMemcpyHostToDevice));
  FD_HIP(hipMemcpy(m.wout.ptr, wo.data(), wo.size() * 4, hipMemcpyHostToDevice));
  FD_HIP(hipMemcpy(m.bout.ptr, bo.data(), bo.size() * 4, hipMemcpyHostToDevice));
  m.input_size = I;
  m.n_out = p.n_out;
  m.loaded = true;
}

void launch_lstm(Engine& e, hipStream_t stream, const float* d_seq, int64_t n, int T, double* d_prob) {
  const LstmModel& m = e.lstm;
  FD_REQUIRE(m.loaded, FD_ERR_NOT_LOADED, "Model lstm_sequential not loaded");
  FD_REQUIRE(T >= 1 && T <= FD_MAX_SEQ_LEN, FD_ERR_INVALID_ARG, "sequence length must be in [1, 16]");
  FD_REQUIRE(n >= 0 && n < (1ll << 31), FD_ERR_INVALID_ARG, "batch size out of range");
  if (n == 0) return;
  FD_REQUIRE(d_seq && d_prob, FD_ERR_INVALID_ARG, "null sequence / output");
  Engine::Timed* ev = e.timing ? e.next_event_pair(FD_TIMING_LSTM) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, stream));
  hipLaunchKernelGGL(lstm_kernel, dim3((unsigned)((n + kRows - 1) / kRows)), dim3(512), 0, stream, d_seq, n, T,
                     m.wpk.as<const float>(), m.bias.as<const float>(), m.wout.as<const float>(),
                     m.bout.as<const float>(), m.n_out, d_prob);
  FD_HIP(hipGetLastError());
  if (ev) FD_HIP(hipEventRecord(ev->b, stream));
}

}  // namespace fd
