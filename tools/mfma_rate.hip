// Micro-benchmark: issue cost and dependent latency of the f32-input MFMA forms the LSTM head uses
// (v_mfma_f32_16x16x4_f32, v_mfma_f32_4x4x1_16b_f32), one wave per SIMD, s_memtime around N MFMAs.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_rate.hip -o tools/mfma_rate && ./tools/mfma_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kN = 1024;

template <int KIND, int CHAINS>
__global__ void __launch_bounds__(256) rate(float* out, long long* cyc, float a, float b) {
  f32x4 acc[CHAINS];
  for (int c = 0; c < CHAINS; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < kN / CHAINS; ++i)
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      if (KIND == 0)
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
      else
        acc[c] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[c], 0, 0, 0);
    }
  float s = 0.f;
  for (int c = 0; c < CHAINS; ++c) s += acc[c][0] + acc[c][3];
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND, int CHAINS>
void run(const char* name, float* out, long long* cyc) {
  long long h[256];
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL((rate<KIND, CHAINS>), dim3(256), dim3(256), 0, 0, out, cyc, 1.0001f, 0.5f);
    hipDeviceSynchronize();
  }
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  long long mn = h[0];
  for (int i = 1; i < 256; ++i) mn = h[i] < mn ? h[i] : mn;
  printf("%-28s chains %2d: %6.2f cycles per MFMA per wave (min over blocks, one wave per SIMD)\n", name, CHAINS,
         (double)mn / kN);
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&cyc, 256 * 8);
  run<0, 1>("mfma_f32_16x16x4_f32", out, cyc);
  run<0, 4>("mfma_f32_16x16x4_f32", out, cyc);
  run<1, 1>("mfma_f32_4x4x1_16b_f32", out, cyc);
  run<1, 2>("mfma_f32_4x4x1_16b_f32", out, cyc);
  run<1, 4>("mfma_f32_4x4x1_16b_f32", out, cyc);
  run<1, 8>("mfma_f32_4x4x1_16b_f32", out, cyc);
  hipFree(out);
  hipFree(cyc);
  return 0;
}
