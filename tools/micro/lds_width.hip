// LDS read cost by width for the fused kernel's walk pattern: each lane chases 8 independent chains through a 64 KiB
// LDS image, one read per chain per step, the next address = a row picked by the value read (x 1 KiB) + the lane's own
// column (conflict-free banks, as the bin tile's reads). Modes: 0 ds_read_u16, 1 ds_read_b32, 2 ds_read_b64 (column
// 8 B), 3 u16 + b64 interleaved (the walk's pair), 4 b32 + b64. Prints ns per launch and LDS read instructions per
// CU-cycle at the clock given.   hipcc --offload-arch=gfx950 -O3 lds_width.hip -o lds_width && ./lds_width
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <typename T>
__device__ __forceinline__ T ld(uint32_t a) {
  return *reinterpret_cast<const __attribute__((address_space(3))) T*>((size_t)a);
}
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ void __launch_bounds__(1024) lds_chase(unsigned* out, int iters) {
  extern __shared__ __attribute__((aligned(16))) unsigned buf[];  // 64 KiB
  const uint32_t base = (uint32_t)(size_t)((__attribute__((address_space(3))) unsigned*)buf);
  for (int i = threadIdx.x; i < 16384; i += 1024) buf[i] = (unsigned)(i * 2654435761u) ^ (unsigned)(i >> 3);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t col4 = lane * 4u, col8 = (lane & 31) * 8u;
  uint32_t a[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = base + (((uint32_t)j * 5u + (threadIdx.x >> 6)) & 63u) * 1024u + col4;
    b[j] = base + (((uint32_t)j * 7u + (threadIdx.x >> 6)) & 63u) * 1024u + col8;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint32_t v;
      if (MODE == 0 || MODE == 3) v = ld<uint16_t>(a[j]);
      else if (MODE == 1 || MODE == 4) v = ld<uint32_t>(a[j]);
      else v = ld<u32x2>(b[j]).x;
      if (MODE >= 3) {
        const u32x2 p = ld<u32x2>(b[j]);
        b[j] = base + ((p.y >> 7) & 63u) * 1024u + col8;
        v ^= p.x;
      }
      if (MODE == 2) b[j] = base + ((v >> 7) & 63u) * 1024u + col8;
      else a[j] = base + ((v >> 5) & 63u) * 1024u + col4;
    }
  }
  unsigned s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += a[j] ^ b[j];
  if (s == 0x12345678u) out[blockIdx.x] = s;
}

int main() {
  unsigned* out;
  hipMalloc(&out, 4096 * 4);
  const int iters = 2000, blocks = 256;
  const char* names[] = {"u16", "b32", "b64", "u16+b64", "b32+b64"};
  void (*ks[])(unsigned*, int) = {lds_chase<0>, lds_chase<1>, lds_chase<2>, lds_chase<3>, lds_chase<4>};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 5; ++m) {
      hipFuncSetAttribute((const void*)ks[m], hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
      hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(1024), 65536, 0, out, 10);
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(1024), 65536, 0, out, iters);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double reads = (double)iters * 8 * 16 * (m >= 3 ? 2 : 1);  // wave-instructions per CU
      const double cyc = ms * 1e-3 * 2.4e9;                              // CU cycles at 2.4 GHz
      printf("%-8s %8.3f ms  %.2f LDS cycles per wave-read (2.4 GHz)\n", names[m], ms, cyc / reads);
    }
  return 0;
}
