// Stream-gap microbenchmark (tools/micro/evgap.hip): the time from one kernel's end to the next kernel's start on
// the same stream, with nothing between them, a hipEventRecord (with / without the system-scope fence), a hipStreamWaitEvent on an event that completed
// long before, or stream memory operations (hipStreamWriteValue32 / hipStreamWaitValue32 already satisfied).
// Kernel A spins ~40 us on the GPU's 100 MHz clock and stamps its end; kernel B stamps its start (one thread each,
// vector stores). Build: hipcc --offload-arch=gfx950 -O2 tools/micro/evgap.hip -o tools/micro/evgap
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

__global__ void spin_end(unsigned long long* out, int slot, unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) out[2 * slot] = __builtin_amdgcn_s_memrealtime();
}

__global__ void stamp_start(unsigned long long* out, int slot) {
  if (threadIdx.x == 0) out[2 * slot + 1] = __builtin_amdgcn_s_memrealtime();
}

int main() {
  const int reps = 200;
  unsigned long long* d = nullptr;
  CK(hipMalloc(&d, sizeof(unsigned long long) * 2 * reps));
  unsigned int* flag = nullptr;
  CK(hipMalloc(&flag, 64));
  CK(hipMemset(flag, 0, 64));
  hipStream_t s, o;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&o, hipStreamNonBlocking));
  hipEvent_t ev, evnf, done;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&evnf, hipEventDisableTiming | hipEventDisableSystemFence));
  CK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
  CK(hipEventRecord(done, o));  // completes at once: "a wait on an event that completed long before"
  CK(hipStreamSynchronize(o));
  const char* names[] = {"nothing", "hipEventRecord", "hipStreamWaitEvent (done)", "hipStreamWriteValue32",
                         "hipStreamWaitValue32 (satisfied)", "hipEventRecord (no system fence)"};
  for (int variant = 0; variant < 6; ++variant) {
    for (int r = 0; r < reps; ++r) {
      hipLaunchKernelGGL(spin_end, dim3(1), dim3(64), 0, s, d, r, 4000ull);  // 40 us
      if (variant == 1) CK(hipEventRecord(ev, s));
      if (variant == 2) CK(hipStreamWaitEvent(s, done, 0));
      if (variant == 3) CK(hipStreamWriteValue32(s, flag, (uint32_t)r + 1, 0));
      if (variant == 4) CK(hipStreamWaitValue32(s, flag + 4, 0, hipStreamWaitValueGte, 0xffffffffu));
      if (variant == 5) CK(hipEventRecord(evnf, s));
      hipLaunchKernelGGL(stamp_start, dim3(1), dim3(64), 0, s, d, r);
    }
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(2 * reps);
    CK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> g;
    for (int r = 10; r < reps; ++r) g.push_back((double)(h[2 * r + 1] - h[2 * r]) * 10.0 / 1000.0);  // us
    std::sort(g.begin(), g.end());
    std::printf("%-34s gap median %6.2f us  p10 %6.2f  p90 %6.2f\n", names[variant], g[g.size() / 2],
                g[g.size() / 10], g[g.size() * 9 / 10]);
  }
  return 0;
}
