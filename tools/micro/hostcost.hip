// Host-cost microbenchmark (tools/micro/hostcost.hip): host microseconds per HIP call of the kinds the pipelined /
// sharded step issues — kernel launch (small and 1.5 KB argument blocks, hipLaunchKernelGGL and hipLaunchKernel),
// hipEventRecord (with / without the system-scope fence), hipStreamWaitEvent on a completed event, a D2D
// hipMemcpyAsync, hipFuncSetAttribute, and a 4-launch captured hipGraph replayed with hipGraphLaunch. Each is timed over
// 2,000 back-to-back calls on an otherwise idle stream (the GPU drains behind), median of 5 repeats.
// Build: hipcc --offload-arch=gfx950 -O2 tools/micro/hostcost.hip -o tools/micro/hostcost
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <functional>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

struct Big {
  int v[384];  // 1.5 KB, the fused kernel's argument block size
};

__global__ void k_small(int* p, int n) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && n < 0) p[0] = n;
}
__global__ void k_big(int* p, Big b) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && b.v[0] < 0) p[0] = b.v[383];
}

static double per_call_us(int calls, const std::function<void()>& f, hipStream_t st) {
  std::vector<double> r;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipStreamSynchronize(st);
    const auto a = std::chrono::steady_clock::now();
    for (int i = 0; i < calls; ++i) f();
    const auto b = std::chrono::steady_clock::now();
    r.push_back(std::chrono::duration<double, std::micro>(b - a).count() / calls);
    (void)hipStreamSynchronize(st);
  }
  std::sort(r.begin(), r.end());
  return r[2];
}

int main() {
  hipStream_t st, st2;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
  int* d = nullptr;
  CK(hipMalloc(&d, 1 << 20));
  hipEvent_t ev_fence, ev_nofence;
  CK(hipEventCreateWithFlags(&ev_fence, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ev_nofence, hipEventDisableTiming | hipEventDisableSystemFence));
  CK(hipEventRecord(ev_nofence, st2));
  CK(hipStreamSynchronize(st2));
  Big big{};
  const int N = 2000;
  std::printf("launch small (GGL, 1 block)         %.2f us\n",
              per_call_us(N, [&] { hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, st, d, 1); }, st));
  std::printf("launch small (GGL, 256 blocks)      %.2f us\n",
              per_call_us(N, [&] { hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, st, d, 1); }, st));
  std::printf("launch 1.5 KB args (GGL)            %.2f us\n",
              per_call_us(N, [&] { hipLaunchKernelGGL(k_big, dim3(256), dim3(1024), 0, st, d, big); }, st));
  {
    void* args[] = {&d, &big};
    std::printf("launch 1.5 KB args (hipLaunchKernel) %.2f us\n",
                per_call_us(N, [&] { (void)hipLaunchKernel((const void*)k_big, dim3(256), dim3(1024), args, 0, st); }, st));
  }
  std::printf("hipEventRecord (system fence)       %.2f us\n",
              per_call_us(N, [&] { (void)hipEventRecord(ev_fence, st); }, st));
  std::printf("hipEventRecord (no system fence)    %.2f us\n",
              per_call_us(N, [&] { (void)hipEventRecord(ev_nofence, st); }, st));
  CK(hipEventRecord(ev_nofence, st2));
  CK(hipStreamSynchronize(st2));
  std::printf("hipStreamWaitEvent (completed)      %.2f us\n",
              per_call_us(N, [&] { (void)hipStreamWaitEvent(st, ev_nofence, 0); }, st));
  std::printf("launch + record + wait (3 calls)    %.2f us\n", per_call_us(N, [&] {
                hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, st, d, 1);
                (void)hipEventRecord(ev_nofence, st);
                (void)hipStreamWaitEvent(st2, ev_nofence, 0);
              }, st));
  {
    uint64_t* flag = nullptr;
    CK(hipMalloc(&flag, 64));
    CK(hipMemset(flag, 0, 64));
    uint64_t v = 0;
    std::printf("hipStreamWriteValue64               %.2f us\n",
                per_call_us(N, [&] { (void)hipStreamWriteValue64(st, flag, ++v, 0); }, st));
    std::printf("hipStreamWaitValue64 (satisfied)    %.2f us\n",
                per_call_us(N, [&] { (void)hipStreamWaitValue64(st2, flag, 1, hipStreamWaitValueGte, ~0ull); }, st2));
    CK(hipStreamSynchronize(st2));
    CK(hipFree(flag));
  }
  std::printf("hipMemcpyAsync D2D 256 KB           %.2f us\n",
              per_call_us(N, [&] { (void)hipMemcpyAsync(d + (1 << 17), d, 1 << 18, hipMemcpyDeviceToDevice, st); }, st));
  std::printf("hipFuncSetAttribute (max dyn LDS)   %.2f us\n", per_call_us(N, [&] {
                (void)hipFuncSetAttribute((const void*)k_big, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
              }, st));
  std::printf("hipGetLastError                     %.2f us\n", per_call_us(N, [&] { (void)hipGetLastError(); }, st));
  // a captured 4-launch graph
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, st, d, 1);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  std::printf("4 launches, one by one               %.2f us\n", per_call_us(N / 4, [&] {
                for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, st, d, 1);
              }, st));
  std::printf("4 launches as hipGraphLaunch          %.2f us\n",
              per_call_us(N / 4, [&] { (void)hipGraphLaunch(ge, st); }, st));
  CK(hipStreamSynchronize(st));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipFree(d));
  return 0;
}
