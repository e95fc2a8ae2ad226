// Do independent branches of a hipGraph run concurrently on gfx950?
// Two kernels that each keep their workgroups busy for ~T us (s_memrealtime
// spin, bounded) are captured (a) back to back on one stream and (b) on two
// streams forked / joined by events; the replay time of (b) against (a) says
// whether the graph runtime overlaps branches.  Variant (c): a 256-workgroup
// "grid" kernel on the main branch and a 1-workgroup kernel on the side branch
// (the LM factorisation overlap this is meant to decide).
// build: hipcc --offload-arch=gfx950 -O2 tools/micro/graph_fork.hip -o /tmp/graph_fork
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                             \
    }                                                                       \
  } while (0)

// spin for `ticks` of the 100 MHz realtime counter, then a vector store
__global__ void k_spin(unsigned long long ticks, float* out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned it = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks && it < (1u << 22)) {
    __builtin_amdgcn_s_sleep(1);
    ++it;
  }
  if (threadIdx.x == 0) out[blockIdx.x] = (float)it;
}

static double replay_us(hipGraphExec_t ge, hipStream_t s, int reps) {
  for (int i = 0; i < 3; ++i) hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; ++i) hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  const auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

int main() {
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  float* out;
  CK(hipMalloc(&out, 4096 * sizeof(float)));
  const unsigned long long T = 2000;  // 20 us at 100 MHz
  const int NK = 20;                   // kernel pairs per graph
  for (const unsigned long long T2 : {500ull, 1500ull}) {
  for (int grid_main : {256}) {
    for (int variant = 0; variant < 3; ++variant) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
      for (int k = 0; k < NK; ++k) {
        if (variant == 0) {
          hipLaunchKernelGGL(k_spin, dim3(grid_main), dim3(256), 0, s0, T, out);
          hipLaunchKernelGGL(k_spin, dim3(1), dim3(256), 0, s0, T2, out + 2048);
        } else {
          CK(hipEventRecord(fork, s0));
          CK(hipStreamWaitEvent(s1, fork, 0));
          hipLaunchKernelGGL(k_spin, dim3(1), dim3(256), 0, s1, T2, out + 2048);
          hipLaunchKernelGGL(k_spin, dim3(grid_main), dim3(256), 0, s0, T, out);
          if (variant == 1 || k == NK - 1) {  // variant 2: one join at the end (fork cost alone)
            CK(hipEventRecord(join, s1));
            CK(hipStreamWaitEvent(s0, join, 0));
          }
        }
      }
      CK(hipStreamEndCapture(s0, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      const double us = replay_us(ge, s0, 20);
      std::printf("main grid %3d (20 us), side %4.1f us, %s: %.1f us per pair (%d pairs)\n", grid_main,
                  T2 / 100.0, variant == 0 ? "serial" : variant == 1 ? "fork+join" : "fork only", us / NK, NK);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  }
  CK(hipFree(out));
  return 0;
}
