// fp64 vs fp32 FMA issue cost and dependent latency on one gfx950 wave, plain
// and with a 64-bit / 32-bit DPP row_newbcast operand (the Cholesky panel's
// v_fmac_*_dpp form, csrc/lm_chol.h), and packed fp32 (v_pk_fma_f32, which has
// no DPP form).  Decides whether an fp32 panel factorisation could issue
// faster than the fp64 one.  Cycles from s_memtime (the shader clock).
// build: hipcc --offload-arch=gfx950 -O2 tools/micro/fma_rate.hip -o tools/micro/fma_rate.bin
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int N = 1024;  // instructions per chain

template <int CH>
__global__ void k_f64(double* out, unsigned long long* cyc, double s) {
  double a[CH];
  for (int c = 0; c < CH; ++c) a[c] = threadIdx.x * 1e-3 + c;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < N / CH; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(a[c]) : "v"(s), "v"(s));
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double r = 0;
  for (int c = 0; c < CH; ++c) r += a[c];
  out[threadIdx.x] = r;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int CH>
__global__ void k_f64_dpp(double* out, unsigned long long* cyc, double s) {
  double a[CH];
  for (int c = 0; c < CH; ++c) a[c] = threadIdx.x * 1e-3 + c;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < N / CH; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c)
      asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a[c]) : "v"(s), "v"(s));
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double r = 0;
  for (int c = 0; c < CH; ++c) r += a[c];
  out[threadIdx.x] = r;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int CH>
__global__ void k_f32(double* out, unsigned long long* cyc, double sd) {
  const float s = (float)sd;
  float a[CH];
  for (int c = 0; c < CH; ++c) a[c] = threadIdx.x * 1e-3f + c;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < N / CH; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[c]) : "v"(s), "v"(s));
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0;
  for (int c = 0; c < CH; ++c) r += a[c];
  out[threadIdx.x] = r;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int CH>
__global__ void k_f32_dpp(double* out, unsigned long long* cyc, double sd) {
  const float s = (float)sd;
  float a[CH];
  for (int c = 0; c < CH; ++c) a[c] = threadIdx.x * 1e-3f + c;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < N / CH; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c)
      asm volatile("v_fmac_f32_dpp %0, %1, -%2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a[c]) : "v"(s), "v"(s));
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0;
  for (int c = 0; c < CH; ++c) r += a[c];
  out[threadIdx.x] = r;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

typedef float f2 __attribute__((ext_vector_type(2)));
template <int CH>
__global__ void k_pk_f32(double* out, unsigned long long* cyc, double sd) {
  const f2 s = {(float)sd, (float)sd};
  f2 a[CH];
  for (int c = 0; c < CH; ++c) a[c] = f2{threadIdx.x * 1e-3f + c, (float)c};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < N / CH; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a[c]) : "v"(s), "v"(s));
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0;
  for (int c = 0; c < CH; ++c) r += a[c].x + a[c].y;
  out[threadIdx.x] = r;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <class K>
static double run(K kern, double* out, unsigned long long* cyc) {
  unsigned long long h = 0, best = ~0ull;
  for (int rep = 0; rep < 5; ++rep) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, out, cyc, 1.0000001);
    if (hipDeviceSynchronize() != hipSuccess) return -1.0;
    if (hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return -1.0;
    if (h < best) best = h;
  }
  return (double)best / N;  // cycles per instruction
}

int main() {
  double* out;
  unsigned long long* cyc;
  if (hipMalloc(&out, 64 * sizeof(double)) != hipSuccess || hipMalloc(&cyc, sizeof(unsigned long long)) != hipSuccess)
    return 1;
  std::printf("cycles per instruction, one wave64 (1 chain = dependent latency, 8 chains = issue rate)\n");
  std::printf("v_fmac_f64       1: %5.2f  8: %5.2f\n", run(k_f64<1>, out, cyc), run(k_f64<8>, out, cyc));
  std::printf("v_fmac_f64_dpp   1: %5.2f  8: %5.2f\n", run(k_f64_dpp<1>, out, cyc), run(k_f64_dpp<8>, out, cyc));
  std::printf("v_fmac_f32       1: %5.2f  8: %5.2f\n", run(k_f32<1>, out, cyc), run(k_f32<8>, out, cyc));
  std::printf("v_fmac_f32_dpp   1: %5.2f  8: %5.2f\n", run(k_f32_dpp<1>, out, cyc), run(k_f32_dpp<8>, out, cyc));
  std::printf("v_pk_fma_f32     1: %5.2f  8: %5.2f  (2 fp32 fmas each)\n", run(k_pk_f32<1>, out, cyc),
              run(k_pk_f32<8>, out, cyc));
  (void)hipFree(out);
  (void)hipFree(cyc);
  return 0;
}
