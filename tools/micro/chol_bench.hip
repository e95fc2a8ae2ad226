// Micro-benchmark of the per-column cost of a one-workgroup Cholesky step on
// gfx950 (diagnostic for k_lm_solve): variant 0 = barrier only, 1 = barrier +
// column broadcast reads, 2 = + register tile update (fp64), 3 = same in fp32.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int V, typename T>
__global__ __launch_bounds__(256) void k_steps(T* out, int P, unsigned long long* t) {
  __shared__ T colb[2][128];
  const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15, wid = tid >> 6;
  T Rg[8][8];
  for (int a = 0; a < 8; ++a)
    for (int b = 0; b < 8; ++b) Rg[a][b] = (T)((ty + 16 * a) == (tx + 16 * b) ? 100.0 : 0.01);
  if (tid < 128) { colb[0][tid] = 1.0; colb[1][tid] = 1.0; }
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int k = 0; k < P; ++k) {
    __syncthreads();
    if (V >= 1 && V != 4) {
      const T* ck = colb[k & 1];
      const T akk = ck[k];
      T rk = V == 4 ? (T)1.0 / akk : (T)__builtin_amdgcn_rcp((double)akk);
      T ri[8], cj[8];
#pragma unroll
      for (int a = 0; a < 8; ++a) ri[a] = ck[ty + 16 * a] * rk;
#pragma unroll
      for (int b = 0; b < 8; ++b) cj[b] = ck[tx + 16 * b];
      if (V >= 2) {
        const int bk = k >> 4;
        const bool la = tx > k - 16 * bk;
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          if (16 * a + wid * 4 + 3 <= k) continue;
#pragma unroll
          for (int b = 0; b <= a; ++b) {
            if (b < bk) continue;
            const T v = Rg[a][b] - ri[a] * cj[b];
            Rg[a][b] = (b > bk || la) ? v : Rg[a][b];
          }
        }
      } else {
#pragma unroll
        for (int a = 0; a < 8; ++a) Rg[a][0] += ri[a] * cj[a];
      }
      if (tx == ((k + 1) & 15)) {
        T* cn = colb[(k + 1) & 1];
#pragma unroll
        for (int a = 0; a < 8; ++a) cn[ty + 16 * a] = (T)1.0 + Rg[a][0] * (T)1e-9;
      }
    }
  }
  if (V == 4) { T q = (T)1.0; for (int k = 0; k < P; ++k) { __syncthreads(); q = (T)1.0 / (q + colb[0][k]); } Rg[0][0] = q; }
  __syncthreads();
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  T s = 0;
  for (int a = 0; a < 8; ++a)
    for (int b = 0; b < 8; ++b) s += Rg[a][b];
  out[tid] = s;
  if (tid == 0) *t = t1 - t0;
}

template <int V, typename T>
void run(const char* name, int P) {
  T* o; unsigned long long* t;
  hipMalloc(&o, 256 * sizeof(T)); hipMalloc(&t, 8);
  hipLaunchKernelGGL((k_steps<V, T>), dim3(1), dim3(256), 0, 0, o, P, t);
  hipDeviceSynchronize();
  hipLaunchKernelGGL((k_steps<V, T>), dim3(1), dim3(256), 0, 0, o, P, t);
  unsigned long long h; hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
  printf("%-28s P=%d  %.2f us  (%.1f ns/step)\n", name, P, h / 100.0, h * 10.0 / P);
  hipFree(o); hipFree(t);
}

int main() {
  run<0, double>("barrier only", 106);
  run<1, double>("barrier+bcast reads fp64", 106);
  run<2, double>("register update fp64", 106);
  run<2, float>("register update fp32", 106);
  run<4, double>("fp64 IEEE division only", 106);
  run<0, double>("barrier only", 1000);
  return 0;
}
