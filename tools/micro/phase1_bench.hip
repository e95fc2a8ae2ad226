// Micro-benchmark of the LM Cholesky's phase 1 (csrc/hedge_lm.hip): per
// panel, row threads factor the 8x8 diagonal block from an LDS-broadcast
// panel and solve their L21 row.  Variants isolate the cost of the parts:
//   0 full phase 1 (+ barrier)      1 barrier only
//   2 loads + stores, no arithmetic 3 diag block only (no row solve)
//   4 full, but rsq without Newton   5 full with one thread row (k0 = 104)
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ double rsq1(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  return y * __builtin_fma(-0.5 * x * y, y, 1.5);
}

template <int V>
__global__ __launch_bounds__(256) void k(double* out, unsigned long long* t, int iters, int kfix) {
  __shared__ double cb[8][128];
  __shared__ double uL[128][9];
  const int tid = threadIdx.x;
  for (int e = tid; e < 8 * 128; e += 256) {
    const int c = e >> 7, i = e & 127;
    cb[c][i] = (i == c) ? 4.0 : 0.01 * ((i * 7 + c * 3) % 11);
  }
  __syncthreads();
  double acc = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
    const int k0 = V == 5 ? 104 : V == 6 ? kfix : V == 7 ? 0 : V == 8 ? kfix + 0 * it : 8 * (it % 13);
    __syncthreads();
    if (V == 1) continue;
    if (tid >= k0 && tid < 112) {
      double L[8][8], rl[8];
      if (V == 2) {
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < 8; ++c)
#pragma unroll
          for (int r = c; r < 8; ++r) s += cb[c][k0 + r];
#pragma unroll
        for (int c = 0; c < 8; ++c) uL[tid][c] = s + cb[c][tid];
        continue;
      }
      if (V == 9 || V == 10) {
        // right-looking 8x8 factor: column c scaled, then the trailing
        // entries updated at once (short dependency chain per pivot)
        double a[8][8];
#pragma unroll
        for (int c = 0; c < 8; ++c)
#pragma unroll
          for (int r = c; r < 8; ++r) a[r][c] = cb[c][k0 + r];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          rl[c] = rsq1(a[c][c]);
          L[c][c] = a[c][c] * rl[c];
#pragma unroll
          for (int r = c + 1; r < 8; ++r) L[r][c] = a[r][c] * rl[c];
#pragma unroll
          for (int q = c + 1; q < 8; ++q)
#pragma unroll
            for (int r = q; r < 8; ++r) a[r][q] = __builtin_fma(-L[r][c], L[q][c], a[r][q]);
        }
        if (V == 9) {
          acc += L[7][7];
          continue;
        }
      } else
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        double sc = cb[c][k0 + c];
#pragma unroll
        for (int p = 0; p < c; ++p) sc -= L[c][p] * L[c][p];
        rl[c] = V == 4 ? __builtin_amdgcn_rsq(sc) : rsq1(sc);
        L[c][c] = sc * rl[c];
#pragma unroll
        for (int r = c + 1; r < 8; ++r) {
          double v = cb[c][k0 + r];
#pragma unroll
          for (int p = 0; p < c; ++p) v -= L[r][p] * L[c][p];
          L[r][c] = v * rl[c];
        }
      }
      if (V == 3) {
        acc += L[7][7];
        continue;
      }
      if (tid >= k0 + 8) {
        double u[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          double v = cb[c][tid];
#pragma unroll
          for (int p = 0; p < c; ++p) v -= u[p] * L[c][p];
          u[c] = v * rl[c];
          uL[tid][c] = u[c];
        }
      } else {
        acc += L[tid - k0][0];
      }
    }
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long c1 = __builtin_readcyclecounter();
  out[tid] = acc + uL[tid & 127][tid & 7];
  if (tid == 0) {
    t[0] = t1 - t0;
    t[1] = c1 - c0;
  }
}

template <int V>
void run(const char* name, int kf = 0) {
  double* o; unsigned long long* t;
  hipMalloc(&o, 256 * 8); hipMalloc(&t, 16);
  const int iters = 1300;
  hipLaunchKernelGGL(k<V>, dim3(1), dim3(256), 0, 0, o, t, iters, kf);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(k<V>, dim3(1), dim3(256), 0, 0, o, t, iters, kf);
  unsigned long long h[2]; hipMemcpy(h, t, 16, hipMemcpyDeviceToHost);
  printf("%-36s %.1f ns per panel  %.0f shader cycles per panel  (clock %.2f GHz)\n", name, h[0] * 10.0 / iters,
         (double)h[1] / iters, h[1] / (h[0] * 10.0));
  hipFree(o); hipFree(t);
}

int main() {
  run<1>("barrier only");
  run<2>("loads + stores");
  run<3>("diag block factor only");
  run<0>("full phase 1");
  run<4>("full, raw rsq (no Newton)");
  run<5>("full, 8 row threads (k0=104)");
  run<6>("full, runtime k0=104 (8 row threads)", 104);
  run<7>("full, static k0=0 (112 row threads)");
  run<8>("full, runtime k0=0 (112 row threads)", 0);
  run<6>("full, runtime k0=56 (56 row threads)", 56);
  run<9>("diag block factor only, right-looking");
  run<10>("full phase 1, right-looking diag");
  return 0;
}
