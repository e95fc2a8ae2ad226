// Accuracy of v_rsq_f64 / v_rcp_f64 with 0, 1, 2 Newton steps vs the IEEE
// 1/sqrt and 1/x (diagnostic for the LM solve's pivots).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>

__global__ void k(const double* x, double* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  double y = __builtin_amdgcn_rsq(v);
  out[6 * i + 0] = y;
  y = y * __builtin_fma(-0.5 * v * y, y, 1.5);
  out[6 * i + 1] = y;
  y = y * __builtin_fma(-0.5 * v * y, y, 1.5);
  out[6 * i + 2] = y;
  double r = __builtin_amdgcn_rcp(v);
  out[6 * i + 3] = r;
  r = __builtin_fma(r, __builtin_fma(-v, r, 1.0), r);
  out[6 * i + 4] = r;
  r = __builtin_fma(r, __builtin_fma(-v, r, 1.0), r);
  out[6 * i + 5] = r;
}

int main() {
  const int n = 1 << 20;
  double *hx = (double*)malloc(n * 8), *ho = (double*)malloc(6 * n * 8);
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const double u = (double)(s >> 11) / 9007199254740992.0;
    hx[i] = pow(10.0, -12.0 + 24.0 * u);
  }
  double *dx, *dout;
  hipMalloc(&dx, n * 8); hipMalloc(&dout, 6 * n * 8);
  hipMemcpy(dx, hx, n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dout, n);
  hipMemcpy(ho, dout, 6 * n * 8, hipMemcpyDeviceToHost);
  double e[6] = {0};
  for (int i = 0; i < n; ++i) {
    const double rs = 1.0 / sqrt(hx[i]), rc = 1.0 / hx[i];
    for (int k2 = 0; k2 < 3; ++k2) e[k2] = fmax(e[k2], fabs(ho[6 * i + k2] / rs - 1.0));
    for (int k2 = 3; k2 < 6; ++k2) e[k2] = fmax(e[k2], fabs(ho[6 * i + k2] / rc - 1.0));
  }
  printf("max rel err rsq: raw %.3e  1NR %.3e  2NR %.3e\n", e[0], e[1], e[2]);
  printf("max rel err rcp: raw %.3e  1NR %.3e  2NR %.3e\n", e[3], e[4], e[5]);
  return 0;
}
