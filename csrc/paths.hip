// rphedge — Monte-Carlo path generation for gfx950:
//   K1  scrambled Sobol (index-addressable, bit-exact with scipy.stats.qmc.Sobol)
//   K2  inverse normal CDF fused into K1 (fp32 Giles / fp64 Acklam+Halley)
//   K3  GBM scans (arithmetic Euler RP:64-65, log-Euler EO:161-165), basket
//   K4  SV scans (reference CIR-on-sigma RP:282-289; full-truncation Heston)
//   K5+K6 mortality intensity Euler + binomial survivors (RP:71-84)
//   K7  payoffs (guarantee RP:88/:184, call/put EO:328-329, basket call)
//
// One thread per path; the time recursion lives in registers; Sobol normals
// are regenerated on the fly (W is never stored); only the coarse rebalancing
// grid (every `reduction` fine steps, RP:92-96) is written, time-major
// [n_coarse][n_local] so each date is one coalesced row per wave.
#include "rph_common.h"
#include "rph_types.h"

namespace rph {
int rph_report(const char* what, const char* msg);  // runtime.cpp
}

namespace rph {

template <typename Real>
RPH_INLINE Real ndtri_u30(uint32_t x);
template <>
RPH_INLINE float ndtri_u30<float>(uint32_t x) {
  x = x == 0u ? 1u : x;  // fp32 path: keep samples finite (x==0 has probability 2^-30)
  return ndtri_u30_f32(x);
}
template <>
RPH_INLINE double ndtri_u30<double>(uint32_t x) {
  return ndtri_u30_f64(x);
}

// Standalone K1+K2: out[i*d + j] (path-major like scipy) of N(0,1) draws.
template <typename Real, bool ALIGNED>
__global__ __launch_bounds__(256) void k_sobol_normal(Real* __restrict__ out, int n, int d,
                                                      const uint32_t* __restrict__ sv,
                                                      const uint32_t* __restrict__ shift,
                                                      long long offset, int raw) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (ALIGNED == false && i >= n) return;
  const uint32_t g = gray_code((uint64_t)(offset + i));
  for (int j = 0; j < d; ++j) {
    const uint32_t x = sobol_point<ALIGNED>(sv + (size_t)j * 32, shift[j], g);
    Real v;
    if (raw) v = (Real)x * (Real)9.313225746154785e-10;
    else v = ndtri_u30<Real>(x);
    if (i < n) out[(size_t)i * d + j] = v;
  }
}

// global (Sobol / Philox) index of local path p (SimDesc.map_blk: the LM Gram
// subsample, a few aligned blocks of the global range, simulated on every rank)
RPH_INLINE long long sim_gidx(const SimDesc& d, int p) {
  return d.map_blk > 0 ? d.path_offset + ((long long)p / d.map_blk) * d.map_stride + (long long)p % d.map_blk
                       : d.path_offset + p;
}

// ---------------------------------------------------------------------------
// Single-asset / SV / Heston / mortality scans.
// ---------------------------------------------------------------------------
template <typename Real, bool ALIGNED, int MODEL>
__global__ __launch_bounds__(256) void k_sim_scan(const SimDesc d) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (!ALIGNED && p >= d.n_local) return;
  const long long gp = sim_gidx(d, p);
  const uint32_t g = gray_code((uint64_t)gp);
  const Real dt = (Real)d.dt;
  const Real sdt = sqrt(dt);
  const Real mu = (Real)d.mu[0], sig = (Real)d.sigma[0];
  const float inv0 = (float)d.inv_norm[0];
  const size_t n = (size_t)d.n_local;

  if (MODEL == SIM_GBM_ARITH || MODEL == SIM_GBM_LOG) {
    Real y = (MODEL == SIM_GBM_LOG) ? log((Real)d.s0[0]) : (Real)d.s0[0];
    const Real drift = (MODEL == SIM_GBM_LOG) ? (mu - (Real)0.5 * sig * sig) * dt : mu * dt;
    const Real vol = sig * sdt;
    d.out[p] = (float)d.s0[0] * inv0;
    for (int t = 1; t < d.n_fine; ++t) {
      const Real z = ndtri_u30<Real>(sobol_point<ALIGNED>(d.sv1 + (size_t)t * 32, d.shift1[t], g));
      if (MODEL == SIM_GBM_LOG) y += drift + vol * z;
      else y = y + y * (drift + vol * z);
      if (t % d.reduction == 0) {
        const int c = t / d.reduction;
        const Real s = (MODEL == SIM_GBM_LOG) ? exp(y) : y;
        if (c < d.n_coarse) d.out[(size_t)c * n + p] = (float)s * inv0;
      }
    }
    const Real s = (MODEL == SIM_GBM_LOG) ? exp(y) : y;
    if (d.final_out) d.final_out[p] = (float)s * inv0;
  } else if (MODEL == SIM_SV_REF || MODEL == SIM_HESTON) {
    // table 1 -> price shocks (W1, seed 1235), table 2 -> variance shocks (W_SV)
    Real ly = log((Real)d.s0[0]);
    Real v = (Real)d.v0;
    d.out[p] = (float)d.s0[0] * inv0;
    if (d.out2) d.out2[p] = (float)v;
    const Real rho = (Real)d.rho, rhoc = sqrt((Real)1 - rho * rho);
    // Andersen (2008) QE constants (uniform over the launch): variance moments
    // m = theta + (v - theta) e^{-kappa dt}, s^2 = v*qc1 + qc2; log-price
    // central discretisation gamma1 = gamma2 = 1/2 (K1..K4) with the
    // martingale-corrected K0* (E[S_{t+dt}] = S_t e^{mu dt} exactly)
    const Real kap = (Real)d.kappa, th = (Real)d.theta, xi = (Real)d.xi;
    const Real ekd = exp(-kap * dt);
    const Real qc1 = xi * xi * ekd * ((Real)1 - ekd) / kap;
    const Real qc2 = th * xi * xi * ((Real)1 - ekd) * ((Real)1 - ekd) / ((Real)2 * kap);
    const Real qK1 = (Real)0.5 * dt * (kap * rho / xi - (Real)0.5) - rho / xi;
    const Real qK2 = (Real)0.5 * dt * (kap * rho / xi - (Real)0.5) + rho / xi;
    const Real qK3 = (Real)0.5 * dt * ((Real)1 - rho * rho);
    const Real qA = qK2 + (Real)0.5 * qK3;
    const Real qK0u = -rho * kap * th * dt / xi;  // uncorrected K0 (when the correction does not exist)
    const bool qe = MODEL == SIM_HESTON && d.scheme == HESTON_QE;
    const Real tau = (Real)d.sv_tscale * dt;  // SV_REF corrected: calibration-day time step
    for (int t = 1; t < d.n_fine; ++t) {
      const Real z1 = ndtri_u30<Real>(sobol_point<ALIGNED>(d.sv1 + (size_t)t * 32, d.shift1[t], g));
      const uint32_t x2 = sobol_point<ALIGNED>(d.sv2 + (size_t)t * 32, d.shift2[t], g);
      if (MODEL == SIM_SV_REF) {
        const Real z2 = ndtri_u30<Real>(x2);
        if (d.sv_tscale > 0.0) {
          // corrected CIR-on-sigma: rates in calibration-day units, full
          // truncation, price shock with the start-of-step volatility
          const Real vp = v > (Real)0 ? v : (Real)0;
          ly += (mu - (Real)0.5 * vp * vp) * dt + vp * sdt * z1;
          v = v + (Real)d.a * ((Real)d.b - vp) * tau + (Real)d.c * sqrt(vp * tau) * z2;
        } else {
          // RP:285  vt = vt + a(b - vt) + c sqrt(vt dt) W_SV   (no dt on the drift: Q5)
          const Real arg = v * dt;
          const Real sq = d.parity ? sqrt(arg) : sqrt(arg > (Real)0 ? arg : (Real)0);  // parity: NaN like numpy
          v = v + (Real)d.a * ((Real)d.b - v) + (Real)d.c * sq * z2;
          // RP:287  logY += (mu - vt^2/2) dt + vt sqrt(dt) W1   (vt used as a volatility)
          ly += (mu - (Real)0.5 * v * v) * dt + v * sdt * z1;
        }
      } else if (qe) {
        const Real m = th + (v - th) * ekd;
        const Real s2 = v * qc1 + qc2;
        const Real psi = s2 / (m * m);
        Real vn, k0;
        if (psi <= (Real)1.5) {  // quadratic branch: v' = a (b + Z)^2
          const Real z2 = ndtri_u30<Real>(x2);
          const Real ip = (Real)2 / psi;
          const Real b2 = ip - (Real)1 + sqrt(ip) * sqrt(ip - (Real)1);
          const Real qa = m / ((Real)1 + b2);
          const Real bz = sqrt(b2) + z2;
          vn = qa * bz * bz;
          const Real den = (Real)1 - (Real)2 * qA * qa;
          k0 = den > (Real)0 ? -qA * b2 * qa / den + (Real)0.5 * log(den) - (qK1 + (Real)0.5 * qK3) * v : qK0u;
        } else {  // exponential branch: point mass p at 0, exponential tail (inverse CDF of the uniform)
          const Real p = (psi - (Real)1) / (psi + (Real)1);
          const Real beta = ((Real)1 - p) / m;
          const Real u = (Real)x2 * (Real)9.313225746154785e-10;
          vn = u <= p ? (Real)0 : log(((Real)1 - p) / ((Real)1 - u)) / beta;
          k0 = beta > qA ? -log(p + beta * ((Real)1 - p) / (beta - qA)) - (qK1 + (Real)0.5 * qK3) * v : qK0u;
        }
        const Real var = qK3 * (v + vn);
        ly += mu * dt + k0 + qK1 * v + qK2 * vn + sqrt(var > (Real)0 ? var : (Real)0) * z1;
        v = vn;
      } else {
        const Real z2 = ndtri_u30<Real>(x2);
        const Real vp = v > (Real)0 ? v : (Real)0;
        const Real sv = sqrt(vp * dt);
        ly += (mu - (Real)0.5 * vp) * dt + sv * (rho * z2 + rhoc * z1);
        v = v + (Real)d.kappa * ((Real)d.theta - vp) * dt + (Real)d.xi * sv * z2;
      }
      if (t % d.reduction == 0) {
        const int c = t / d.reduction;
        if (c < d.n_coarse) {
          d.out[(size_t)c * n + p] = (float)exp(ly) * inv0;
          if (d.out2) d.out2[(size_t)c * n + p] = (float)v;
        }
      }
    }
    if (d.final_out) d.final_out[p] = (float)exp(ly) * inv0;
  } else if (MODEL == SIM_MORTALITY) {
    // RP:73-76 lambda Euler (Sobol seed 1234); RP:78-84 N_t ~ Binom(N_{t-1}, exp(-lambda_t dt)).
    Real lam = (Real)d.l0;
    int N = d.n0;
    const float invn = 1.0f / (float)d.n0;
    d.out2[p] = 1.0f;
    if (d.out3) d.out3[p] = (float)lam;
    const Real lc = (Real)d.lc, eta_sdt = (Real)d.eta * sdt;
    for (int t = 1; t < d.n_fine; ++t) {
      const Real z = ndtri_u30<Real>(sobol_point<ALIGNED>(d.sv2 + (size_t)t * 32, d.shift2[t], g));
      lam = lam + (lc * lam * dt + eta_sdt * z);
      // binomial deaths by inversion (mean N q << 1 per fine step)
      double q = 1.0 - exp(-(double)lam * (double)dt);
      q = q < 0.0 ? 0.0 : (q > 1.0 ? 1.0 : q);
      if (N > 0 && q > 0.0) {
        const u32x4 r = philox4x32_10({(uint32_t)gp, (uint32_t)(gp >> 32),
                                       (uint32_t)t, 0xB1A0u},
                                      d.seed, 0x1234u);
        const double u = u01d(r.x, r.y);
        const double mean = (double)N * q;
        int D;
        if (mean < 200.0 && q < 1.0) {
          double f = exp((double)N * log1p(-q));  // P(D = 0)
          double F = f;
          const double ratio = q / (1.0 - q);
          D = 0;
          while (u > F && D < N) {
            f *= (double)(N - D) / (double)(D + 1) * ratio;
            ++D;
            F += f;
            if (f < 1e-300 && F < u) { break; }
          }
        } else {
          // normal approximation (never reached by the reference configurations)
          const double z2n = ndtri_u30<double>((uint32_t)(u * 1073741824.0) | 1u);
          double dd = mean + sqrt(mean * (1.0 - q)) * z2n + 0.5;
          dd = dd < 0.0 ? 0.0 : (dd > (double)N ? (double)N : dd);
          D = (int)dd;
        }
        N -= D;
      }
      if (d.parity) {  // Q3: lambda is NOT subsampled in the reference (RP:200 uses fine index t_i)
        if (t < d.n_coarse && d.out3) d.out3[(size_t)t * n + p] = (float)lam;
      }
      if (t % d.reduction == 0) {
        const int c = t / d.reduction;
        if (c < d.n_coarse) {
          d.out2[(size_t)c * n + p] = (float)N * invn;
          if (!d.parity && d.out3) d.out3[(size_t)c * n + p] = (float)lam;
        }
      }
    }
    if (d.final2_out) d.final2_out[p] = (float)N * invn;
  }
}

// ---------------------------------------------------------------------------
// Correlated basket (log-Euler), Cholesky factor in kernel args (uniform).
// Sobol dimension of (step t, asset a) = a * n_fine + t  (column 0 unused, Q8).
// ---------------------------------------------------------------------------
template <int NA, bool ALIGNED>
__global__ __launch_bounds__(256) void k_sim_basket(const SimDesc d) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (!ALIGNED && p >= d.n_local) return;
  const uint32_t g = gray_code((uint64_t)sim_gidx(d, p));
  const float dt = (float)d.dt, sdt = sqrtf(dt);
  float ly[NA], drift[NA], vol[NA], inv[NA], ch[NA * (NA + 1) / 2];
  const size_t n = (size_t)d.n_local;
#pragma unroll
  for (int a = 0, i = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b <= a; ++b, ++i) ch[i] = (float)d.chol[a * MAXIN + b];  // hoisted fp64 -> fp32
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    ly[a] = logf((float)d.s0[a]);
    drift[a] = (float)((d.mu[a] - 0.5 * d.sigma[a] * d.sigma[a]) * d.dt);
    vol[a] = (float)d.sigma[a] * sdt;
    inv[a] = (float)d.inv_norm[a];
    d.out[(size_t)a * n + p] = (float)d.s0[a] * inv[a];
  }
  for (int t = 1; t < d.n_fine; ++t) {
    float w[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const int dim = a * d.n_fine + t;
      w[a] = ndtri_u30<float>(sobol_point<ALIGNED>(d.sv1 + (size_t)dim * 32, d.shift1[dim], g));
    }
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      float z = 0.f;
#pragma unroll
      for (int b = 0; b <= a; ++b) z = fmaf(ch[a * (a + 1) / 2 + b], w[b], z);
      ly[a] += drift[a] + vol[a] * z;
    }
    if (t % d.reduction == 0) {
      const int c = t / d.reduction;
      if (c < d.n_coarse) {
#pragma unroll
        for (int a = 0; a < NA; ++a) d.out[((size_t)c * NA + a) * n + p] = __expf(ly[a]) * inv[a];
      }
    }
  }
  if (d.final_out) {
#pragma unroll
    for (int a = 0; a < NA; ++a) d.final_out[(size_t)a * n + p] = __expf(ly[a]) * inv[a];
  }
}

// ---------------------------------------------------------------------------
// K7 payoffs (normalised units).
//   0 guarantee: max(Y_T, K) * N_T/N      (RP:88, :184)
//   1 call: max(S_T - K, 0)   2 put: max(K - S_T, 0)   (EO cell 8)
//   3 basket call: max(sum_a w_a S_a,T - K, 0)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_payoff(int kind, int n, int na, const float* __restrict__ s,
                                                const float* __restrict__ nfrac, float strike,
                                                const float* __restrict__ wts, float* __restrict__ out) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  float v;
  if (kind == 0) {
    const float y = s[p];
    v = (y > strike ? y : strike) * (nfrac ? nfrac[p] : 1.f);
  } else if (kind == 1) {
    v = fmaxf(s[p] - strike, 0.f);
  } else if (kind == 2) {
    v = fmaxf(strike - s[p], 0.f);
  } else {
    float b = 0.f;
    for (int a = 0; a < na; ++a) b = fmaf(wts[a], s[(size_t)a * n + p], b);
    v = fmaxf(b - strike, 0.f);
  }
  out[p] = v;
}

// ---------------------------------------------------------------------------
// K13 building block: radix-select histogram of monotone float keys.
// key(x) = x>=0 ? bits|0x80000000 : ~bits.  Counts keys whose (key & pmask) ==
// prefix, binned by (key >> shift) & (nbins-1).  LDS histogram per workgroup,
// one global atomic per non-empty bin.
// ---------------------------------------------------------------------------
RPH_INLINE uint32_t fkey(float x) {
  const uint32_t b = __float_as_uint(x);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__global__ __launch_bounds__(256) void k_radix_hist(const float* __restrict__ x, long long n, uint32_t pmask,
                                                    uint32_t prefix, int shift, int nbins,
                                                    unsigned int* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) unsigned int h[];
  for (int i = threadIdx.x; i < nbins; i += 256) h[i] = 0u;
  __syncthreads();
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const uint32_t k = fkey(x[i]);
    if ((k & pmask) == prefix) atomicAdd(&h[(k >> shift) & (uint32_t)(nbins - 1)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nbins; i += 256)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

}  // namespace rph

using namespace rph;

static inline int grid_for(int n) { return (n + 255) / 256; }

extern "C" int rph_sobol_normal(void* out, int n, int d, const uint32_t* sv, const uint32_t* shift,
                                long long offset, int fp64, int raw, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const bool aligned = (n % 256 == 0) && (offset % 64 == 0);
  if (fp64) {
    if (aligned) hipLaunchKernelGGL((k_sobol_normal<double, true>), dim3(grid_for(n)), dim3(256), 0, s, (double*)out, n, d, sv, shift, offset, raw);
    else hipLaunchKernelGGL((k_sobol_normal<double, false>), dim3(grid_for(n)), dim3(256), 0, s, (double*)out, n, d, sv, shift, offset, raw);
  } else {
    if (aligned) hipLaunchKernelGGL((k_sobol_normal<float, true>), dim3(grid_for(n)), dim3(256), 0, s, (float*)out, n, d, sv, shift, offset, raw);
    else hipLaunchKernelGGL((k_sobol_normal<float, false>), dim3(grid_for(n)), dim3(256), 0, s, (float*)out, n, d, sv, shift, offset, raw);
  }
  return (int)hipGetLastError();
}

template <typename Real, bool AL>
static int launch_scan(const SimDesc* d, hipStream_t s) {
  const dim3 grid(grid_for(d->n_local)), block(256);
  switch (d->model) {
    case SIM_GBM_ARITH: hipLaunchKernelGGL((k_sim_scan<Real, AL, SIM_GBM_ARITH>), grid, block, 0, s, *d); break;
    case SIM_GBM_LOG: hipLaunchKernelGGL((k_sim_scan<Real, AL, SIM_GBM_LOG>), grid, block, 0, s, *d); break;
    case SIM_SV_REF: hipLaunchKernelGGL((k_sim_scan<Real, AL, SIM_SV_REF>), grid, block, 0, s, *d); break;
    case SIM_HESTON: hipLaunchKernelGGL((k_sim_scan<Real, AL, SIM_HESTON>), grid, block, 0, s, *d); break;
    case SIM_MORTALITY: hipLaunchKernelGGL((k_sim_scan<Real, AL, SIM_MORTALITY>), grid, block, 0, s, *d); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

template <bool AL>
static int launch_basket(const SimDesc* d, hipStream_t s) {
  const dim3 grid(grid_for(d->n_local)), block(256);
  switch (d->na) {
    case 1: hipLaunchKernelGGL((k_sim_basket<1, AL>), grid, block, 0, s, *d); break;
    case 2: hipLaunchKernelGGL((k_sim_basket<2, AL>), grid, block, 0, s, *d); break;
    case 3: hipLaunchKernelGGL((k_sim_basket<3, AL>), grid, block, 0, s, *d); break;
    case 4: hipLaunchKernelGGL((k_sim_basket<4, AL>), grid, block, 0, s, *d); break;
    case 5: hipLaunchKernelGGL((k_sim_basket<5, AL>), grid, block, 0, s, *d); break;
    case 6: hipLaunchKernelGGL((k_sim_basket<6, AL>), grid, block, 0, s, *d); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int rph_simulate(const SimDesc* d, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (d->map_blk < 0 || (d->map_blk > 0 && d->map_stride < d->map_blk)) return rph_report("rph_simulate", "bad path-index map");
  // (aligned: every wave's 64 paths are one aligned range of global indices)
  const bool aligned = (d->n_local % 256 == 0) && (d->path_offset % 64 == 0) &&
                       (d->map_blk == 0 || (d->map_blk % 64 == 0 && d->map_stride % 64 == 0));
  if (d->model == SIM_BASKET) return aligned ? launch_basket<true>(d, s) : launch_basket<false>(d, s);
  if (d->fp64) return aligned ? launch_scan<double, true>(d, s) : launch_scan<double, false>(d, s);
  return aligned ? launch_scan<float, true>(d, s) : launch_scan<float, false>(d, s);
}

extern "C" int rph_payoff(int kind, int n, int na, const float* s, const float* nfrac, float strike,
                          const float* wts, float* out, void* stream) {
  hipLaunchKernelGGL(k_payoff, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, kind, n, na, s, nfrac,
                     strike, wts, out);
  return (int)hipGetLastError();
}

extern "C" int rph_radix_hist(const float* x, long long n, uint32_t pmask, uint32_t prefix, int shift,
                              int nbins, unsigned int* hist, void* stream) {
  long long blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_radix_hist, dim3((unsigned)blocks), dim3(256), nbins * sizeof(unsigned int),
                     (hipStream_t)stream, x, n, pmask, prefix, shift, nbins, hist);
  return (int)hipGetLastError();
}
