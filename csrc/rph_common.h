// rphedge — shared device utilities for the MI355X (gfx950 / CDNA4) kernels.
//
// Everything here is written for 64-wide wavefronts.  Reference parity notes
// cite /root/reference files (read-only) as file:line.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RPH_WAVE 64
#define RPH_INLINE __device__ __forceinline__

// Device-side invariant checks, compiled in only for `python -m rphedge.build
// --debug` (-DRPH_DEBUG=1).  A failed check prints and ends the kernel (no
// trap: a GPU fault would reset the device); use at kernel scope only.
#if defined(RPH_DEBUG) && RPH_DEBUG
#define RPH_DASSERT(cond)                                                                          \
  do {                                                                                             \
    if (!(cond)) {                                                                                 \
      if (threadIdx.x == 0) printf("RPH_DASSERT %s:%d block %d: %s\n", __FILE__, __LINE__, (int)blockIdx.x, #cond); \
      return;                                                                                      \
    }                                                                                              \
  } while (0)
#else
#define RPH_DASSERT(cond) do { } while (0)
#endif

namespace rph {

// diagnostic clock (s_memrealtime, 100 MHz) read where the program puts it:
// a volatile asm keeps its place among the other side-effecting instructions
// (the builtin may be scheduled freely, which let phase stamps of the solve
// land out of program order), and the wait makes the value ready at once
RPH_INLINE unsigned long long rph_stamp_clock() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}

// Pull the kernel-argument segment (the by-value launch descriptor, up to 10
// 64-byte lines) into the scalar cache with every miss in flight at once.
// Without it the compiler's own kernarg loads form a chain of 4-6 dependent
// scalar round trips (loads issued where each field is first needed, with
// s_waitcnt between), which every workgroup pays at kernel start (~1 us of
// an 11 us training step).  Scalar LOADS only (the scalar cache is never
// written).  All ten loads target ONE scratch SGPR (the values are never
// read), so the register allocator has no reason to make the compiler's own
// early kernarg loads wait first; the token keeps that SGPR reserved until
// prefetch_kernarg_end, whose s_waitcnt (or any earlier compiler lgkmcnt(0)
// wait) retires the loads.
template <int BYTES>
RPH_INLINE uint32_t prefetch_kernarg_begin() {
  static_assert(BYTES >= 4 && BYTES <= 640, "kernarg prefetch covers 1..10 lines");
#define RPH_KO(i) ((i) * 64 < BYTES ? (i) * 64 : ((BYTES - 4) & ~3))
  auto kp = __builtin_amdgcn_kernarg_segment_ptr();
  uint32_t t;
  asm volatile(
      "s_load_dword %0, %1, %2\n\t"
      "s_load_dword %0, %1, %3\n\t"
      "s_load_dword %0, %1, %4\n\t"
      "s_load_dword %0, %1, %5\n\t"
      "s_load_dword %0, %1, %6\n\t"
      "s_load_dword %0, %1, %7\n\t"
      "s_load_dword %0, %1, %8\n\t"
      "s_load_dword %0, %1, %9\n\t"
      "s_load_dword %0, %1, %10\n\t"
      "s_load_dword %0, %1, %11"
      : "=&s"(t)
      : "s"(kp), "i"(RPH_KO(0)), "i"(RPH_KO(1)), "i"(RPH_KO(2)), "i"(RPH_KO(3)), "i"(RPH_KO(4)),
        "i"(RPH_KO(5)), "i"(RPH_KO(6)), "i"(RPH_KO(7)), "i"(RPH_KO(8)), "i"(RPH_KO(9)));
#undef RPH_KO
  return t;
}

RPH_INLINE void prefetch_kernarg_end(uint32_t t) { asm volatile("s_waitcnt lgkmcnt(0)" : : "s"(t)); }

template <int BYTES>
RPH_INLINE void prefetch_kernarg() { prefetch_kernarg_end(prefetch_kernarg_begin<BYTES>()); }

// ---------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG (Salmon et al. 2011).  Used for binomial
// survivor draws (reference uses numpy MT19937 reseeded per step,
// Replicating_Portfolio.py:81-84 — not reproducible in parallel, so parity is
// statistical), minibatch chunk permutations and weight initialisation.
// A host/numpy twin lives in rphedge/ops/philox.py and is tested bit-exact.
// ---------------------------------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

RPH_INLINE __host__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)M0 * c.x;
    const uint64_t p1 = (uint64_t)M1 * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    u32x4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// (0,1) uniforms
RPH_INLINE float u01f(uint32_t x) { return ((x >> 8) + 0.5f) * (1.0f / 16777216.0f); }
RPH_INLINE double u01d(uint32_t hi, uint32_t lo) {
  const uint64_t m = ((uint64_t)hi << 21) ^ (uint64_t)(lo >> 11);  // 53 bits
  return ((double)(m & ((1ull << 53) - 1)) + 0.5) * (1.0 / 9007199254740992.0);
}

// ---------------------------------------------------------------------------
// Inverse normal CDF (K2).  Input is the raw 30-bit Sobol integer x (u = x/2^30),
// which lets us form u, 1-u and 2u-1 without cancellation.
//   fp32: Giles' single-precision erfinv (w = -log(4u(1-u)) formulation).
//   fp64: Acklam rational approximation + one Halley step on erfc (≈1e-15 rel),
//         parity mode vs scipy.stats.norm.ppf (Replicating_Portfolio.py:57).
// ---------------------------------------------------------------------------
RPH_INLINE float ndtri_u30_f32(uint32_t x) {
  const float s = 9.313225746154785e-10f;  // 2^-30
  const float a = (float)x * s;
  const float b = (float)(1073741824u - x) * s;
  const float y = (float)((int32_t)(x << 1) - (int32_t)1073741824) * s;  // 2u-1, exact int diff
  float w = -__logf(4.0f * a * b);
  float p;
  if (w < 5.0f) {
    w = w - 2.5f;
    p = 2.81022636e-08f;
    p = fmaf(p, w, 3.43273939e-07f);
    p = fmaf(p, w, -3.5233877e-06f);
    p = fmaf(p, w, -4.39150654e-06f);
    p = fmaf(p, w, 0.00021858087f);
    p = fmaf(p, w, -0.00125372503f);
    p = fmaf(p, w, -0.00417768164f);
    p = fmaf(p, w, 0.246640727f);
    p = fmaf(p, w, 1.50140941f);
  } else {
    w = sqrtf(w) - 3.0f;
    p = -0.000200214257f;
    p = fmaf(p, w, 0.000100950558f);
    p = fmaf(p, w, 0.00134934322f);
    p = fmaf(p, w, -0.00367342844f);
    p = fmaf(p, w, 0.00573950773f);
    p = fmaf(p, w, -0.0076224613f);
    p = fmaf(p, w, 0.00943887047f);
    p = fmaf(p, w, 1.00167406f);
    p = fmaf(p, w, 2.83297682f);
  }
  return 1.41421356237309505f * p * y;
}

RPH_INLINE double ndtri_acklam_f64(double p, double q /* = 1-p, exact */) {
  const double a1 = -3.969683028665376e+01, a2 = 2.209460984245205e+02, a3 = -2.759285104469687e+02,
               a4 = 1.383577518672690e+02, a5 = -3.066479806614716e+01, a6 = 2.506628277459239e+00;
  const double b1 = -5.447609879822406e+01, b2 = 1.615858368580409e+02, b3 = -1.556989798598866e+02,
               b4 = 6.680131188771972e+01, b5 = -1.328068155288572e+01;
  const double c1 = -7.784894002430293e-03, c2 = -3.223964580411365e-01, c3 = -2.400758277161838e+00,
               c4 = -2.549732539343734e+00, c5 = 4.374664141464968e+00, c6 = 2.938163982698783e+00;
  const double d1 = 7.784695709041462e-03, d2 = 3.224671290700398e-01, d3 = 2.445134137142996e+00,
               d4 = 3.754408661907416e+00;
  const double plow = 0.02425;
  double z;
  if (p < plow) {
    const double t = sqrt(-2.0 * log(p));
    z = (((((c1 * t + c2) * t + c3) * t + c4) * t + c5) * t + c6) / ((((d1 * t + d2) * t + d3) * t + d4) * t + 1.0);
  } else if (q < plow) {
    const double t = sqrt(-2.0 * log(q));
    z = -(((((c1 * t + c2) * t + c3) * t + c4) * t + c5) * t + c6) / ((((d1 * t + d2) * t + d3) * t + d4) * t + 1.0);
  } else {
    const double r0 = p - 0.5, r = r0 * r0;
    z = (((((a1 * r + a2) * r + a3) * r + a4) * r + a5) * r + a6) * r0 /
        (((((b1 * r + b2) * r + b3) * r + b4) * r + b5) * r + 1.0);
  }
  // One Halley refinement step against Phi(z) = erfc(-z/sqrt2)/2.  Work on the
  // smaller tail so the residual has full relative precision.
  const double inv_sqrt2 = 0.70710678118654752440;
  double e;
  if (p < 0.5) e = 0.5 * erfc(-z * inv_sqrt2) - p;
  else e = q - 0.5 * erfc(z * inv_sqrt2);
  const double u = e * 2.50662827463100050242 * exp(0.5 * z * z);
  z = z - u / (1.0 + 0.5 * z * u);
  return z;
}

RPH_INLINE double ndtri_u30_f64(uint32_t x) {
  if (x == 0u) return -INFINITY;  // scipy: norm.ppf(0) = -inf
  const double s = 9.313225746154785e-10;
  return ndtri_acklam_f64((double)x * s, (double)(1073741824u - x) * s);
}

// ---------------------------------------------------------------------------
// Scrambled Sobol point (K1), index-addressable.  scipy's random_base2 emits
// point i = shift ^ XOR_{k in bits(gray(i))} sv[k] (verified bit-exact for
// scipy 1.15; Replicating_Portfolio.py:55-56).  sv is stored [dim][32] u32.
// ALIGNED: all 64 lanes of the wave hold path indices of one 64-aligned block,
// so bits >= 6 of gray(i) are wave-uniform and are folded on the scalar unit.
// ---------------------------------------------------------------------------
template <bool ALIGNED>
RPH_INLINE uint32_t sobol_point(const uint32_t* __restrict__ sv_d, uint32_t shift_d, uint32_t gray) {
  uint32_t x = shift_d;
  if (ALIGNED) {
#pragma unroll
    for (int k = 0; k < 6; ++k) x ^= ((gray >> k) & 1u) ? sv_d[k] : 0u;
    uint32_t h = __builtin_amdgcn_readfirstlane(gray >> 6);
    while (h) {
      const int k = __builtin_ctz(h);
      x ^= sv_d[6 + k];
      h &= h - 1u;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 30; ++k) x ^= ((gray >> k) & 1u) ? sv_d[k] : 0u;
  }
  return x;
}

RPH_INLINE uint32_t gray_code(uint64_t i) { return (uint32_t)(i ^ (i >> 1)); }

// LeakyReLU (Keras-2 default alpha=0.3)
// For 0 <= alpha <= 1 (checked on the host, validate_train), max(z, alpha z)
// equals the select bit for bit and costs 2 VALU ops (mul + max, the mul packs)
// instead of 3 (cmp + mul + cndmask).
RPH_INLINE float lrelu(float z, float alpha) { return fmaxf(z, alpha * z); }
RPH_INLINE float lrelu_d(float z, float alpha) { return z > 0.f ? 1.f : alpha; }

// ---------------------------------------------------------------------------
// Cross-lane moves for in-wave reductions (gfx9 DPP / ds_swizzle / bpermute).
// Each returns the value of a partner lane whose lane-id differs in exactly the
// bit being reduced and agrees on all higher bits already reduced.
// ---------------------------------------------------------------------------
RPH_INLINE float xlane_bit5(float v) { return __shfl_xor(v, 32, 64); }
RPH_INLINE float xlane_bit4(float v) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401F));  // xor 16 in 32-groups
}
RPH_INLINE float xlane_bit3(float v) {  // row_mirror: lane i <-> 15-i within 16
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
}
RPH_INLINE float xlane_bit2(float v) {  // row_half_mirror: i <-> 7-i within 8
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
}
RPH_INLINE float xlane_bit1(float v) {  // quad_perm [2,3,0,1]
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
}
RPH_INLINE float xlane_bit0(float v) {  // quad_perm [1,0,3,2]
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}

// Recursive-halving ("reduce-scatter in a wave") of an R-vector held by every
// lane.  After the call lane L holds the wave-total of entries
// [L*(R/64), (L+1)*(R/64)) in v[0 .. R/64).  All indices are compile-time (no
// scratch).  Cross-lane moves, cheapest first on the largest arrays:
//   bit 5: v_permlane32_swap (a HALF exchange: lanes 32-63 of the first operand
//          swap with lanes 0-31 of the second) -> after swap(v[i], v[i+H])
//          every lane's two registers hold exactly its own and its partner's
//          share, so the step is ONE swap + ONE add per pair, no selects;
//   bit 4: ds_swizzle xor-16 butterfly;
//   bits 3..0: DPP (row_mirror / row_half_mirror / quad_perm) butterflies
//          whose adds fold the DPP move (v_add_f32_dpp).
template <int LEN>
RPH_INLINE void halve_bit5(float* v) {
  constexpr int H = LEN / 2;
#pragma unroll
  for (int i = 0; i < H; ++i) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]), __float_as_uint(v[i + H]), false, false);
    v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
}

template <int LEN, int BIT>
RPH_INLINE void halve_step(float* v, int lane) {
  constexpr int H = LEN / 2;
  const bool up = (lane >> BIT) & 1;
#pragma unroll
  for (int i = 0; i < H; ++i) {
    if (BIT == 4) {
      const float keep = up ? v[i + H] : v[i];
      const float send = up ? v[i] : v[i + H];
      v[i] = keep + xlane_bit4(send);
    } else {
      float lo, hi;
      if (BIT == 3) { lo = v[i] + xlane_bit3(v[i]); hi = v[i + H] + xlane_bit3(v[i + H]); }
      else if (BIT == 2) { lo = v[i] + xlane_bit2(v[i]); hi = v[i + H] + xlane_bit2(v[i + H]); }
      else if (BIT == 1) { lo = v[i] + xlane_bit1(v[i]); hi = v[i + H] + xlane_bit1(v[i + H]); }
      else { lo = v[i] + xlane_bit0(v[i]); hi = v[i + H] + xlane_bit0(v[i + H]); }
      v[i] = up ? hi : lo;
    }
  }
}

template <int R>
RPH_INLINE void wave_reduce_scatter(float* v, int lane) {
  static_assert(R >= 64 && (R & (R - 1)) == 0, "R must be a power of two >= 64");
  halve_bit5<R>(v);
  halve_step<R / 2, 4>(v, lane);
  halve_step<R / 4, 3>(v, lane);
  halve_step<R / 8, 2>(v, lane);
  halve_step<R / 16, 1>(v, lane);
  halve_step<R / 32, 0>(v, lane);
}

// Plain full-wave sum (for a handful of scalars).
RPH_INLINE float wave_sum(float v) {
  v += xlane_bit0(v);
  v += xlane_bit1(v);
  v += xlane_bit2(v);
  v += xlane_bit3(v);
  v += xlane_bit4(v);
  v += xlane_bit5(v);
  return v;
}
RPH_INLINE double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace rph
