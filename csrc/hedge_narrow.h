// rphedge — NarrowBody: the thread-per-path fp32 forward/backward + in-wave
// reduce-scatter body of the reference's 8-unit hedge nets (K8/K9), shared by
// the step schedules (hedge_mlp.hip, hedge_fit.h, hedge_lag.h) and the
// Levenberg-Marquardt pass kernel (hedge_lm.hip).
#pragma once
#include "hedge_core.h"

namespace rph {

// ---------------------------------------------------------------------------
// Per-workgroup gradient packet of one minibatch step, thread-per-path VALU
// (the reference's 8-unit nets).  Used by the per-step kernel below and by the
// persistent per-fit kernel (hedge_fit.h).
// ---------------------------------------------------------------------------
template <int NIN, int H, int NO, int HEAD, int WPE = 1, int PFD = 1, bool LDSW = (WPE > 1), bool HYB = false>
struct NarrowBody {
  static constexpr int WAVES_PER_SIMD = WPE;
  static constexpr int NIN_ = NIN, H_ = H, NO_ = NO, HEAD_ = HEAD;
  // LDSW: weights are re-read from LDS every path iteration instead of being
  // hoisted into registers (needed at 2 waves/SIMD; at 1 wave/SIMD it keeps
  // the wide-packet nets - basket 5-8-6, R = 256 - out of scratch spills)
  static constexpr bool LDS_WEIGHTS = LDSW;
  // path-data prefetch distance in loop iterations (1: the next path is loaded
  // while the current one computes; >1 keeps PFD loads in flight, so a thread's
  // later paths never wait on a fresh L2/MALL round trip)
  static constexpr int PF = PFD;
  using S = NetShape<NIN, H, NO, HEAD>;
  static constexpr int P = S::P;
  static constexpr int R = S::R;
  static constexpr int NR = (R + 255) / 256;  // packet entries per thread (1)
  static constexpr int NREP = NARROW_NREP;    // lagged schedule: float-atomic replicas
  static constexpr bool ACC_PLAIN = true;      // lagged prologue: cached (L2-shared) accumulator loads
  static constexpr int NHOLD = S::NHOLD;
  static constexpr int SCRATCH_FLOATS = (4 * R > 1024 ? 4 * R : 1024) + 8;
  struct Frags {};  // (weights are read from LDS)
  struct Pre {      // first path of the step, loaded ahead by the caller
    float x[NIN], pr[NHOLD], y;
    bool valid;
  };

  RPH_INLINE static void make_frags(const float*, Frags&) {}

  RPH_INLINE static long long first(int wid) { return (long long)(blockIdx.x * 4 + wid) * 64; }

  RPH_INLINE static void load(const TrainDesc& d, int step, const Perm& perm, long long j0, int lane, Pre& p) {
    const long long jl = j0 + lane;
    const long long j = (long long)step * d.batch + jl;
    p.valid = (jl < d.batch) && (j < d.n_local);
    const uint32_t q = p.valid ? perm_path(perm, (uint32_t)j, d.chunk_log2, d.n_local) : 0u;
#pragma unroll
    for (int f = 0; f < NIN; ++f) p.x[f] = d.feat[f][q];  // raw, unselected (q = 0 when invalid; invalid paths carry dV = 0):
                                                   // no v_cndmask forcing an early vmcnt wait
#pragma unroll
    for (int k = 0; k < NHOLD - 1; ++k) p.pr[k] = d.price[k][q];
    p.pr[NHOLD - 1] = d.bond;
    p.y = d.target[q];
  }

  // W: weights in LDS; lds: SCRATCH_FLOATS of LDS; pre: the first path (loaded).
  // Returns in val[0] (threads < R) the workgroup sum of packet entry tid.
  RPH_INLINE static void partial(const TrainDesc& d, int step, const Perm& perm, const float* __restrict__ W,
                                 const Frags&, float* lds, Pre& pre, float (&val)[NR]) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const long long stride = (long long)gridDim.x * 4 * 64;
    float g[R];
#pragma unroll
    for (int i = 0; i < R; ++i) g[i] = 0.f;
    const float alpha = d.alpha;
    // ring of prefetched paths: q[0] = current (loaded by the caller), q[i] the
    // path i iterations ahead
    Pre q[PF];
    q[0] = pre;
#pragma unroll
    for (int i = 1; i < PF; ++i) {
      q[i].valid = false;
      if (first(wid) + i * stride < d.batch) load(d, step, perm, first(wid) + i * stride, lane, q[i]);
    }
    for (long long j0 = first(wid); j0 < d.batch; j0 += stride) {
      // WPE 1: the loop-invariant LDS weights are hoisted into registers (AGPR
      // overflow); WPE 2: an opaque zero offset makes every iteration re-read
      // them as LDS broadcasts, so the kernel fits 256 registers = 2 waves/SIMD
      // HYB: only the W2 block (the most-used weights, forward and backward)
      // is hoisted into registers, the rest is re-read from LDS, so the
      // hoisted weights fit in VGPRs instead of overflowing to AGPRs (each
      // AGPR-resident weight costs a v_accvgpr_read per use)
      const float* __restrict__ Wi = W;
      if constexpr (LDSW || HYB) {
        // opaque 16-byte-aligned base: every use is a ds_read_b128 broadcast
        // off ONE address register with an immediate offset
        uint32_t z = 0;
        asm volatile("" : "+v"(z));
        Wi = (const float*)__builtin_assume_aligned(W + (z & ~3u), 16);
      }
      const float* __restrict__ W2s = HYB ? W : Wi;
      float x[NIN], pr[NHOLD];
#pragma unroll
      for (int f = 0; f < NIN; ++f) x[f] = (q[0].x[f] - d.fmu[f]) * d.fisd[f];
#pragma unroll
      for (int k = 0; k < NHOLD; ++k) pr[k] = q[0].pr[k];
      const float y = q[0].y;
      const bool valid = q[0].valid;
#pragma unroll
      for (int i = 0; i + 1 < PF; ++i) q[i] = q[i + 1];
      if (j0 + PF * stride < d.batch) load(d, step, perm, j0 + PF * stride, lane, q[PF - 1]);  // software pipelining

      float z1[H], a1[H], z2[H], a2[H], hold[NHOLD];
      net_forward<NIN, H, NO, HEAD>(Wi, x, alpha, z1, a1, z2, a2, hold, W2s);
      float V = 0.f;
#pragma unroll
      for (int k = 0; k < NHOLD; ++k) V = fmaf(hold[k], pr[k], V);
      float l, dV;
      path_loss(d.loss, d.quantile, V, y, l, dV);  // dL/dV (mean over the global batch below)
      dV = valid ? dV * d.inv_batch : 0.f;
      const float ae = fabsf(V - y);
      g[P + 0] += valid ? l : 0.f;
      g[P + 1] += valid ? ae : 0.f;
      g[P + 2] += valid ? ae * __frcp_rn(fmaxf(fabsf(y), 1e-7f)) : 0.f;
      g[P + 3] += valid ? 1.f : 0.f;

      // backward
      float dout[NO];
      if (HEAD == HEAD_COMPLEMENT) {
        dout[0] = dV * (pr[0] - pr[1]);
      } else {
#pragma unroll
        for (int k = 0; k < NO; ++k) dout[k] = dV * pr[k];
      }
#pragma unroll
      for (int k = 0; k < NO; ++k) g[S::OB3 + k] += dout[k];
      float dz2[H];
#pragma unroll
      for (int j = 0; j < H; ++j) {
        float da = 0.f;
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          g[S::OW3 + j * NO + k] = fmaf(a2[j], dout[k], g[S::OW3 + j * NO + k]);
          da = fmaf(Wi[S::OW3 + j * NO + k], dout[k], da);
        }
        dz2[j] = da * lrelu_d(a2[j], alpha);  // (a > 0 <=> z > 0 for 0 <= alpha: z1/z2 need not stay live)
        g[S::OB2 + j] += dz2[j];
      }
#pragma unroll
      for (int i = 0; i < H; ++i) {
        float da = 0.f;
#pragma unroll
        for (int j = 0; j < H; ++j) {
          g[S::OW2 + i * H + j] = fmaf(a1[i], dz2[j], g[S::OW2 + i * H + j]);
          da = fmaf(W2s[S::OW2 + i * H + j], dz2[j], da);
        }
        const float dz1 = da * lrelu_d(a1[i], alpha);
        g[S::OB1 + i] += dz1;
#pragma unroll
        for (int f = 0; f < NIN; ++f) g[S::OW1 + f * H + i] = fmaf(x[f], dz1, g[S::OW1 + f * H + i]);
      }
    }
    RPH_STAMP(5);  // path loop done (Adam fits: every workgroup's own row)
    // ---- in-wave reduce-scatter, cross-wave LDS sum ------------------------
    wave_reduce_scatter<R>(g, lane);
    constexpr int PER = R / 64;
#pragma unroll
    for (int i = 0; i < PER; ++i) lds[wid * R + lane * PER + i] = g[i];
    __syncthreads();
    const int t = threadIdx.x;
    val[0] = (t < R) ? (lds[t] + lds[R + t]) + (lds[2 * R + t] + lds[3 * R + t]) : 0.f;
    __syncthreads();
  }
};

// ---------------------------------------------------------------------------
// Full-batch MSE pass body of the Levenberg-Marquardt fits (k_lm_pass): TWO
// paths per lane per iteration (lane l: paths j0 + l and j0 + 64 + l, both
// coalesced), carried as float2 so the forward and backward matrix-vector
// products issue as packed fp32 (v_pk_fma_f32: two paths per instruction)
// and every weight read from LDS serves both paths.  The per-lane gradient
// sums stay scalar (two fmas per entry and pair: a packed accumulator would
// double the 128 accumulator registers past the 2-waves-per-SIMD budget).
// Same packet layout and in-wave reduce-scatter as NarrowBody.
// ---------------------------------------------------------------------------
typedef float nb_f2 __attribute__((ext_vector_type(2)));

RPH_INLINE nb_f2 nb_s(float w) { return nb_f2{w, w}; }
RPH_INLINE nb_f2 nb_fma(nb_f2 a, nb_f2 b, nb_f2 c) { return __builtin_elementwise_fma(a, b, c); }
RPH_INLINE nb_f2 nb_lrelu(nb_f2 z, float alpha) { return __builtin_elementwise_max(z, z * alpha); }
// d(lrelu)/dz * da (a = lrelu(z): a > 0 <=> z > 0 for 0 <= alpha)
RPH_INLINE nb_f2 nb_lrelu_bwd(nb_f2 a, nb_f2 da, float alpha) {
  const nb_f2 t = da * alpha;
  return nb_f2{a.x > 0.f ? da.x : t.x, a.y > 0.f ? da.y : t.y};
}
// g += a.x * b.x + a.y * b.y (the pair's contribution to one gradient entry)
RPH_INLINE float nb_acc(float g, nb_f2 a, nb_f2 b) { return fmaf(a.x, b.x, fmaf(a.y, b.y, g)); }

typedef __bf16 nb_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 nb_bf16x4 __attribute__((ext_vector_type(4)));
typedef float nb_f32x16 __attribute__((ext_vector_type(16)));
typedef short nb_s16x4 __attribute__((ext_vector_type(4)));
typedef short nb_s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) nb_s16x4 nb_lds_s16x4;

// bf16 hi / lo image of a [row][unit] fp32 matrix in LDS for the matrix
// cores (rows = paths): hi = bf16(u), lo = bf16(u - hi), 16 significant bits;
// a row is [hi: NU units | lo: NU units] (+ padding in PITCH).  nb_img_put
// writes units [c0, c0 + 4) of a row; nb_img_frag reads the MFMA fragment of
// unit block ub (ub + NU / 32: its lo half), K-step s (16 rows): unit
// 32 ub + lane % 32 of the 8 rows 16 s + 8 (lane / 32) .. + 7, by two
// transposing reads (ds_read_b64_tr_b16).  G = sum_rows u u^T is then
// hi hi^T + hi lo^T + lo hi^T on v_mfma_f32_32x32x16_bf16.
template <int PITCH, int NU>
RPH_INLINE void nb_img_put(unsigned char* img, int row, int c0, float u0, float u1, float u2, float u3) {
  const __bf16 h0 = (__bf16)u0, h1 = (__bf16)u1, h2 = (__bf16)u2, h3 = (__bf16)u3;
  const nb_bf16x4 h = {h0, h1, h2, h3};
  const nb_bf16x4 l = {(__bf16)(u0 - (float)h0), (__bf16)(u1 - (float)h1), (__bf16)(u2 - (float)h2),
                       (__bf16)(u3 - (float)h3)};
  *(nb_bf16x4*)(img + row * PITCH + 2 * c0) = h;
  *(nb_bf16x4*)(img + row * PITCH + 2 * (NU + c0)) = l;
}
template <int PITCH>
RPH_INLINE nb_bf16x8 nb_img_frag(const unsigned char* img, int s, int ub, int lane) {
  const int grp = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int c0 = 32 * ub + 16 * (grp & 1), hh = grp >> 1;
  const int off = (16 * s + 8 * hh + q) * PITCH + (c0 + 4 * p) * 2;
  const nb_s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((nb_lds_s16x4*)(img + off));
  const nb_s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((nb_lds_s16x4*)(img + off + 4 * PITCH));
  // whole-vector bit cast: inserting the elements one by one as
  // bit_cast<__bf16>(r[e]) was miscompiled into splats of r[0]
  return __builtin_bit_cast(nb_bf16x8, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int NIN, int H, int NO, int HEAD, bool OG = false>
struct NarrowPairBody {
  // pass workgroups per CU: two for the 1- and 2-input free-head nets without
  // the output Gram (their body fits 256 VGPRs and 46 KB of LDS, so two waves
  // share each SIMD and fill each other's dependency stalls), else one (the
  // output-Gram body needs 80 KB of LDS; aliased onto the Gram tile's image
  // and capped at 256 VGPRs (4 spills) it gained 0.4 % and the bench P&L went
  // wrong, cause not isolated: reverted, BENCHMARKS.md round 6)
  static constexpr int WAVES_PER_SIMD = (!OG && NIN <= 2 && HEAD == HEAD_FREE && NO <= 2) ? 2 : 1;
  static constexpr int NIN_ = NIN, H_ = H, NO_ = NO, HEAD_ = HEAD;
  using S = NetShape<NIN, H, NO, HEAD>;
  static constexpr int P = S::P;
  static constexpr int R = S::R;
  static constexpr int NR = (R + 255) / 256;
  static constexpr int NHOLD = S::NHOLD;
  static constexpr int SCRATCH_FLOATS = (4 * R > 1024 ? 4 * R : 1024) + 8;
  static_assert(R <= 256, "one packet entry per thread");
  // Full-batch output-layer Gram matrix (OG: the last passes of an lm_out_fix
  // fit): the value is linear in the output layer's NU parameters, u_p =
  // dV/dtheta_o = [a2_j c_k (j, k), c_k] with c = the held prices (complement
  // head: c_0 = S - B), and sum_p u_p u_p^T is a GEMM over the paths.  Per
  // 64-path half of an iteration every lane writes its path's u as a row of a
  // [path][unit] LDS image, split u = hi + lo into two bf16 halves (hi =
  // bf16(u), lo = bf16(u - hi): 16 significant bits), the operands (unit r of
  // 8 consecutive paths) come back with the transposing read
  // ds_read_b64_tr_b16, and v_mfma_f32_32x32x16_bf16 accumulates hi hi^T +
  // hi lo^T + lo hi^T of the 32 x 32 block(s) in fp32 - 24 (NU <= 32) or 72
  // (NU <= 64) matrix-core ops per 128 paths, issued beside the VALU body.
  // bf16 alone is not enough: the output Gram of a fitted net has condition
  // numbers of 1e9 and beyond (collinear hidden units), and 2^-8 rounding of u
  // moved the Newton step by 100x its length (tools/og_precision.py); the
  // split matches the fp64 step to 1e-5 of its loss reduction.
  static constexpr int NU = HEAD == HEAD_FREE ? H * NO + NO : H + 1;
  static constexpr int NUP = NU <= 32 ? 32 : 64;
  static constexpr int NBO = NUP == 32 ? 1 : 3;  // upper-triangular 32 x 32 blocks
  static constexpr int OG_PITCH = 4 * NUP + 8;   // bytes per image row: [hi | lo] (+8: write-conflict padding)
  static constexpr int OG_ROWS = 64;             // one path per lane per half-iteration
  static constexpr int OG_LDS = 4 * OG_ROWS * OG_PITCH;
  static constexpr bool OGM = OG && NU <= 64;
  static_assert(!OG || NU <= 64, "output-layer Gram: at most 64 output parameters");
  static_assert(4 * NBO * 1024 * 4 <= OG_LDS, "the waves' output-Gram tiles reuse the image LDS");
  struct Frags {};
  struct Pre {
    nb_f2 x[NIN], pr[NHOLD], y;
    nb_f2 m;  // 1: a path of the shard, 0: past its end
  };

  RPH_INLINE static void make_frags(const float*, Frags&) {}
  RPH_INLINE static long long first(int wid) { return (long long)(blockIdx.x * 4 + wid) * 128; }

  // the 128-path blocks of this wave: b0, b0 + bstep, ... < bend.  The waves
  // of the first gram_wgs workgroups (which also build a Gram tile after the
  // paths) take gram_skip blocks fewer than an even split; the others share
  // the rest (gram_skip = 0: every wave cyclic over all blocks)
  struct Sched {
    long long b0, bstep, bend;
  };
  // (num_wgs: the path workgroups; a pass grid may carry Gram-only workgroups beyond them)
  RPH_INLINE static Sched sched(const TrainDesc& d, int num_wgs, int gram_wgs, int gram_skip, int leaf_blocks = 0) {
    const long long nblk = (d.batch + 127) / 128;
    const int TW = num_wgs * 4, w = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    if (leaf_blocks > 0) {  // contiguous leaves (LmDesc.leaf_blocks)
      const long long b0 = (long long)w * leaf_blocks, b1 = b0 + leaf_blocks;
      return {b0, 1, b1 < nblk ? b1 : nblk};
    }
    const int GW = (gram_wgs < num_wgs ? gram_wgs : num_wgs) * 4;
    const long long per = nblk / TW;
    if (gram_skip <= 0 || GW >= TW || per <= 0) return {w, TW, nblk};
    const long long gb = per > gram_skip ? per - gram_skip : 0;
    if (w < GW) return {w, GW, GW * gb};
    return {GW * gb + (w - GW), TW - GW, nblk};
  }

  RPH_INLINE static void load(const TrainDesc& d, int, const Perm&, long long j0, int lane, Pre& p) {
    const long long ja = j0 + lane, jb = ja + 64;
    const bool va = ja < d.batch, vb = jb < d.batch;
    const long long qa = va ? ja : 0, qb = vb ? jb : 0;
#pragma unroll
    for (int f = 0; f < NIN; ++f) p.x[f] = nb_f2{d.feat[f][qa], d.feat[f][qb]};
#pragma unroll
    for (int k = 0; k < NHOLD - 1; ++k) p.pr[k] = nb_f2{d.price[k][qa], d.price[k][qb]};
    p.pr[NHOLD - 1] = nb_s(d.bond);
    p.y = nb_f2{d.target[qa], d.target[qb]};
    p.m = nb_f2{va ? 1.f : 0.f, vb ? 1.f : 0.f};
  }

  // wave-level LDS ordering around the image (all lanes of the wave active)
  RPH_INLINE static void og_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // this lane's unit slice [c0, c0 + 4) of row `row` of the image (nb_img_put)
  RPH_INLINE static void og_put(unsigned char* img, int row, int c0, float u0, float u1, float u2, float u3) {
    nb_img_put<OG_PITCH, NUP>(img, row, c0, u0, u1, u2, u3);
  }
  RPH_INLINE static nb_bf16x8 og_frag(const unsigned char* img, int s, int ub, int lane) {
    return nb_img_frag<OG_PITCH>(img, s, ub, lane);
  }

  // one 128-path iteration of the output-layer Gram: u of both paths
  // (masked) -> the [path][unit] image (bf16 hi / lo halves, 64 rows per
  // half-iteration) -> hi hi^T + hi lo^T + lo hi^T on the matrix cores
  RPH_INLINE static void og_accum(unsigned char* img, nb_f32x16 (&oacc)[NBO], const nb_f2 (&a2)[H],
                                  const nb_f2 (&pr)[NHOLD], const nb_f2 m, const int lane) {
    nb_f2 c[NO];
    if (HEAD == HEAD_COMPLEMENT) {
      c[0] = (pr[0] - pr[1]) * m;
    } else {
#pragma unroll
      for (int k = 0; k < NO; ++k) c[k] = pr[k] * m;
    }
    float ua[(NU + 3) / 4 * 4], ub[(NU + 3) / 4 * 4];
#pragma unroll
    for (int j = 0; j < H; ++j)
#pragma unroll
      for (int k = 0; k < NO; ++k) {
        const nb_f2 v = a2[j] * c[k];
        ua[j * NO + k] = v.x;
        ub[j * NO + k] = v.y;
      }
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      ua[H * NO + k] = c[k].x;
      ub[H * NO + k] = c[k].y;
    }
#pragma unroll
    for (int e = NU; e < (NU + 3) / 4 * 4; ++e) ua[e] = ub[e] = 0.f;
    constexpr int LO = NUP / 32;  // unit block of the lo half
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      og_wave_sync();  // the previous half's fragment reads are done
#pragma unroll
      for (int c0 = 0; c0 < NU; c0 += 4) {
        if (h2) og_put(img, lane, c0, ub[c0], ub[c0 + 1], ub[c0 + 2], ub[c0 + 3]);
        else og_put(img, lane, c0, ua[c0], ua[c0 + 1], ua[c0 + 2], ua[c0 + 3]);
      }
      og_wave_sync();
#pragma unroll
      for (int s2 = 0; s2 < OG_ROWS / 16; ++s2) {
        const nb_bf16x8 h0 = og_frag(img, s2, 0, lane), l0 = og_frag(img, s2, LO, lane);
        oacc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(h0, h0, oacc[0], 0, 0, 0);
        oacc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(h0, l0, oacc[0], 0, 0, 0);
        oacc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(l0, h0, oacc[0], 0, 0, 0);
        if constexpr (NBO == 3) {
          const nb_bf16x8 h1 = og_frag(img, s2, 1, lane), l1 = og_frag(img, s2, LO + 1, lane);
          oacc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(h0, h1, oacc[1], 0, 0, 0);
          oacc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(h0, l1, oacc[1], 0, 0, 0);
          oacc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(l0, h1, oacc[1], 0, 0, 0);
          oacc[2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(h1, h1, oacc[2], 0, 0, 0);
          oacc[2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(h1, l1, oacc[2], 0, 0, 0);
          oacc[2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(l1, h1, oacc[2], 0, 0, 0);
        }
      }
    }
  }

  // og_lds: OG_LDS bytes of LDS (the OG instantiation), og_out: this
  // workgroup's NBO x 1024 output-Gram floats (MFMA register layout)
  RPH_INLINE static void partial(const TrainDesc& d, int step, const Perm& perm, const float* __restrict__ W,
                                 const Frags&, float* lds, Pre& pre, float (&val)[NR], const Sched& sc,
                                 const bool og = false, unsigned char* og_lds = nullptr,
                                 float* __restrict__ og_out = nullptr) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const long long stride = sc.bstep * 128;
    const long long jend = sc.bend * 128 < d.batch ? sc.bend * 128 : d.batch;
    // PKG (an even output count, so every parameter group has an even size
    // and offset): the gradient sums as PAIRS of adjacent parameters, updated
    // by packed fmas whose operands are the per-path values regrouped by
    // parameter (one 2 x 2 transpose per pair of units) and the other
    // factor's per-path value broadcast - instead of two scalar fmas per
    // entry, which the compiler packed with a v_mov gather per operand.  Same
    // operations per entry in the same order (bitwise the scalar form).
    // With the backward's own weight reads (below) the path loop issues 555
    // VALU instructions per iteration instead of 682 (171 -> 92 v_mov, no
    // AGPR traffic); the pass takes 20.8 / 28.5 µs instead of 21.0 / 29.8
    // (plain / output-Gram; profiles/r5/pkg_ab/) - the loop is latency-bound
    // at one wave per SIMD, not issue-bound.
    constexpr bool PKG = HEAD == HEAD_FREE && NO % 2 == 0 && P % 2 == 0;
    float g[R];
    nb_f2 gv[PKG ? R / 2 : 1];
#pragma unroll
    for (int i = 0; i < R; ++i) g[i] = 0.f;
#pragma unroll
    for (int i = 0; i < (PKG ? R / 2 : 1); ++i) gv[i] = nb_s(0.f);
    const float alpha = d.alpha;
    const float two_inv = 2.f * d.inv_batch;
    const bool pinball = d.loss == LOSS_PINBALL;
    const float q = d.quantile;
    Pre cur = pre;
    nb_f32x16 oacc[NBO];
    unsigned char* const img = og_lds + wid * OG_ROWS * OG_PITCH;
    if constexpr (OGM) {
#pragma unroll
      for (int b = 0; b < NBO; ++b) oacc[b] = nb_f32x16{};
      if (og) {
        // the image's padding units [NU4, NUP) stay zero (written once)
        constexpr int NU4 = (NU + 3) / 4 * 4;
#pragma unroll
        for (int c0 = NU4; c0 < NUP; c0 += 4) og_put(img, lane, c0, 0.f, 0.f, 0.f, 0.f);
      }
    }
    for (long long j0 = sc.b0 * 128; j0 < jend; j0 += stride) {
      // opaque 16-byte-aligned weight base: every weight use is an LDS
      // broadcast read off one address register (register budget)
      uint32_t z = 0;
      asm volatile("" : "+v"(z));
      const float* __restrict__ Wi = (const float*)__builtin_assume_aligned(W + (z & ~3u), 16);
      nb_f2 x[NIN], pr[NHOLD];
#pragma unroll
      for (int f = 0; f < NIN; ++f) x[f] = (cur.x[f] - d.fmu[f]) * d.fisd[f];
#pragma unroll
      for (int k = 0; k < NHOLD; ++k) pr[k] = cur.pr[k];
      const nb_f2 y = cur.y, m = cur.m;
      if (j0 + stride < jend) load(d, step, perm, j0 + stride, lane, cur);  // the next pair, in flight

      // forward
      nb_f2 a1[H], a2[H], o[NO];
#pragma unroll
      for (int j = 0; j < H; ++j) {
        nb_f2 acc = nb_s(Wi[S::OB1 + j]);
#pragma unroll
        for (int f = 0; f < NIN; ++f) acc = nb_fma(x[f], nb_s(Wi[S::OW1 + f * H + j]), acc);
        a1[j] = nb_lrelu(acc, alpha);
      }
      // layer 2 with the row index outer: H independent accumulator chains
      // (a dependent v_pk_fma_f32 pair costs a hazard wait state and the
      // result latency; one wave per SIMD has nothing to fill them with)
#pragma unroll
      for (int j = 0; j < H; ++j) a2[j] = nb_s(Wi[S::OB2 + j]);
#pragma unroll
      for (int i = 0; i < H; ++i)
#pragma unroll
        for (int j = 0; j < H; ++j) a2[j] = nb_fma(a1[i], nb_s(Wi[S::OW2 + i * H + j]), a2[j]);
#pragma unroll
      for (int j = 0; j < H; ++j) a2[j] = nb_lrelu(a2[j], alpha);
      // output layer: NO x 2 chains (even / odd hidden units)
#pragma unroll
      for (int k = 0; k < NO; ++k) {
        nb_f2 acc0 = nb_s(Wi[S::OB3 + k]), acc1 = nb_s(0.f);
#pragma unroll
        for (int j = 0; j < H; j += 2) {
          acc0 = nb_fma(a2[j], nb_s(Wi[S::OW3 + j * NO + k]), acc0);
          acc1 = nb_fma(a2[j + 1], nb_s(Wi[S::OW3 + (j + 1) * NO + k]), acc1);
        }
        o[k] = acc0 + acc1;
      }
      nb_f2 V;
      if (HEAD == HEAD_COMPLEMENT) {  // psi = 1 - phi
        V = nb_fma(o[0], pr[0] - pr[1], pr[1]);
      } else {
        V = o[0] * pr[0];
#pragma unroll
        for (int k = 1; k < NO; ++k) V = nb_fma(o[k], pr[k], V);
      }
      // MSE loss statistics and dL/dV (mean over the global batch)
      const nb_f2 e = V - y;
      // per-path loss and dL/dV: MSE, or the reference's pinball loss
      // (Replicating_Portfolio.py:138-145; uniform branch on the descriptor)
      nb_f2 le, dV;
      if (pinball) {
        float lx, ly, gx, gy;
        path_loss(LOSS_PINBALL, q, V.x, y.x, lx, gx);
        path_loss(LOSS_PINBALL, q, V.y, y.y, ly, gy);
        le = nb_f2{lx, ly} * m;
        dV = nb_f2{gx, gy} * m * d.inv_batch;
      } else {
        le = e * e * m;
        dV = e * m * two_inv;
      }
      const nb_f2 ae = nb_f2{fabsf(e.x), fabsf(e.y)} * m;
      const nb_f2 ape = ae * nb_f2{__builtin_amdgcn_rcpf(fmaxf(fabsf(y.x), 1e-7f)),
                                   __builtin_amdgcn_rcpf(fmaxf(fabsf(y.y), 1e-7f))};
      if constexpr (PKG) {
        gv[P / 2].x += le.x + le.y;
        gv[P / 2].y += ae.x + ae.y;
        gv[P / 2 + 1].x += ape.x + ape.y;
        gv[P / 2 + 1].y += m.x + m.y;
      } else {
        g[P + 0] += le.x + le.y;
        g[P + 1] += ae.x + ae.y;
        g[P + 2] += ape.x + ape.y;
        g[P + 3] += m.x + m.y;
      }
      if constexpr (OGM) {
        if (og) og_accum(img, oacc, a2, pr, m, lane);
      }

      // backward
      nb_f2 dout[NO];
      if (HEAD == HEAD_COMPLEMENT) {
        dout[0] = dV * (pr[0] - pr[1]);
      } else {
#pragma unroll
        for (int k = 0; k < NO; ++k) dout[k] = dV * pr[k];
      }
      if constexpr (PKG) {
        // the backward's weight reads from their own opaque base: not CSEd
        // with the forward's, each broadcast has one use (an op_sel operand)
        uint32_t zb = 0;
        asm volatile("" : "+v"(zb));
        const float* __restrict__ Wb = (const float*)__builtin_assume_aligned(W + (zb & ~3u), 16);
        auto tx = [](nb_f2 a, nb_f2 b) { return nb_f2{a.x, b.x}; };
        auto ty = [](nb_f2 a, nb_f2 b) { return nb_f2{a.y, b.y}; };
        auto bx = [](nb_f2 a) { return nb_f2{a.x, a.x}; };
        auto by = [](nb_f2 a) { return nb_f2{a.y, a.y}; };
        // g += a.x b.x + a.y b.y per entry: fma(a.x, b.x, fma(a.y, b.y, g))
        auto acc2 = [&](int e, nb_f2 a, nb_f2 bxp, nb_f2 byp) {
          gv[e / 2] = nb_fma(bx(a), bxp, nb_fma(by(a), byp, gv[e / 2]));
        };
#pragma unroll
        for (int k = 0; k < NO; k += 2) {
          const nb_f2 dx = tx(dout[k], dout[k + 1]), dy = ty(dout[k], dout[k + 1]);
          gv[(S::OB3 + k) / 2] += dx + dy;
#pragma unroll
          for (int j = 0; j < H; ++j) acc2(S::OW3 + j * NO + k, a2[j], dx, dy);
        }
        nb_f2 dz2[H];
#pragma unroll
        for (int j = 0; j < H; ++j) {
          nb_f2 da = nb_s(0.f);
#pragma unroll
          for (int k = 0; k < NO; ++k) da = nb_fma(nb_s(Wb[S::OW3 + j * NO + k]), dout[k], da);
          dz2[j] = nb_lrelu_bwd(a2[j], da, alpha);
        }
        // layer-2 backward: per unit i two chains (even / odd j), all 2 H
        // chains interleaved (j outer) - the same sums as the serial form
        nb_f2 da0[H], da1[H];
#pragma unroll
        for (int i = 0; i < H; ++i) da0[i] = da1[i] = nb_s(0.f);
#pragma unroll
        for (int j = 0; j < H; ++j)
#pragma unroll
          for (int i = 0; i < H; ++i) {
            if (j & 1) da1[i] = nb_fma(nb_s(Wb[S::OW2 + i * H + j]), dz2[j], da1[i]);
            else da0[i] = nb_fma(nb_s(Wb[S::OW2 + i * H + j]), dz2[j], da0[i]);
          }
#pragma unroll
        for (int j = 0; j < H; j += 2) {
          const nb_f2 zx = tx(dz2[j], dz2[j + 1]), zy = ty(dz2[j], dz2[j + 1]);
          gv[(S::OB2 + j) / 2] += zx + zy;
#pragma unroll
          for (int i = 0; i < H; ++i) acc2(S::OW2 + i * H + j, a1[i], zx, zy);
        }
        nb_f2 dz1[H];
#pragma unroll
        for (int i = 0; i < H; ++i) dz1[i] = nb_lrelu_bwd(a1[i], da0[i] + da1[i], alpha);
#pragma unroll
        for (int i = 0; i < H; i += 2) {
          const nb_f2 zx = tx(dz1[i], dz1[i + 1]), zy = ty(dz1[i], dz1[i + 1]);
          gv[(S::OB1 + i) / 2] += zx + zy;
#pragma unroll
          for (int f = 0; f < NIN; ++f) acc2(S::OW1 + f * H + i, x[f], zx, zy);
        }
      } else {
#pragma unroll
      for (int k = 0; k < NO; ++k) g[S::OB3 + k] += dout[k].x + dout[k].y;
      nb_f2 dz2[H];
#pragma unroll
      for (int j = 0; j < H; ++j) {
        nb_f2 da = nb_s(0.f);
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          g[S::OW3 + j * NO + k] = nb_acc(g[S::OW3 + j * NO + k], a2[j], dout[k]);
          da = nb_fma(nb_s(Wi[S::OW3 + j * NO + k]), dout[k], da);
        }
        dz2[j] = nb_lrelu_bwd(a2[j], da, alpha);
        g[S::OB2 + j] += dz2[j].x + dz2[j].y;
      }
#pragma unroll
      for (int i = 0; i < H; ++i) {
        nb_f2 da0 = nb_s(0.f), da1 = nb_s(0.f);  // two chains (even / odd j)
#pragma unroll
        for (int j = 0; j < H; ++j) {
          g[S::OW2 + i * H + j] = nb_acc(g[S::OW2 + i * H + j], a1[i], dz2[j]);
          if (j & 1) da1 = nb_fma(nb_s(Wi[S::OW2 + i * H + j]), dz2[j], da1);
          else da0 = nb_fma(nb_s(Wi[S::OW2 + i * H + j]), dz2[j], da0);
        }
        const nb_f2 dz1 = nb_lrelu_bwd(a1[i], da0 + da1, alpha);
        g[S::OB1 + i] += dz1.x + dz1.y;
#pragma unroll
        for (int f = 0; f < NIN; ++f) g[S::OW1 + f * H + i] = nb_acc(g[S::OW1 + f * H + i], x[f], dz1);
      }
      }  // (PKG)
    }
    if constexpr (PKG) {
#pragma unroll
      for (int i = 0; i < R / 2; ++i) {
        g[2 * i] = gv[i].x;
        g[2 * i + 1] = gv[i].y;
      }
    }
    RPH_STAMP_BODY(5);  // path loop done
    wave_reduce_scatter<R>(g, lane);
    constexpr int PER = R / 64;
#pragma unroll
    for (int i = 0; i < PER; ++i) lds[wid * R + lane * PER + i] = g[i];
    if constexpr (OGM) {
      if (og) {
        // the four waves' output-Gram tiles -> one workgroup tile (fixed order)
        float* ot = reinterpret_cast<float*>(og_lds);
        __syncthreads();  // every wave's last fragment reads are done
#pragma unroll
        for (int b = 0; b < NBO; ++b)
#pragma unroll
          for (int q = 0; q < 16; ++q) ot[(wid * NBO + b) * 1024 + q * 64 + lane] = oacc[b][q];
      }
    }
    __syncthreads();
    const int t = threadIdx.x;
    val[0] = (t < R) ? (lds[t] + lds[R + t]) + (lds[2 * R + t] + lds[3 * R + t]) : 0.f;
    if constexpr (OGM) {
      if (og) {
        const float* ot = reinterpret_cast<const float*>(og_lds);
        for (int e = t; e < NBO * 1024; e += 256)
          og_out[e] = (ot[e] + ot[NBO * 1024 + e]) + (ot[2 * NBO * 1024 + e] + ot[3 * NBO * 1024 + e]);
      }
    }
    __syncthreads();
  }
};

}  // namespace rph
