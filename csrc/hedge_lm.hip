// rphedge — Levenberg-Marquardt (damped Gauss-Newton) fits of the reference's
// 8-unit hedge nets on gfx950: the MSE objective of one backward-induction
// date, mean over paths of (h(state_t) . prices_{t+1} - V_{t+1})^2
// (Replicating_Portfolio.py:211, the fit that Keras-Adam runs for 500 / 100
// epochs), solved by full-batch damped Gauss-Newton steps instead.
//
// One PASS evaluates one trial point theta:
//   k_lm_pass    every local path: loss, |e|, ape and the exact gradient
//                g = (2/n) sum_p e_p J_p on the VALU (NarrowBody, the same fused
//                fwd/bwd body as the Adam step kernels, full batch, no shuffle);
//                the Gram matrix of a 64-path tile per gram workgroup,
//                G += J^T J over the tile, on the matrix cores
//                (v_mfma_f32_32x32x2_f32, J staged through LDS, upper-
//                triangular 32x32 blocks spread over the 4 waves);
//                per-workgroup results go to slabs (no float atomics)
//   k_lm_reduce  fixed-order sums of the slabs -> one reduced block
//                [G | g | stats] (bitwise reproducible run to run)
//   (data parallel: one all-reduce of the reduced block between the two)
//   k_lm_solve   one workgroup: accept the trial if its loss beats the best
//                point (damping down) or reject it (damping up), then the
//                Marquardt step (2G + lam diag(2G) + ridge) d = -g by an fp64
//                Cholesky factorisation in LDS and the next trial
//                theta_best + d; the last pass writes theta_best to the
//                canonical NetWeights and the FitState bookkeeping.
// The start point is pass 0; `passes` trial points follow.  Everything stays
// on the device and graph-captures with the rest of the induction.
#include <utility>

#include "hedge_core.h"
#include "hedge_narrow.h"

namespace rph {

typedef float lm_f32x16 __attribute__((ext_vector_type(16)));

template <int P>
struct LmShape {
  static constexpr int NP = ((P + 31) / 32) * 32;  // padded to MFMA blocks
  static constexpr int NB = NP / 32;
  static constexpr int NBLK = NB * (NB + 1) / 2;    // upper-triangular 32x32 blocks
  static constexpr int JP = NP + 33;                // LDS pitch of the J tile (odd*32+1: conflict-free)
  static_assert(NP <= LM_NPMAX && NBLK * 1024 <= LM_GBLK_MAX, "network too large for the LM solver");
};

// compile-time unrolled loop: f(std::integral_constant<int, j>) for j in [0, N)
template <class F, int... J>
RPH_INLINE void lm_static_for(F&& f, std::integer_sequence<int, J...>) {
  (f(std::integral_constant<int, J>{}), ...);
}
template <int N, class F>
RPH_INLINE void lm_static_for(F&& f) {
  lm_static_for(f, std::make_integer_sequence<int, N>{});
}

}  // namespace rph
#include "lm_chol.h"
namespace rph {

// The solve's tile-store image of the Gram (strictly lower entries x2, at
// their tile-store offsets), written by k_lm_reduce beside the 32 x 32 blocks
// in the unused tail of the Gram region: the solve then stages it with
// contiguous loads of 56 KB instead of gathering from 80 KB of blocks
// (nets whose blocks and image fit the region, up to 48 tiles)
template <int P>
struct LmTPack {
  using TG = TileGrid<P>;
  static constexpr int OFF = LmShape<P>::NBLK * 1024;  // image offset in the reduced block
  static constexpr int LEN = TG::NTILE * 256;
  static constexpr bool ON = TG::NX > 0 && OFF + LEN <= LM_GBLK_MAX;
  static constexpr int COPY = ON ? LEN : 0;  // doubles the best-block copy adds
};

// upper-triangular block b -> (mb, nb), mb <= nb, row-major
RPH_INLINE void lm_blk(int b, int NB, int& mb, int& nb) {
  int m = 0;
  while (b >= NB - m) {
    b -= NB - m;
    ++m;
  }
  mb = m;
  nb = m + b;
}

// unit (row) of 32x32 accumulator register q in lane half h
RPH_INLINE constexpr int lm_row(int q, int h) { return (q & 3) + 8 * (q >> 2) + 4 * h; }

// ---------------------------------------------------------------------------
// Pass kernel.  B = NarrowBody<...> (full batch: batch = n_local, no shuffle).
// ---------------------------------------------------------------------------
template <class B>
__global__ __launch_bounds__(256, B::WAVES_PER_SIMD) void k_lm_pass(const TrainDesc d, const LmDesc lm, const int pass,
                                                                   const double* __restrict__ red_new) {
  constexpr int P = B::P;
  constexpr int R = B::R;
  constexpr int NR = B::NR;
  using S = typename B::S;
  using LS = LmShape<P>;
  constexpr int NP = LS::NP, NB = LS::NB, NBLK = LS::NBLK, JP = LS::JP;
  constexpr int NIN = B::NIN_, H = B::H_, NO = B::NO_, HEAD = B::HEAD_, NHOLD = B::NHOLD;
  const uint32_t kat = prefetch_kernarg_begin<(sizeof(TrainDesc) + sizeof(LmDesc) + 16 < 640 ? sizeof(TrainDesc) + sizeof(LmDesc) + 16 : 640)>();
  __shared__ __attribute__((aligned(16))) float scratch[B::SCRATCH_FLOATS];
  __shared__ __attribute__((aligned(16))) float wl[P + 4];
  __shared__ __attribute__((aligned(16))) float jt[LM_TILE * JP];
  // the output-Gram image of the OG instantiation (the last passes of an lm_out_fix fit)
  __shared__ __attribute__((aligned(16))) unsigned char og_img[B::OGM ? B::OG_LDS : 16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  prefetch_kernarg_end(kat);
  // diagnostic phase stamps of every workgroup but 0 and 1 (tools/stamp_lm.py;
  // rows 0 and 1 belong to k_lm_solve)
  const bool stamp_wg = blockIdx.x >= 2 && blockIdx.y == 0;
#define RPH_STAMPP(k)                 \
  do {                                \
    if (stamp_wg) RPH_STAMP(k);       \
  } while (0)
  RPH_STAMPP(0);
  // instance (multi-start exploration: grid y) -> its state, slabs, reduced block
  const int inst = blockIdx.y;
  double* st = lm.state + (size_t)inst * LMS_FLOATS;
  red_new += (size_t)inst * LM_RED;
  float* const slab_b = lm.slab_b + (size_t)inst * lm.num_wgs * R;
  float* const slab_g = lm.slab_g + (size_t)inst * lm.gram_wgs * NBLK * 1024;
  double* sl = st + LMS_SLOTS + LM_SLOT * (pass & 1);  // this pass's scalars (written by the last solve)
  // trial point: pass 0 = the start point (canonical weights, published as
  // slot 0); later passes = the slot k_lm_solve wrote
  const int trial = pass == 0 ? 0 : 1 - (int)sl[LSS_BEST];
  const Perm perm = make_perm(1u, 0u, 0u, false);
  // workgroups [num_wgs, grid) only add a Gram tile (a Gram subsample larger
  // than 64 x the path grid: the subsample is the same at every world size)
  const bool path_wg = (int)blockIdx.x < lm.num_wgs;
  typename B::Pre pre;
  // (the output-Gram instantiation does not fit twice on a CU: its Gram tiles
  // stay in the path workgroups)
  const int gram_base = B::OGM ? 0 : lm.gram_base;
  // the final evaluation builds no Gram tile: its solve only accepts / rejects
  // and takes the output-layer (or bias) Newton step, which read g, the
  // statistics and the output Gram - so its path schedule is the even one
  const bool fin = pass == lm.passes;
  const typename B::Sched sc =
      B::sched(d, lm.num_wgs, (gram_base > 0 || fin) ? 0 : lm.gram_wgs, lm.gram_skip, lm.leaf_blocks);
  if (path_wg) B::load(d, 0, perm, sc.b0 * 128, lane, pre);
  for (int i = tid; i < P; i += 256) {
    float w;
    if (pass == 0) {
      const float* w0p = lm.w0 != nullptr ? lm.w0 + inst * LM_NPMAX : d.wts->w[0];
      w = w0p[i];
      if (lm.renorm) {
        // x_old = x_new (isd_old / isd_new) + (mu_new - mu_old) isd_old: W1 rescaled,
        // b1 absorbs the shift (fp64, rounded once)
        if (i >= S::OW1 && i < S::OW1 + NIN * H) {
          const int f = (i - S::OW1) / H;
          w = (float)((double)w * ((double)lm.ren_isd[f] / (double)d.fisd[f]));
        } else if (i >= S::OB1 && i < S::OB1 + H) {
          double acc = (double)w;
#pragma unroll
          for (int f = 0; f < NIN; ++f)
            acc += (double)w0p[S::OW1 + f * H + (i - S::OB1)] * (double)lm.ren_isd[f] *
                   ((double)d.fmu[f] - (double)lm.ren_mu[f]);
          w = (float)acc;
        }
      }
    } else {
      w = (float)st[LMS_W + trial * LM_NPMAX + i];
    }
    wl[i] = w;
    if (pass == 0 && blockIdx.x == 0) st[LMS_W + i] = (double)w;
  }
  if (pass > 0 && sl[LSS_COPY] != 0.0) {
    // the previous solve accepted its trial: best block := that trial's
    // reduced block (G, g, stats), spread over the grid; red_new is rewritten
    // only by this pass's reduce kernel, which runs after this one
    constexpr int NG = LmShape<P>::NBLK * 1024 + LmTPack<P>::COPY;  // blocks (+ the tile-store image)
    // g | stats | output Gram (its entry 0 is -1 when the trial's pass did not build it)
    constexpr int NGR = LM_RED_OUTG - LM_GBLK_MAX + (B::NU <= LM_OG_MAX ? B::NU * (B::NU + 1) / 2 : 1);
    double* best_red = st + LMS_RED;
    for (int e = blockIdx.x * 256 + tid; e < NG + NGR; e += (int)gridDim.x * 256) {
      const int o = e < NG ? e : LM_GBLK_MAX + e - NG;
      best_red[o] = red_new[o];
    }
  }
  if (pass > 0 && sl[LSS_STOP] != 0.0) return;  // adaptive budget spent: nothing to evaluate
  // fused data-parallel exchange: this pass's reduce pushes and sums under the
  // next sequence number (every rank evaluates the same passes)
  if (lm.dp_fused && blockIdx.x == 0 && tid == 0)
    __hip_atomic_fetch_add(lm.dp.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (pass == 0 && blockIdx.x == 0 && tid == 0) {
    sl[LSS_BEST] = 1.0;
    // (state[LMS_LAM] = the previous fit's final damping on this state)
    sl[LSS_LAM] = lm.lam_carry > 0.f ? fmax(st[LMS_LAM] * (double)lm.lam_carry, (double)lm.lam_min) : (double)lm.lam0;
    sl[LSS_NU] = 2.0;
    sl[LSS_PRED] = 0.0;
    sl[LSS_COPY] = 0.0;
    sl[LSS_SPEC_IDX] = (double)LM_SPEC;
    sl[LSS_LBEST] = INFINITY;
    sl[LSS_STOP] = 0.0;
    st[LMS_NACC] = 0.0;
    st[LMS_FAIL] = 0.0;
  }
  if (pass == 0 && blockIdx.x == 0 && inst == 0 && !lm.weights_only && !lm.explore) {
    // the loss history: passes an adaptive budget skips stay NaN
    for (int k = tid; k < MAXHIST; k += 256) d.fit->hist[k] = __builtin_nanf("");
  }
  __syncthreads();
  RPH_STAMPP(1);
  // ---- loss + exact gradient over every local path (VALU) -------------------
  if (path_wg) {
    typename B::Frags fr;
    B::make_frags(wl + S::OW2, fr);
    float val[NR];
    B::partial(d, 0, perm, wl, fr, scratch, pre, val, sc, lm.out_gram != 0, og_img,
               lm.slab_o + ((size_t)inst * lm.num_wgs + blockIdx.x) * 3 * 1024);
#pragma unroll
    for (int j = 0; j < NR; ++j)
      if (tid + 256 * j < R) slab_b[(size_t)blockIdx.x * R + tid + 256 * j] = val[j];
  }
  RPH_STAMPP(2);
  const int gtile = (int)blockIdx.x - gram_base;  // this workgroup's Gram tile
  if (fin || gtile < 0 || gtile >= lm.gram_wgs) return;
  // ---- Gram tile of 64 subsample paths (matrix cores) ------------------------
  if (wid == 0) {
    const long long slot = (long long)gtile * LM_TILE + lane;
    float x[NIN], pr[NHOLD];
    bool ok;
    if (lm.gram_side) {
      // the global subsample, simulated on this rank (slot order): every rank
      // builds the same Gram matrix
      ok = true;
#pragma unroll
      for (int f = 0; f < NIN; ++f) x[f] = (lm.gfeat[f][slot] - d.fmu[f]) * d.fisd[f];
#pragma unroll
      for (int k = 0; k < NHOLD - 1; ++k) pr[k] = lm.gprice[k][slot];
    } else {
      const long long p = (slot / lm.gram_blk) * lm.gram_blk_stride + slot % lm.gram_blk;
      ok = p < d.n_local;
      const long long q = ok ? p : 0;
#pragma unroll
      for (int f = 0; f < NIN; ++f) x[f] = (d.feat[f][q] - d.fmu[f]) * d.fisd[f];
#pragma unroll
      for (int k = 0; k < NHOLD - 1; ++k) pr[k] = d.price[k][q];
    }
    pr[NHOLD - 1] = d.bond;
    float z1[H], a1[H], z2[H], a2[H], hold[NHOLD];
    net_forward<NIN, H, NO, HEAD>(wl, x, d.alpha, z1, a1, z2, a2, hold);
    // pinball fits (IRLS Gauss-Newton): the Gram is the curvature of the
    // pinball loss's quadratic majoriser at this point, mean_p w_p J_p J_p^T / 2
    // with w_p = 1 / (2 max(|r_p|, delta)) (r = V - y), i.e. the row scaled by
    // 1 / (2 sqrt(max(|r_p|, delta))); delta = max(q_delta, q_kappa x the mean
    // |r| of this 64-path tile) keeps the weights of the small residuals
    // bounded (a near-zero residual would otherwise dominate the step).  The
    // targets: the shard's (shard subsample) or the simulated subsample's own
    // (gram_side: LmDesc.gtarget, the same on every rank)
    float wq = 1.f;
    if (d.loss == LOSS_PINBALL) {
      const long long p = (slot / lm.gram_blk) * lm.gram_blk_stride + slot % lm.gram_blk;
      float V = 0.f;
#pragma unroll
      for (int k = 0; k < NHOLD; ++k) V = fmaf(hold[k], pr[k], V);
      const float y = lm.gram_side ? lm.gtarget[slot] : d.target[ok ? p : 0];
      const float ra = ok ? fabsf(V - y) : 0.f;
      float sa = ra, sc = ok ? 1.f : 0.f;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        sa += __shfl_xor(sa, o, 64);
        sc += __shfl_xor(sc, o, 64);
      }
      const float dl = fmaxf(lm.q_delta, lm.q_kappa * sa / fmaxf(sc, 1.f));
      wq = 0.5f * __builtin_amdgcn_rsqf(fmaxf(ra, dl));
    }
    // J_p = dV_p / dtheta  (dV = 1)
    float dout[NO];
    if (HEAD == HEAD_COMPLEMENT) {
      dout[0] = pr[0] - pr[1];
    } else {
#pragma unroll
      for (int k = 0; k < NO; ++k) dout[k] = pr[k];
    }
    float* row = jt + lane * JP;
    const float m = ok ? wq : 0.f;  // paths beyond the shard contribute nothing
#pragma unroll
    for (int k = 0; k < NO; ++k) row[S::OB3 + k] = m * dout[k];
    float dz2[H];
#pragma unroll
    for (int j = 0; j < H; ++j) {
      float da = 0.f;
#pragma unroll
      for (int k = 0; k < NO; ++k) {
        row[S::OW3 + j * NO + k] = m * a2[j] * dout[k];
        da = fmaf(wl[S::OW3 + j * NO + k], dout[k], da);
      }
      dz2[j] = m * da * lrelu_d(a2[j], d.alpha);
      row[S::OB2 + j] = dz2[j];
    }
#pragma unroll
    for (int i = 0; i < H; ++i) {
      float da = 0.f;
#pragma unroll
      for (int j = 0; j < H; ++j) {
        row[S::OW2 + i * H + j] = a1[i] * dz2[j];
        da = fmaf(wl[S::OW2 + i * H + j], dz2[j], da);
      }
      const float dz1 = da * lrelu_d(a1[i], d.alpha);
      row[S::OB1 + i] = dz1;
#pragma unroll
      for (int f = 0; f < NIN; ++f) row[S::OW1 + f * H + i] = x[f] * dz1;
    }
#pragma unroll
    for (int i = P; i < NP; ++i) row[i] = 0.f;
  }
  __syncthreads();
  RPH_STAMPP(3);
  const int h = lane >> 5, r = lane & 31;
  for (int b = wid; b < NBLK; b += 4) {
    int mb, nb;
    lm_blk(b, NB, mb, nb);
    lm_f32x16 acc = {};
#pragma unroll 8
    for (int s = 0; s < LM_TILE / 2; ++s) {
      const float* row = jt + (2 * s + h) * JP;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(row[mb * 32 + r], row[nb * 32 + r], acc, 0, 0, 0);
    }
    float* out = slab_g + ((size_t)gtile * NBLK + b) * 1024;
#pragma unroll
    for (int q = 0; q < 16; ++q) out[q * 64 + lane] = acc[q];
  }
  RPH_STAMPP(4);
#undef RPH_STAMPP
}

// ---------------------------------------------------------------------------
// Fused data-parallel exchange (LmDesc.dp_fused), called by wave 0 of a
// k_lm_reduce workgroup: lane l < n holds this rank's value v of gradient-
// region entry e (offset from LM_GBLK_MAX).  Push to every peer's mailbox row
// (slot, me) with system-scope stores, raise flag fi (system-scope release),
// wait for every peer's flag fi of the same sequence number (bounded acquire
// spin -> dp.error), return the fixed rank-order sum (every rank gets the
// bitwise-identical value).  The sequence number is the exchange counter the
// pass kernel advanced (graph replays never see stale flags).
// ---------------------------------------------------------------------------
RPH_INLINE double lm_dp_sum_wave(const LmDpDesc& x, const unsigned seq, const int fi, const double v, const int e,
                                 const bool act) {
  const int W = x.world, me = x.rank, lane = threadIdx.x & 63;
  const int slot = (int)(seq % DP_SLOTS);
  if (act)
    for (int q = 0; q < W; ++q)
      if (q != me)
        __hip_atomic_store(x.mbox[q] + ((size_t)slot * W + me) * x.pitch + e, v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  if (lane < W && lane != me) {
    unsigned* fo = reinterpret_cast<unsigned*>(x.mbox[lane] + ((size_t)slot * W + me) * x.pitch + LM_RED + fi);
    __hip_atomic_store(fo, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);  // (after the wave's pushes)
    const unsigned* fin =
        reinterpret_cast<const unsigned*>(x.mbox[me] + ((size_t)slot * W + lane) * x.pitch + LM_RED + fi);
    unsigned it = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(fin, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
      __builtin_amdgcn_s_sleep(1);
      if ((++it & 255u) == 0u && (__builtin_amdgcn_s_memrealtime() - t0 > DP_SPIN_TICKS ||
                                  __hip_atomic_load(x.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)) {
        __hip_atomic_store(x.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // every lane: the peers' rows after their flags
  // rank order, adjacent pairs first: ((r0 + r1) + (r2 + r3)) + ... - the top
  // of the reduce's contiguous-halves tree over the leaves
  double a[8];
#pragma unroll
  for (int q = 0; q < 8; ++q)
    a[q] = (q >= W || (x.fault == 1 && q == W - 1)) ? 0.0  // (fault: the probe tests' wrong sum)
           : q == me ? v
                     : (act ? __hip_atomic_load(x.mbox[me] + ((size_t)slot * W + q) * x.pitch + e,
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                            : 0.0);
#pragma unroll
  for (int st = 1; st < 8; st <<= 1)
#pragma unroll
    for (int q = 0; q < 8; q += 2 * st) a[q] += a[q + st];
  return a[0];
}

// ---------------------------------------------------------------------------
// Reduce kernel: red[e] = fixed-order sums of the slabs.
// ---------------------------------------------------------------------------
// workgroups of the output-Gram part of k_lm_reduce (64 packed entries each)
// (16 packed entries per workgroup - every thread loads 4 rows, one round
// trip - unless that needs more than 32 workgroups: then 64 entries x 16 rows)
constexpr int lm_og_epw(int NU) { return NU * (NU + 1) / 2 <= 512 ? 16 : 64; }
constexpr int lm_og_wgs(int NU) { return NU <= LM_OG_MAX ? (NU * (NU + 1) / 2 + lm_og_epw(NU) - 1) / lm_og_epw(NU) : 0; }

// Gram slabs up to this many (the multi-start exploration's 16-workgroup
// instances): k_lm_reduce sums each Gram entry in ONE thread (1,024 entries
// per workgroup) instead of 16 threads + an LDS combine - the same adds in
// the same order, 16 x fewer workgroups (16 instances: 720 instead of 3,120)
constexpr int LM_TPE_MAX = 16;
__host__ __device__ constexpr int lm_gram_red_wgs(int ng, int gram_wgs) { return gram_wgs <= LM_TPE_MAX ? ng / 1024 : ng / 64; }
// the gradient packet likewise, for <= 16 packet rows (no fused exchange):
// one workgroup, thread = entry, the rows' contiguous-halves tree in registers;
// <= 32 rows (the exploration's instances at two workgroups per CU): 32
// entries per workgroup
constexpr int LM_PK_C_MAX = 32;
__host__ __device__ constexpr int lm_pk_red_wgs(int R, int num_wgs, int dp_fused) {
  return dp_fused ? R / 4 : num_wgs <= LM_TPE_MAX ? 1 : num_wgs <= LM_PK_C_MAX ? R / 32 : R / 4;
}


template <int P, int R, int NU>
__global__ __launch_bounds__(1024) void k_lm_reduce(const LmDesc lm, double* __restrict__ red, const int pass,
                                                 const int wg0) {
  using LS = LmShape<P>;
  constexpr int NG = LS::NBLK * 1024;
  __shared__ double part[1024];
  const int inst = blockIdx.y;  // multi-start instance
  if (pass > 0 && lm.state[(size_t)inst * LMS_FLOATS + LMS_SLOTS + LM_SLOT * (pass & 1) + LSS_STOP] != 0.0) return;
  // fused data-parallel exchange: the sequence number the pass kernel advanced
  const unsigned seq = lm.dp_fused ? __hip_atomic_load(lm.dp.counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  red += (size_t)inst * LM_RED;
  const float* const slab_g = lm.slab_g + (size_t)inst * lm.gram_wgs * NG;
  const float* const slab_b = lm.slab_b + (size_t)inst * lm.num_wgs * R;
  const int tid = threadIdx.x;
  // (wg0: the final evaluation's launch starts past the Gram workgroups)
  const int bx = (int)blockIdx.x + wg0;
  const int NGW = lm_gram_red_wgs(NG, lm.gram_wgs);       // Gram workgroups
  const int NPW = lm_pk_red_wgs(R, lm.num_wgs, lm.dp_fused);  // packet workgroups
  if (bx >= NGW + NPW) {
    // full-batch output-layer Gram (packed upper triangle, mean over every
    // path); a pass that did not build it marks entry 0 with -1
    const bool og_pass = lm.out_gram && pass > lm.passes - LM_OUTG_TAIL;
    const int ob = bx - (NGW + NPW);
    if (!og_pass) {
      if (ob == 0 && tid == 0) red[LM_RED_OUTG] = -1.0;
      return;
    }
    constexpr int NPK = NU * (NU + 1) / 2;
    constexpr int EPW = lm_og_epw(NU);
    auto slab_off = [&](const int e) {
      int off = 0;
      if (e < NPK) {
        int i = 0, r = e;  // e -> (i, j), row-major upper triangle
        while (r >= NU - i) {
          r -= NU - i;
          ++i;
        }
        const int j = i + r;
        const int b = (i >> 5) == 0 ? ((j >> 5) == 0 ? 0 : 1) : 2;
        const int ii = i & 31, jj = j & 31;
        off = b * 1024 + ((ii & 3) + 4 * (ii >> 3)) * 64 + ((ii >> 2) & 1) * 32 + jj;
      }
      return off;
    };
    if constexpr (EPW == 16) {
      // thread (wave w, k = lane / 16, le = lane % 16): entry 16 ob + le, rows
      // 16 w + 4 k + [0, 4); the 4 rows, then the k pairs (xor 16, 32), then
      // the 16 waves, each by an adjacent-pairs tree - the same perfect binary
      // tree over the (<= 256) rows as the 64-entry form below, bit for bit
      const int lane = tid & 63, w = tid >> 6, le = lane & 15, k = lane >> 4;
      const int e = ob * 16 + le;
      const float* const so = lm.slab_o + (size_t)inst * lm.num_wgs * 3 * 1024 + slab_off(e);
      double v;
      if (lm.num_wgs > 256) {
        // (<= 512 rows: rows 32 w + 8 k + [0, 8), the same tree one level deeper)
        double r[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int row = 32 * w + 8 * k + u;
          r[u] = (e < NPK && row < lm.num_wgs) ? (double)so[(size_t)row * 3 * 1024] : 0.0;
        }
        v = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
      } else {
        double r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int row = 16 * w + 4 * k + u;
          r[u] = (e < NPK && row < lm.num_wgs) ? (double)so[(size_t)row * 3 * 1024] : 0.0;
        }
        v = (r[0] + r[1]) + (r[2] + r[3]);
      }
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (k == 0) part[w * 16 + le] = v;
      __syncthreads();
      if (w == 0) {
        double c[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) c[q] = part[q * 16 + le];
#pragma unroll
        for (int st = 1; st < 16; st <<= 1)
#pragma unroll
          for (int q = 0; q < 16; q += 2 * st) c[q] += c[q + st];
        double t = c[0];
        const bool act = k == 0 && e < NPK;
        if (lm.dp_fused) t = lm_dp_sum_wave(lm.dp, seq, R / 4 + ob, t, LM_RED_OUTG - LM_GBLK_MAX + e, act);
        if (act) red[LM_RED_OUTG + e] = t * (double)lm.inv_n;
      }
      return;
    }
    const int l = tid & 63, g = tid >> 6;
    const int e = ob * 64 + l;
    int off = 0;
    if (e < NPK) {
      int i = 0, r = e;  // e -> (i, j), row-major upper triangle
      while (r >= NU - i) {
        r -= NU - i;
        ++i;
      }
      const int j = i + r;
      const int b = (i >> 5) == 0 ? ((j >> 5) == 0 ? 0 : 1) : 2;
      const int ii = i & 31, jj = j & 31;
      off = b * 1024 + ((ii & 3) + 4 * (ii >> 3)) * 64 + ((ii >> 2) & 1) * 32 + jj;
    }
    const float* const slab_o = lm.slab_o + (size_t)inst * lm.num_wgs * 3 * 1024 + off;
    // rows [16 g, 16 g + 16) by a pairwise tree, then the 16 groups by a
    // pairwise tree: a contiguous-halves tree over the (<= 256) rows (<= 512:
    // rows [32 g, 32 g + 32) in two halves, one level deeper)
    const int RPG = lm.num_wgs > 256 ? 32 : 16;
    double h[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      double r[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int w = RPG * g + 16 * hh + u;
        r[u] = (e < NPK && w < lm.num_wgs && (hh == 0 || RPG == 32)) ? (double)slab_o[(size_t)w * 3 * 1024] : 0.0;
      }
#pragma unroll
      for (int st = 1; st < 16; st <<= 1)
#pragma unroll
        for (int u = 0; u < 16; u += 2 * st) r[u] += r[u + st];
      h[hh] = r[0];
    }
    part[tid] = RPG == 32 ? h[0] + h[1] : h[0];
    __syncthreads();
    if (g == 0) {
      double v = 0.0;
      if (e < NPK) {
        double c[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) c[q] = part[q * 64 + l];
#pragma unroll
        for (int st = 1; st < 16; st <<= 1)
#pragma unroll
          for (int q = 0; q < 16; q += 2 * st) c[q] += c[q + st];
        v = c[0];
      }
      // the ranks' UNSCALED tree sums travel and the mean is taken after the
      // rank tree, as in the one-rank run (bitwise world-invariant for any n)
      if (lm.dp_fused)
        v = lm_dp_sum_wave(lm.dp, seq, R / 4 + ob, v, LM_RED_OUTG - LM_GBLK_MAX + e, e < NPK);
      if (e < NPK) red[LM_RED_OUTG + e] = v * (double)lm.inv_n;
    }
    return;
  }
  // this entry's place in the solve's tile store (strictly lower only)
  auto tpack = [&](const int e, const double v) {
    if constexpr (LmTPack<P>::ON) {
      using TG = TileGrid<P>;
      const int b = e >> 10, f = e & 1023;
      int mb = 0, rem = b;
      while (rem >= TG::NBG - mb) rem -= TG::NBG - mb++;
      const int q = f >> 6, h = (f >> 5) & 1;
      const int lo = 32 * mb + (q & 3) + 4 * h + 8 * (q >> 2), hi = 32 * (mb + rem) + (f & 31);
      if (lo < hi && hi < P) red[LmTPack<P>::OFF + TG::tidx(hi >> 4, lo >> 4) * 256 + tg_off(hi & 15, lo & 15)] = 2.0 * v;
    }
  };
  if (NGW == NG / 1024 && bx < NGW) {
    // <= 16 slabs: thread = entry, the 16 "group" partial sums (slab g or 0)
    // combined in the LDS form's order: even groups, odd groups, their sum
    const int e = bx * 1024 + tid;
    const float* col = slab_g + e;
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int q = 0; q < 16; q += 2) {
      const double p0 = q < lm.gram_wgs ? (0.0 + (double)col[(size_t)q * NG]) + 0.0 : 0.0 + 0.0;
      const double p1 = q + 1 < lm.gram_wgs ? (0.0 + (double)col[(size_t)(q + 1) * NG]) + 0.0 : 0.0 + 0.0;
      a += p0;
      b += p1;
    }
    const double v = (a + b) * (double)lm.inv_ns;
    red[e] = v;
    tpack(e, v);
    return;
  }
  if (bx < NGW) {
    // Gram: workgroup handles entries [64 b, 64 b + 64); thread (g, l) sums
    // the slabs g, g + 16, ... of entry 64 b + l (every load of a 64-slab
    // reduction in flight at once: 4 per thread), the 16 partial sums
    // combined in LDS in fixed order
    const int l = tid & 63, g = tid >> 6;
    const int e = bx * 64 + l;
    const float* col = slab_g + e;
    double s0 = 0.0, s1 = 0.0;
    int w = g;
    for (; w + 16 < lm.gram_wgs; w += 32) {
      s0 += (double)col[(size_t)w * NG];
      s1 += (double)col[(size_t)(w + 16) * NG];
    }
    if (w < lm.gram_wgs) s0 += (double)col[(size_t)w * NG];
    part[tid] = s0 + s1;
    __syncthreads();
    if (g == 0) {
      double a = 0.0, b = 0.0;
#pragma unroll
      for (int q = 0; q < 16; q += 2) {
        a += part[q * 64 + l];
        b += part[(q + 1) * 64 + l];
      }
      const double v = (a + b) * (double)lm.inv_ns;
      red[e] = v;
      tpack(e, v);
    }
    return;
  }
  // gradient packet: workgroup pw handles entries [4 pw, 4 pw + 4); thread
  // (grp, k) loads row bitrev8(grp) (<= 256 pass workgroups) of entry 4 pw + k,
  // and the LDS tree below combines grp with grp + st: rows 2m and 2m + 1
  // first - a contiguous-halves tree over the rows, so a rank's rows (a
  // contiguous run of leaves, LmDesc.leaf_blocks) form a complete subtree and
  // the sum over the ranks (lm_dp_sum_wave) finishes the same tree
  if (NPW == 1) {
    // <= 16 rows: thread = entry; the LDS tree below puts row r at position
    // bitrev8(r) = 16 bitrev4(r) and adds position p + st to p for st = 128 ..
    // 1 - on these rows a pairwise tree over bitrev4 positions, then +0.0 for
    // the all-zero rest (the same adds, so the same bits)
    const int i = tid;
    if (i < P + 4) {
      double a[16];
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        const int r = (int)(__builtin_bitreverse32((unsigned)p) >> 28);
        a[p] = r < lm.num_wgs ? (double)slab_b[(size_t)r * R + i] : 0.0;
      }
#pragma unroll
      for (int st = 8; st >= 1; st >>= 1)
#pragma unroll
        for (int p = 0; p < st; ++p) a[p] += a[p + st];
      const int e = i < P ? i : LM_NPMAX + i - P;
      red[LM_GBLK_MAX + e] = a[0] + 0.0;
    }
    return;
  }
  if (lm.num_wgs <= LM_PK_C_MAX && !lm.dp_fused) {
    // 32 entries x 32 row positions: position q holds row bitrev5(q), and the
    // LDS tree adds q + st to q for st = 16 .. 1 - the contiguous-halves tree
    const int pw = bx - NGW;
    const int k = tid & 31, q = tid >> 5;
    const int i = pw * 32 + k;
    const int row = (int)(__builtin_bitreverse32((unsigned)q) >> 27);
    part[tid] = row < lm.num_wgs ? (double)slab_b[(size_t)row * R + i] : 0.0;
    __syncthreads();
#pragma unroll
    for (int st = 16; st >= 1; st >>= 1) {
      if (q < st) part[tid] += part[tid + 32 * st];
      __syncthreads();
    }
    if (tid < 32 && i < P + 4) red[LM_GBLK_MAX + (i < P ? i : LM_NPMAX + i - P)] = part[tid];
    return;
  }
  const int pw = bx - NGW;
  const int k = tid & 3, grp = tid >> 2;
  const int i = pw * 4 + k;
  const int row = (int)(__builtin_bitreverse32((unsigned)grp) >> 24);
  if (lm.num_wgs > 256) {
    // (<= 512 rows: position grp holds rows bitrev9(grp) = 2 bitrev8(grp) and
    // bitrev9(grp + 256) = 2 bitrev8(grp) + 1 - the first level of the
    // contiguous-halves tree over 512 rows; the LDS tree below is the rest)
    const int r0 = 2 * row;
    const double a = r0 < lm.num_wgs ? (double)slab_b[(size_t)r0 * R + i] : 0.0;
    const double b = r0 + 1 < lm.num_wgs ? (double)slab_b[(size_t)(r0 + 1) * R + i] : 0.0;
    part[tid] = a + b;
  } else {
    part[tid] = row < lm.num_wgs ? (double)slab_b[(size_t)row * R + i] : 0.0;
  }
  __syncthreads();
#pragma unroll
  for (int st = 128; st >= 1; st >>= 1) {
    if (grp < st) part[tid] += part[tid + 4 * st];
    __syncthreads();
  }
  if (tid < 64) {
    // entry i of the gradient region: g (i < P) or the packet statistics
    const int e = i < P ? i : LM_NPMAX + i - P;
    const bool act = tid < 4 && i < P + 4;
    double v = tid < 4 ? part[tid] : 0.0;
    if (lm.dp_fused) v = lm_dp_sum_wave(lm.dp, seq, pw, v, e, act);
    if (act) red[LM_GBLK_MAX + e] = v;
  }
}

// ---------------------------------------------------------------------------
// Solve kernel (one workgroup): accept / reject, damping, Cholesky, next trial.
// red_new: the reduced block of the trial just evaluated (all-reduced when
// data parallel); the state keeps the best point's block.
// ---------------------------------------------------------------------------
// fp64 reciprocal / reciprocal square root from the hardware approximations
// (v_rcp_f64 / v_rsq_f64, max rel. error 4.6e-8 / 5.2e-8 on gfx950) + ONE
// Newton step: 2.2e-15 / 4.0e-15 (tools/micro/rsq_prec.hip); the IEEE division
// and sqrt sequences cost ~100 ns each on the dependency chains of the solver
RPH_INLINE double lm_rcp(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return __builtin_fma(r, __builtin_fma(-x, r, 1.0), r);
}
RPH_INLINE double lm_rsq(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  return y * __builtin_fma(-0.5 * x * y, y, 1.5);
}


// Exact Newton step on the OUTPUT block at the best point (the value is
// linear in the output layer's N = out_n parameters [P - N, P), so the loss
// is exactly quadratic in them): 2 G_oo d = -g_o with the FULL-BATCH output
// Gram matrix gog (packed upper triangle, built on the matrix cores by the
// fit's last passes), the full-batch gradient, a Marquardt damping out_mu
// (relative, on the diagonal) and a ridge of lm.ridge x mean diagonal.  The
// N x N system goes to LDS, the whole workgroup eliminates it (LDL^T, one
// barrier per column), wave 0 runs both triangular solves by v_readlane (lane
// i owns entry i, N <= 64), d -> out[0, N).  *dl = the exact full-batch loss
// change g_o.d + d.G_oo d (< 0 for any positive damping).  False (nothing to
// apply) when a pivot is not positive.  Called by workgroup 0 of the final
// pass only.
RPH_INLINE double lm_og(const double* gog, int N, int i, int j) {
  const int lo = i < j ? i : j, hi = i < j ? j : i;
  return gog[lo * N - lo * (lo - 1) / 2 + (hi - lo)];
}

// ``pre`` (N * N <= 512): the caller's prefetched entries e = tid and tid +
// 256 of the row-major N x N Gram and this lane's gradient entry (loaded in
// the solve's prologue with everything else: no dependent round trip here)
struct LmOgPre {
  double v[2];
  double gi;
};

template <int P>
RPH_INLINE bool lm_out_newton(const double* gog, const double* g, const int N, const float ridge, const float mu,
                              double* A, double* out, double* dl, const LmOgPre* pre = nullptr) {
#pragma clang fp contract(off)
  const int tid = threadIdx.x, lane = tid & 63;
  const int o0 = P - N, LDA = 65;
  __shared__ double s_rid;
  double* const G2d = out + 64;  // the undamped diagonal 2 G_ii (the elimination overwrites A's)
  if (pre != nullptr) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + 256 * u;
      if (e < N * N) {
        const int i = e / N, j = e % N;
        A[i * LDA + j] = 2.0 * pre->v[u];
        if (i == j) G2d[i] = 2.0 * pre->v[u];
      }
    }
  } else {
    for (int e = tid; e < N * N; e += 256) {
      const int i = e / N, j = e % N;
      const double v = 2.0 * lm_og(gog, N, i, j);
      A[i * LDA + j] = v;
      if (i == j) G2d[i] = v;
    }
  }
  __syncthreads();
  if (tid < 64) {
    double dg = lane < N ? A[lane * LDA + lane] : 0.0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) dg += __shfl_xor(dg, o, 64);
    if (lane == 0) s_rid = (double)ridge * dg / (double)N;
  }
  __syncthreads();
  if (tid < N) {
    const double a = A[tid * LDA + tid];
    A[tid * LDA + tid] = (a + a * (double)mu) + s_rid;
  }
  __syncthreads();
  // LDL^T elimination over the whole workgroup (lower triangle): step k
  // subtracts A_ik A_jk / A_kk from every (i, j), k < j <= i; D_k = A_kk
  bool ok = true;
  // (one or two entries per thread: every load of a step in flight at once;
  // the upper triangle stays 2 G for the exact loss change below)
  for (int k = 0; k < N; ++k) {
    const double akk = A[k * LDA + k];
    ok = ok && akk > 0.0;
    const double inv = lm_rcp(akk);
    const int m = N - k - 1;
    for (int e = tid; e < m * m; e += 256) {
      const int i = k + 1 + e / m, j = k + 1 + e % m;
      if (j <= i) A[i * LDA + j] -= (A[i * LDA + k] * A[j * LDA + k]) * inv;
    }
    __syncthreads();
  }
  if (tid < 64) {
    // L z = b (L_ik = A_ik / D_k), z / D, L^T d = z: lane i holds entry i and
    // 1 / D_i (v_rcp_f64 + one Newton step, as lm_rcp)
    const double di = lane < N ? A[lane * LDA + lane] : 1.0;
    const double ri = lm_rcp(di);
    const double gi = lane < N ? (pre != nullptr ? pre->gi : g[o0 + lane]) : 0.0;
    double b = -gi;
    for (int k = 0; k < N; ++k) {
      const double zk = lmc_readlane(b, k) * lmc_readlane(ri, k);  // L_ik z_k = A_ik (z_k / D_k)
      if (lane > k && lane < N) b -= A[lane * LDA + k] * zk;
    }
    b *= ri;
    for (int k = N - 1; k >= 0; --k) {
      const double dk = lmc_readlane(b, k);
      if (lane < k) b -= (A[k * LDA + lane] * ri) * dk;
    }
    if (lane >= N) b = 0.0;
    if (lane < N) out[lane] = b;
    // exact loss change of the quadratic: g.d + d.G d (G undamped, full
    // batch: A's untouched upper triangle and the saved diagonal, from LDS)
    double gd = 0.0;
    for (int j = 0; j < N; ++j) {
      const int lo = lane < j ? lane : j, hi = lane < j ? j : lane;
      const double gj = lane < N ? (lane == j ? G2d[lane] : A[lo * LDA + hi]) : 0.0;
      gd += (0.5 * gj) * lmc_readlane(b, j);
    }
    double t = b * (gi + gd), tl = b * gi;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      t += __shfl_xor(t, o, 64);
      tl += __shfl_xor(tl, o, 64);
    }
    if (lane == 0) {
      *dl = t;
      dl[1] = tl;  // g.d (the linear part; the quadratic part d.G d = dl - g.d)
    }
  }
  __syncthreads();
  return ok;
}

// lm_out_newton for the net's own N = NU <= 22 output parameters with the
// prologue's prefetched entries: the same arithmetic in the same order
// (bitwise the same step), but after the workgroup-wide fill ONE wave does
// the elimination (wave-synchronous LDS, a wavefront fence per column instead
// of a workgroup barrier; compile-time N, every step's loads in flight at
// once) and the triangular solves with each lane's row / column of the
// factor loaded up front (readlane + fma chains only).  Every thread calls it.
template <int P, int N>
RPH_INLINE bool lm_out_newton_w1(const LmOgPre& pre, const float ridge, const float mu, double* A, double* out,
                                 double* dl) {
#pragma clang fp contract(off)
  static_assert(N >= 1 && N * N <= 512, "prefetched output step: N * N <= 512");
  const int tid = threadIdx.x, lane = tid & 63;
  constexpr int LDA = 65;
  __shared__ int s_ok;
  double* const G2d = out + 64;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = tid + 256 * u;
    if (e < N * N) {
      const int i = e / N, j = e % N;
      A[i * LDA + j] = 2.0 * pre.v[u];
      if (i == j) G2d[i] = 2.0 * pre.v[u];
    }
  }
  __syncthreads();
  if (tid < 64) {
    double dg = lane < N ? A[lane * LDA + lane] : 0.0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) dg += __shfl_xor(dg, o, 64);
    const double rid = (double)ridge * dg / (double)N;
    if (lane < N) {
      const double a = A[lane * LDA + lane];
      A[lane * LDA + lane] = (a + a * (double)mu) + rid;
    }
    lmc_wave_sync();
    bool ok = true;
    lm_static_for<N>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      constexpr int MK = N - k - 1;                 // trailing rows / columns
      constexpr int NT = (MK * MK + 63) / 64;       // square slots per lane (c > r skipped)
      const double akk = A[k * LDA + k];
      double aik[NT > 0 ? NT : 1], ajk[NT > 0 ? NT : 1], aij[NT > 0 ? NT : 1];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int e = lane + 64 * t < MK * MK ? lane + 64 * t : 0;
        const int i = k + 1 + e / MK, j = k + 1 + e % MK;
        aik[t] = A[i * LDA + k];
        ajk[t] = A[j * LDA + k];
        aij[t] = A[i * LDA + j];
      }
      ok = ok && akk > 0.0;
      const double inv = lm_rcp(akk);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int e = lane + 64 * t;
        if (e < MK * MK) {
          const int i = k + 1 + e / MK, j = k + 1 + e % MK;
          if (j <= i) A[i * LDA + j] = aij[t] - (aik[t] * ajk[t]) * inv;
        }
      }
      lmc_wave_sync();
    });
    // L z = b, z / D, L^T d = z (lm_out_newton's order): this lane's row and
    // column of the factor first
    const int li = lane < N ? lane : 0;
    double rw[N], cl[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
      rw[k] = A[li * LDA + k];
      cl[k] = A[k * LDA + li];
    }
    const double di = lane < N ? A[lane * LDA + lane] : 1.0;
    const double ri = lm_rcp(di);
    const double gi = lane < N ? pre.gi : 0.0;
    double b = -gi;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const double zk = lmc_readlane(b, k) * lmc_readlane(ri, k);
      if (lane > k && lane < N) b -= rw[k] * zk;
    }
    b *= ri;
#pragma unroll
    for (int k = N - 1; k >= 0; --k) {
      const double dk = lmc_readlane(b, k);
      if (lane < k) b -= (cl[k] * ri) * dk;
    }
    if (lane >= N) b = 0.0;
    if (lane < N) out[lane] = b;
    // exact loss change: g.d + d.G d (G undamped: A's upper triangle, G2d)
    double gd = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const double gj = lane < N ? (lane == j ? G2d[li] : (lane < j ? rw[j] : cl[j])) : 0.0;
      gd += (0.5 * gj) * lmc_readlane(b, j);
    }
    double t = b * (gi + gd), tl = b * gi;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      t += __shfl_xor(t, o, 64);
      tl += __shfl_xor(tl, o, 64);
    }
    if (lane == 0) {
      *dl = t;
      dl[1] = tl;
      s_ok = ok ? 1 : 0;
    }
  }
  __syncthreads();
  return s_ok != 0;
}

// Solve kernel, LM_SPEC workgroups.  Every workgroup takes the same
// accept / reject decision from the same inputs (the scalar slot of this
// pass's parity, which no workgroup of this launch writes: workgroup 0
// writes the other slot).  Then:
//  * final pass: workgroup 0 publishes the best point;
//  * a rejection whose damping was precomputed (LSS_SPEC_IDX): workgroup 0
//    publishes that step, no factorisation;
//  * otherwise (accept, or no precomputed step): workgroup m factorises the
//    system at the damping after m further consecutive rejections (m = 0 is
//    this solve's own step) — the same arithmetic a later serial solve would
//    do, so the results are bitwise those of one-solve-per-pass.
template <int P, int R, int NU>
__global__ __launch_bounds__(256) void k_lm_solve(const TrainDesc d, const LmDesc lm, const double* __restrict__ red_new,
                                                  const int pass) {
  // no implicit fma contraction: every workgroup (own step or a speculative
  // one) must round identically, whatever code copy the compiler makes
#pragma clang fp contract(off)
  using LS = LmShape<P>;
  constexpr int NB = LS::NB, NBLK = LS::NBLK;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int s_fail;
  __shared__ double s_diag;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m = blockIdx.x;
  // diagnostic phase stamps (tools/stamp_lm.py) of the own-step workgroup,
  // kept in registers of thread 0 and written to stamp row 0 only at the end
  // of a full factorising solve, so the row never mixes solves of different kinds
  unsigned long long ts[8] = {};
  const bool stamp_on = d.stamps != nullptr && m == 0 && blockIdx.y == 0 && tid == 0;
#define RPH_STAMPS(k)                                        \
  do {                                                       \
    if (stamp_on) ts[(k)] = rph_stamp_clock();                \
  } while (0)
  RPH_STAMPS(0);
#ifdef RPH_LDS_POISON
  // diagnostic build: every dynamic-LDS double starts as NaN (a read before
  // any write then shows in the result instead of an earlier kernel's data)
  for (int i = tid; i < TileGrid<P>::LDS_BYTES / 8; i += 256) lds[i] = __builtin_nan("");
  __syncthreads();
#endif
  const int inst = blockIdx.y;  // multi-start instance
  double* st = lm.state + (size_t)inst * LMS_FLOATS;
  red_new += (size_t)inst * LM_RED;
  double* best_red = st + LMS_RED;  // the best point's reduced block
  const double* sin = st + LMS_SLOTS + LM_SLOT * (pass & 1);  // read by every workgroup
  double* sout = st + LMS_SLOTS + LM_SLOT * ((pass + 1) & 1);  // written by workgroup 0
  // ---- scalars of this pass ------------------------------------------------------
  // Every load of the prologue is unconditional (clamped indices, both
  // outcomes of the acceptance test), so all of them are in flight at once: a
  // load under a condition waits out its own round trip, and the solve's
  // setup was a chain of them
  const double sv_best = sin[LSS_BEST], sv_lbest = sin[LSS_LBEST], sv_stop = sin[LSS_STOP];
  const double sv_lam = sin[LSS_LAM], sv_nu = sin[LSS_NU], sv_pred = sin[LSS_PRED], sv_sidx = sin[LSS_SPEC_IDX];
  // the trial's packet statistics [loss, |e|, ape, count]
  const double t_loss = red_new[LM_GBLK_MAX + LM_NPMAX], cnt = red_new[LM_GBLK_MAX + LM_NPMAX + 3];
  double sp_lam[LM_SPEC], sp_ok[LM_SPEC], sp_pred[LM_SPEC];
#pragma unroll
  for (int k = 0; k < LM_SPEC; ++k) {
    sp_lam[k] = st[LMS_SPEC_LAM + k];
    sp_ok[k] = st[LMS_SPEC_OK + k];
    sp_pred[k] = st[LMS_SPEC_PRED + k];
  }
  // per-parameter values of a full solve, for either best point
  constexpr int NDS = (P + 63) / 64;  // diagonal entries per lane (the damping scale)
  const int tc = tid < P ? tid : P - 1;
  const double w_slot0 = st[LMS_W + tc], w_slot1 = st[LMS_W + LM_NPMAX + tc];
  const double g_new = red_new[LM_GBLK_MAX + tc], g_old = best_red[LM_GBLK_MAX + tc];
  const double d_new = lmc_gram<TileGrid<P>::NBG>(red_new, tc, tc), d_old = lmc_gram<TileGrid<P>::NBG>(best_red, tc, tc);
  double ds_new[NDS], ds_old[NDS];
#pragma unroll
  for (int k = 0; k < NDS; ++k) {
    const int i = lane + 64 * k < P ? lane + 64 * k : P - 1;
    ds_new[k] = lmc_gram<TileGrid<P>::NBG>(red_new, i, i);
    ds_old[k] = lmc_gram<TileGrid<P>::NBG>(best_red, i, i);
  }
  // final pass: the output step's inputs for either outcome (the trial's and
  // the best point's packed output Gram, its marker and gradient entries)
  // with the rest of the prologue - a dependent round trip each otherwise
  const bool final_pass = pass == lm.passes;
  constexpr bool OG_PRE = NU * NU <= 512;
  LmOgPre og_pre[2];  // [trial block, best block]
  double ogm_new = -1.0, ogm_old = -1.0;
  if constexpr (OG_PRE) {
    if (final_pass && m == 0 && lm.out_gram && lm.out_n == NU) {
      ogm_new = red_new[LM_RED_OUTG];
      ogm_old = best_red[LM_RED_OUTG];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int e = tid + 256 * u < NU * NU ? tid + 256 * u : 0;
        og_pre[0].v[u] = lm_og(red_new + LM_RED_OUTG, NU, e / NU, e % NU);
        og_pre[1].v[u] = lm_og(best_red + LM_RED_OUTG, NU, e / NU, e % NU);
      }
      const int gl = P - NU + (lane < NU ? lane : 0);
      og_pre[0].gi = red_new[LM_GBLK_MAX + gl];
      og_pre[1].gi = best_red[LM_GBLK_MAX + gl];
    }
  }
  const int best_old = pass == 0 ? 1 : (int)sv_best;
  const int trial = 1 - best_old;
  const double Lt = t_loss / fmax(cnt, 1.0);
  const double Lb = pass == 0 ? INFINITY : sv_lbest;
  // adaptive budget spent at an earlier solve: the trial block is stale
  const bool stopped = pass > 0 && sv_stop != 0.0;
  const bool accept = !stopped && (pass == 0 || (Lt == Lt && Lt < Lb));
  double lam = sv_lam, nu = sv_nu;
  const double pred_prev = sv_pred;
  const int sidx = (int)sv_sidx;
  int best = best_old;
  if (stopped) {
  } else if (accept) {
    best = trial;
    if (pass > 0 && lm.damping == 1) {
      // Nielsen: gain ratio of the actual to the model-predicted reduction
      const double rho = pred_prev > 0.0 ? (Lb - Lt) / pred_prev : 1.0;
      const double t = 2.0 * rho - 1.0;
      lam = fmax(lam * fmax(1.0 / 3.0, 1.0 - t * t * t), (double)lm.lam_min);
      nu = 2.0;
    } else if (pass > 0) {
      lam = fmax(lam * lm.lam_down, (double)lm.lam_min);
    }
  } else if (lm.damping == 1) {
    lam = fmin(lam * nu, (double)lm.lam_max);
    nu *= 2.0;
  } else {
    lam = fmin(lam * lm.lam_up, (double)lm.lam_max);
  }
  // a rejection whose step the last full solve precomputed (same damping,
  // same best point: rejections do not move it)
  double sl = 0.0, so = 0.0, sq = 0.0;
#pragma unroll
  for (int k = 1; k < LM_SPEC; ++k)
    if (k == sidx) {
      sl = sp_lam[k];
      so = sp_ok[k];
      sq = sp_pred[k];
    }
  const bool spec = !final_pass && !accept && pass > 0 && sidx >= 1 && sidx < LM_SPEC && sl == lam;
  const int spec_ok = spec ? (so != 0.0) : 0;
  const double spec_pred = spec ? sq : 0.0;
  // the damping of this workgroup's system: m further rejections
  double lam_m = lam, nu_m = nu;
  for (int k = 0; k < m; ++k) {
    if (lm.damping == 1) {
      lam_m = fmin(lam_m * nu_m, (double)lm.lam_max);
      nu_m *= 2.0;
    } else {
      lam_m = fmin(lam_m * lm.lam_up, (double)lm.lam_max);
    }
  }
  // the next pass's scalars (workgroup 0, thread 0): best slot, damping, growth
  // factor, predicted reduction, copy flag (the best point's block := the
  // trial's, copied by the next pass kernel), next precomputed step, best loss
  auto publish = [&](double lam_out, double pred_out, double sidx_out) {
    if (tid == 0) {
      // adaptive budget: an ACCEPTED step that lowered the best loss by less
      // than stop_tol (rejections only raise the damping: with lam_carry warm
      // starts the first trial is often rejected before any progress)
      const bool stop_now = lm.stop_tol > 0.f && pass >= lm.stop_min && accept && !(Lb - Lt > (double)lm.stop_tol * Lt);
      sout[LSS_STOP] = stop_now ? (double)pass : 0.0;
      sout[LSS_BEST] = (double)best;
      sout[LSS_LAM] = lam_out;
      sout[LSS_NU] = nu;
      sout[LSS_PRED] = pred_out;
      sout[LSS_COPY] = accept ? 1.0 : 0.0;
      sout[LSS_SPEC_IDX] = sidx_out;
      sout[LSS_LBEST] = accept ? Lt : Lb;
      st[LMS_BEST] = (double)best;  // host mirrors
      st[LMS_LAM] = lam_out;
      if (accept && pass > 0) st[LMS_NACC] += 1.0;
      if (pass < MAXHIST && !lm.weights_only && !lm.explore) d.fit->hist[pass] = (float)Lt;
    }
  };
  if (stopped && !final_pass) {  // carry the scalars to the next pass (no copy of the stale block)
    if (m == 0 && tid < LM_SLOT) sout[tid] = tid == LSS_COPY ? 0.0 : sin[tid];
    return;
  }
  RPH_STAMPS(1);
  const double* src = accept ? red_new : best_red;  // the best point's block
  const double* g = src + LM_GBLK_MAX;
  if (final_pass) {  // publish the best point
    if (m != 0) return;
    if (stopped) {
      if (tid == 0) {
        st[LMS_BEST] = (double)best;
        st[LMS_LAM] = lam;
      }
    } else {
      publish(lam, pred_prev, (double)LM_SPEC);
    }
    if (tid == 0) st[LMS_LFIN] = accept ? Lt : Lb;
    if (lm.explore) return;  // exploration: k_lm_select publishes the chosen start point
    // exact Newton step on the whole (linear) output layer with the
    // full-batch output Gram (when the best point's pass built it), else on
    // the bond bias alone
    const int on = lm.out_n;
    __shared__ double s_dl2[2];  // the step's exact loss change, its linear part g.d
    double& s_dl = s_dl2[0];
    const bool on_ok = on > 0 && on <= LM_OG_MAX && on <= P && lm.out_gram;
    // the last evaluation (this pass) built the output Gram: the out step at
    // the best point when it was accepted, else at the rejected last trial -
    // published when trial + step beats the best point (its loss change is
    // exact: the trial's own full-batch Gram and gradient)
    const bool pre_ok = OG_PRE && on == NU;  // (the prologue loaded both candidates)
    const bool have_og = on_ok && (pre_ok ? (accept ? ogm_new : ogm_old) : src[LM_RED_OUTG]) >= 0.0;
    auto newton = [&](const double* gog, const double* gg, const LmOgPre* pr) {
      if constexpr (OG_PRE) {
        if (pre_ok) return lm_out_newton_w1<P, NU>(*pr, lm.ridge, lm.out_mu, lds, lds + 64 * 65, s_dl2);
      }
      return lm_out_newton<P>(gog, gg, on, lm.ridge, lm.out_mu, lds, lds + 64 * 65, s_dl2, pre_ok ? pr : nullptr);
    };
    // trust region (lm.out_tr > 0): ||d|| <= out_tr x max(||w_o||, 1e-3
    // sqrt(on)) for the output weights w_o of point pt; a longer step is
    // scaled onto the boundary and its exact loss change (a g.d + a^2 d.G d,
    // the loss is quadratic along d) replaces s_dl - before any decision on it
    __shared__ double s_nrm[2][4];
    auto trust = [&](const int pt) {
      if (!(lm.out_tr > 0.f)) return;
      double dd = 0.0, ww = 0.0;
      if (tid < P && tid >= P - on) {
        const double di = lds[64 * 65 + tid - (P - on)], wi = pt == 0 ? w_slot0 : w_slot1;
        dd = di * di;
        ww = wi * wi;
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        dd += __shfl_xor(dd, o, 64);
        ww += __shfl_xor(ww, o, 64);
      }
      if (lane == 0) {
        s_nrm[0][wid] = dd;
        s_nrm[1][wid] = ww;
      }
      __syncthreads();
      const double nd = sqrt((s_nrm[0][0] + s_nrm[0][1]) + (s_nrm[0][2] + s_nrm[0][3]));
      const double nw = sqrt((s_nrm[1][0] + s_nrm[1][1]) + (s_nrm[1][2] + s_nrm[1][3]));
      const double rad = (double)lm.out_tr * fmax(nw, 1e-3 * sqrt((double)on));
      if (nd > rad) {
        const double a = rad / nd;
        if (tid < on) lds[64 * 65 + tid] *= a;
        if (tid == 0) s_dl2[0] = a * s_dl2[1] + a * a * (s_dl2[0] - s_dl2[1]);
      }
      __syncthreads();
    };
    bool out_ok = have_og && newton(src + LM_RED_OUTG, g, &og_pre[accept ? 0 : 1]);
    if (out_ok) trust(best);
    bool use_trial = false;
    // (only for a trial within 2x the best loss: the step must then remove
    // little more than Lt - Lb, and its predicted change, exact up to the
    // Gram's ~1e-5 rounding, is a reliable decision - a far-off trial's
    // Lt + dl would cancel catastrophically)
    if (!have_og && !stopped && !accept && on_ok && (pre_ok ? ogm_new : red_new[LM_RED_OUTG]) >= 0.0 && Lt == Lt &&
        Lt < 2.0 * Lb) {
      const bool ok_t = newton(red_new + LM_RED_OUTG, red_new + LM_GBLK_MAX, &og_pre[0]);
      if (ok_t) trust(trial);
      use_trial = ok_t && Lt == Lt && Lt + s_dl < Lb;
      out_ok = use_trial;
    }
    __syncthreads();
    const int pub_pt = use_trial ? trial : best;  // the point the published weights start from

    for (int i = tid; i < P; i += 256) {
      double wd = pub_pt == 0 ? w_slot0 : w_slot1;  // (the prologue's loads: i = tid < P <= 256)
      if (out_ok) {
        if (i >= P - on) wd += lds[64 * 65 + i - (P - on)];
      } else if (i == lm.bias_index) {
        // exact Newton step on this bias alone (the loss is quadratic in it):
        // d = -g_i / (2 G_ii); the bias is the bond holding's, dV / db = B_{t+1}
        // on every path, so G_ii = B^2 exactly (not the subsample Gram's
        // rounded entry): d = -mean(e) / B
        const double gii = (double)d.bond * (double)d.bond;
        if (gii > 0.0) wd -= g[i] / (2.0 * gii);
      }
      const float w = (float)wd;
      d.wts->w[0][i] = w;
      d.fit->w_best[i] = w;
    }
    if (tid == 0 && !lm.weights_only) {
      const double* sb = src + LM_GBLK_MAX + LM_NPMAX;
      const double c = fmax(sb[3], 1.0);
      FitState* f = d.fit;
      // (after an output step: the exact full-batch loss of the published weights)
      const double lbest = (use_trial ? Lt : accept ? Lt : Lb) + (out_ok ? s_dl : 0.0);
      f->best_loss = (float)lbest;
      f->last_loss = (float)lbest;
      f->last_mae = (float)(sb[1] / c);
      f->last_mape = (float)(100.0 * sb[2] / c);
      f->epoch = (float)((stopped ? (int)sin[LSS_STOP] : pass) + 1);  // points evaluated
      f->stopped = 1.f;
      f->has_best = 1.f;
      f->wait = 0.f;
      f->loss_sum = f->abs_sum = f->ape_sum = f->loss_cnt = 0.f;
    }
    return;
  }
  if (spec) {  // rejection with a precomputed step: publish it
    if (m != 0) return;
    for (int i = tid; i < P; i += 256)
      st[LMS_W + (1 - best) * LM_NPMAX + i] =
          spec_ok ? st[LMS_SPEC_W + sidx * LM_NPMAX + i] : st[LMS_W + best * LM_NPMAX + i];
    if (spec_ok) {
      publish(lam, spec_pred, (double)(sidx + 1));
    } else {  // not positive definite at this damping: as the serial solve's failure branch
      publish(fmin(lam * lm.lam_up * lm.lam_up, (double)lm.lam_max), pred_prev, (double)LM_SPEC);
      if (tid == 0) {
        st[LMS_FAIL] += 1.0;
        st[LMS_FAILTOT] += 1.0;
      }
    }
    return;
  }
  // a precomputed step is used at the solve of pass + m (< passes): skip the rest
  if (m > 0 && pass + m > lm.passes - 1) return;
  // ---- tile-store Cholesky (lm_chol.h): panel wave 0, owner waves 1..3 ------
  using TG = TileGrid<P>;
  double* T = lds;
  double* vec = lds + TG::OFF_D;  // the solution d
  unsigned* pub = reinterpret_cast<unsigned*>(lds + TG::OFF_FLAGS);
  unsigned* fac = pub + TG::NT + 1;
  unsigned* xdone = fac + TG::NT + 1;  // owner waves done inverting the diagonal blocks
  static_assert(P <= 256, "one parameter per thread");
  const double gi = tid < P ? (accept ? g_new : g_old) : 0.0;
  const double wbest = tid < P ? (best == 0 ? w_slot0 : w_slot1) : 0.0;  // for the final update
  const double a_ii = tid < P ? 2.0 * (accept ? d_new : d_old) : 0.0;
  // the Gram block into the tile store with coalesced loads, in flight
  // across the damping setup below (up to 16 tiles per owner wave: the larger
  // nets' owners load their tiles from the Gram block after the setup)
  constexpr bool STAGED = TG::TPW <= 16;
  if constexpr (LmTPack<P>::ON) {
    // the reduce kernel's tile-store image: a contiguous copy (every load
    // in flight before the first store)
    static_assert(LmTPack<P>::LEN % 256 == 0, "whole tiles");
    constexpr int NQ = LmTPack<P>::LEN / 256;  // loads per thread
    const double* s1 = src + LmTPack<P>::OFF;
    double v[NQ];
#pragma unroll
    for (int u = 0; u < NQ; ++u) v[u] = s1[u * 256 + tid];
#pragma unroll
    for (int u = 0; u < NQ; ++u) T[u * 256 + tid] = v[u];
  } else if constexpr (STAGED) {
    lmc_stage<P>(T, src);
  }
  if (wid == 0) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < NDS; ++k)
      if (lane + 64 * k < P) s += 2.0 * (accept ? ds_new[k] : ds_old[k]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) {
      s_diag = s / P;
      s_fail = 0;
    }
  }
  if (tid < 2 * (TG::NT + 1) + 1) pub[tid] = 0u;  // pub, fac, xdone
  __syncthreads();
  double dmp = 0.0;  // this parameter's damping term lam 2G_ii + ridge (for the predicted reduction)
  if (tid < P) {
    // Marquardt scaling with a floor: a parameter whose subsample curvature
    // vanishes (a hidden unit dead on the Gram subsample, active elsewhere)
    // still gets damped, so growing lam always shortens its step
    dmp = fmax(a_ii, (double)lm.diag_floor * s_diag) * lam_m + (double)lm.ridge * s_diag;
    lds[TG::OFF_DIAG + tid] = a_ii + dmp;
    // the rhs row -g into the staged store (after the setup barrier: the image
    // copy above writes these places too)
    if constexpr (STAGED) T[TG::tidx(P >> 4, tid >> 4) * 256 + tg_off(P & 15, tid & 15)] = -gi;
  }
  RPH_STAMPS(2);
  __syncthreads();  // the damped diagonal is in place
  switch (wid) {
    case 0:
    {
      unsigned long long* stp = (m == 0 && blockIdx.y == 0 && d.stamps != nullptr) ? reinterpret_cast<unsigned long long*>(d.stamps) + 8 : nullptr;
      lmc_panels<P>(T, lds + TG::OFF_RDG, lds + TG::OFF_BC, pub, fac, &s_fail, stp);
    }
      RPH_STAMPS(6);
      lmc_backward<P>(T, lds + TG::OFF_RDG, vec, lds + TG::OFF_X, xdone, &s_fail);
      RPH_STAMPS(7);
      break;
    case 1:
      LmcOwner<P, 0>::template run<STAGED>(src, lds + TG::OFF_DIAG, g, T, pub, fac, &s_fail, lds + TG::OFF_RDG,
                                             lds + TG::OFF_X, xdone);
      break;
    case 2:
      LmcOwner<P, 1>::template run<STAGED>(src, lds + TG::OFF_DIAG, g, T, pub, fac, &s_fail, lds + TG::OFF_RDG,
                                             lds + TG::OFF_X, xdone);
      break;
    default:
      LmcOwner<P, 2>::template run<STAGED>(src, lds + TG::OFF_DIAG, g, T, pub, fac, &s_fail, lds + TG::OFF_RDG,
                                             lds + TG::OFF_X, xdone);
      break;
  }
  __syncthreads();
  RPH_STAMPS(3);
#ifdef RPH_DUMP_T
  // diagnostic build: the factored tile store -> d.stamps (as doubles)
  if (m == 0 && d.stamps != nullptr)
    for (int i = tid; i < TG::NTILE * 256 + 2 * TG::PT; i += 256) reinterpret_cast<double*>(d.stamps)[i] = lds[i];
#endif
  const bool failed = s_fail != 0;
  // predicted reduction of the quadratic model at the step d:
  // -(g.d)/2 + d.(lam D + ridge) d / 2   ((2G + lam D + ridge) d = -g)
  __shared__ double s_pred[4];
  if (!failed) {
    double pv = 0.0;
    if (tid < P) {
      const double dv = vec[tid];
      pv = 0.5 * (dmp * dv * dv - gi * dv);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) pv += __shfl_xor(pv, o, 64);
    if (lane == 0) s_pred[wid] = pv;
    __syncthreads();
  }
  const double pred = (s_pred[0] + s_pred[1]) + (s_pred[2] + s_pred[3]);
  if (m > 0) {  // speculative step: its own slot of the state
    if (tid < P) st[LMS_SPEC_W + m * LM_NPMAX + tid] = failed ? wbest : wbest + vec[tid];
    if (tid == 0) {
      st[LMS_SPEC_LAM + m] = lam_m;
      st[LMS_SPEC_PRED + m] = failed ? 0.0 : pred;
      st[LMS_SPEC_OK + m] = failed ? 0.0 : 1.0;
    }
    return;
  }
  RPH_STAMPS(4);
  if (failed) {
    // not positive definite at this damping: re-evaluate the best point with
    // more damping (trial := best)
    if (tid < P) st[LMS_W + (1 - best) * LM_NPMAX + tid] = wbest;
    publish(fmin(lam * lm.lam_up * lm.lam_up, (double)lm.lam_max), pred_prev, (double)LM_SPEC);
    if (tid == 0) {
      st[LMS_FAIL] += 1.0;
      st[LMS_FAILTOT] += 1.0;
    }
    return;
  }
  RPH_STAMPS(5);
  if (tid < P) st[LMS_W + (1 - best) * LM_NPMAX + tid] = wbest + vec[tid];
  publish(lam, pred, 1.0);
  if (stamp_on)
    for (int k = 0; k < 8; ++k) d.stamps[k] = ts[k];
#undef RPH_STAMPS
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
template <int NIN, int H, int NO, int HEAD>
struct LmKernels {
  // two paths per lane, packed fp32; one or two pass workgroups per CU
  // (Body::WAVES_PER_SIMD: two where the plain body fits 256 VGPRs)
  using Body = NarrowPairBody<NIN, H, NO, HEAD>;
  // the same body + the full-batch output-layer Gram on the matrix cores (the
  // last LM_OUTG_TAIL passes of an lm_out_fix fit)
  using BodyOG = NarrowPairBody<NIN, H, NO, HEAD, true>;
  using S = NetShape<NIN, H, NO, HEAD>;
  // the tile store + vectors + hand-off counters (lm_chol.h)
  static constexpr int smem() { return TileGrid<S::P>::LDS_BYTES; }
  static_assert(smem() + 128 <= 160 * 1024, "LM solve exceeds the LDS of one workgroup");
};

static int lm_validate(const TrainDesc* d, const LmDesc* lm, int P, int R, int nblk, int nu) {
  if (int rc = validate_train(d, 3 /* no schedule buffers */, "rph_lm")) return rc;
  if (!lm->state || !lm->slab_b || !lm->slab_g) return rph_report("rph_lm", "null LM buffer");
  if (d->batch != d->n_local || d->steps_per_epoch != 1) return rph_report("rph_lm", "LM fits are full batch");
  if (lm->num_wgs < 1 || lm->num_wgs > LM_PASS_WGS_MAX || lm->passes < 0 || lm->passes >= MAXHIST)
    return rph_report("rph_lm", "bad num_wgs (1..512) / passes");
  if (lm->leaf_blocks < 0 || (lm->leaf_blocks > 0 && (long long)lm->leaf_blocks * 128 * 4 * lm->num_wgs < d->batch))
    return rph_report("rph_lm", "leaf_blocks: the waves' leaves must cover the shard");
  if (lm->gram_wgs < 1 || lm->gram_wgs > 65535) return rph_report("rph_lm", "bad Gram workgroup count");
  if (lm->gram_base != 0 && (lm->gram_base != lm->num_wgs || lm->inst != 1))
    return rph_report("rph_lm", "gram_base: 0 or the path grid (one instance)");
  if (lm->gram_side) {
    // the subsample comes from gfeat / gprice ([gram_wgs x 64] each)
    const int nhold = d->head == HEAD_COMPLEMENT ? 2 : d->nout;
    for (int f = 0; f < d->nin; ++f)
      if (!lm->gfeat[f]) return rph_report("rph_lm", "null Gram subsample feature");
    for (int k = 0; k < nhold - 1; ++k)
      if (!lm->gprice[k]) return rph_report("rph_lm", "null Gram subsample price");
  } else {
    // (Gram-only workgroups past num_wgs read the shard too)
    if (lm->gram_blk < 1 || lm->gram_blk > lm->gram_blk_stride)
      return rph_report("rph_lm", "bad Gram subsample geometry");
    const long long ns = (long long)lm->gram_wgs * LM_TILE;  // the last slot must stay inside the shard
    const long long last = ((ns - 1) / lm->gram_blk) * lm->gram_blk_stride + (ns - 1) % lm->gram_blk;
    if (last >= d->n_local) return rph_report("rph_lm", "Gram subsample leaves the shard");
  }
  if (lm->red_wgs != nblk * 1024 / 64 + R / 4 + lm_og_wgs(nu)) return rph_report("rph_lm", "bad red_wgs");
  if (lm->out_gram && (!lm->slab_o || nu > LM_OG_MAX)) return rph_report("rph_lm", "output Gram needs slab_o (<= 64 output parameters)");
  if (d->loss != LOSS_MSE && d->loss != LOSS_PINBALL) return rph_report("rph_lm", "LM fits: MSE or pinball loss");
  if (d->loss == LOSS_PINBALL && ((lm->gram_side && !lm->gtarget) || lm->out_gram || lm->out_n > 0 ||
                                  lm->bias_index >= 0 || !(lm->q_delta > 0.f)))
    return rph_report("rph_lm", "pinball LM fits: subsample targets with a simulated subsample, no output / "
                                "bias step, q_delta > 0");
  if (R != 128 && R != 256) return rph_report("rph_lm", "packet width must be 128 or 256");
  if (lm->inst < 1 || lm->inst > LM_SEL_MAX) return rph_report("rph_lm", "bad instance count");
  if (lm->inst > 1 && !lm->explore) return rph_report("rph_lm", "several instances are exploration fits only");
  if (lm->dp_fused) {
    const int nflags = R / 4 + lm_og_wgs(nu);
    if (!lm->gram_side || lm->inst != 1 || lm->explore || lm->weights_only)
      return rph_report("rph_lm", "fused DP exchange: one main fit on the shared Gram subsample only");
    if (lm->dp.world < 2 || lm->dp.world > 8 || lm->dp.rank < 0 || lm->dp.rank >= lm->dp.world ||
        lm->dp.pitch < LM_DP_PITCH || !lm->dp.counter || !lm->dp.error || nflags > LM_DP_FLAGS)
      return rph_report("rph_lm", "fused DP exchange: bad mailbox descriptor");
    for (int q = 0; q < lm->dp.world; ++q)
      if (!lm->dp.mbox[q]) return rph_report("rph_lm", "fused DP exchange: null peer mailbox");
  }
  if (lm->explore && lm->weights_only) return rph_report("rph_lm", "exploration fits publish nothing");
  (void)P;
  return 0;
}

template <int A, int B, int C, int E>
static int lm_pass_launch(const TrainDesc* d, const LmDesc* lm, int pass, const double* red_new, hipStream_t s) {
  using K = LmKernels<A, B, C, E>;
  // path workgroups + Gram-only workgroups past them (Gram subsample > 64 x path grid)
  const bool og = lm->out_gram && pass > lm->passes - LM_OUTG_TAIL;
  // (the final evaluation builds no Gram tile: the path grid alone)
  const int gend = pass == lm->passes ? 0 : (og && K::BodyOG::OGM ? 0 : lm->gram_base) + lm->gram_wgs;
  const unsigned grid = (unsigned)(gend > lm->num_wgs ? gend : lm->num_wgs);
  if constexpr (K::BodyOG::OGM) {
    // the last LM_OUTG_TAIL evaluations of an lm_out_fix fit build the output Gram
    if (og) {
      hipLaunchKernelGGL((k_lm_pass<typename K::BodyOG>), dim3(grid, lm->inst), dim3(256), 0, s, *d, *lm, pass,
                         red_new);
      return (int)hipGetLastError();
    }
  }
  hipLaunchKernelGGL((k_lm_pass<typename K::Body>), dim3(grid, lm->inst), dim3(256), 0, s, *d, *lm, pass, red_new);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Data-parallel all-reduce of the LM reduced block [G | g | stats] over the
// IPC-mapped peer mailboxes (the xGMI transport; RCCL otherwise).  Workgroup
// wg owns one chunk of the block: it pushes its chunk into every peer's
// mailbox with system-scope stores, drains, raises one flag per peer, waits
// for every peer's flag of the same chunk, and sums the W chunks in fixed
// rank order — every rank gets the bitwise-identical block (so the solves and
// the accept / reject decisions agree).  The tag is a per-rank device
// exchange counter (graph replays never see stale flags); the last workgroup
// to finish advances it.  Spins are bounded (DP_SPIN_TICKS -> error[0]).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_lm_dp_exchange(const LmDpDesc x, double* __restrict__ red, const int ng,
                                                         const int p) {
  __shared__ unsigned s_seq;
  const int tid = threadIdx.x, wg = blockIdx.x, W = x.world, me = x.rank;
  if (tid == 0) s_seq = __hip_atomic_load(x.counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const unsigned seq = s_seq;
  const int slot = (int)(seq % DP_SLOTS);
  (void)p;
  const int len = ng + (LM_RED - LM_GBLK_MAX), chunk = (len + LM_DP_WGS - 1) / LM_DP_WGS;
  const int e0 = wg * chunk, e1 = min(len, e0 + chunk);
  auto off = [&](int e) {  // block entry -> offset in red: the ng Gram entries, then the gradient region
    return e < ng ? e : LM_GBLK_MAX + e - ng;
  };
  for (int e = e0 + tid; e < e1; e += 256) {
    const double v = red[off(e)];
    for (int q = 0; q < W; ++q)
      if (q != me)
        __hip_atomic_store(x.mbox[q] + ((size_t)slot * W + me) * x.pitch + e, v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (tid < W && tid != me) {
    unsigned* fo = reinterpret_cast<unsigned*>(x.mbox[tid] + ((size_t)slot * W + me) * x.pitch + LM_RED + wg);
    __hip_atomic_store(fo, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* fi =
        reinterpret_cast<const unsigned*>(x.mbox[me] + ((size_t)slot * W + tid) * x.pitch + LM_RED + wg);
    unsigned it = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(fi, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
      __builtin_amdgcn_s_sleep(2);
      if ((++it & 255u) == 0u && (__builtin_amdgcn_s_memrealtime() - t0 > DP_SPIN_TICKS ||
                                  __hip_atomic_load(x.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)) {
        __hip_atomic_store(x.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
  for (int e = e0 + tid; e < e1; e += 256) {
    const int o = off(e);
    double s = 0.0;
    for (int q = 0; q < W; ++q)
      s += q == me ? red[o]
                   : __hip_atomic_load(x.mbox[me] + ((size_t)slot * W + q) * x.pitch + e, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
    red[o] = s;
  }
  __syncthreads();
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add(x.counter + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == LM_DP_WGS - 1) {
      __hip_atomic_store(x.counter + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(x.counter, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------------------
// Data-parallel all-reduce of the gradient region [g | stats | output Gram]
// = the first `len` doubles of red[LM_GBLK_MAX, LM_RED) (200 doubles = 1.6 KB;
// + the packed output Gram in the last passes of an lm_out_fix fit: 171 more
// for the 1-8-8-2 net) when every rank builds the same Gram matrix from the
// simulated global subsample (LmDesc.gram_side): ONE workgroup, every lane
// pushes 16-byte pairs to every peer with a
// write-through (sc0 sc1: system scope) global_store_dwordx4, drain, one
// flag per peer (system-scope release), bounded acquire waits, fixed-rank-
// order sums (bitwise-identical replicas).  Same mailbox rows, flag slot and
// exchange counter as k_lm_dp_exchange (the sequence tags stay monotonic).
// ---------------------------------------------------------------------------
constexpr int LM_GREG = LM_RED - LM_GBLK_MAX;  // doubles of the gradient region

RPH_INLINE void lm_store_sys_b128(double* p, double a, double b) {
  typedef unsigned lm_u4 __attribute__((ext_vector_type(4)));
  const unsigned long long ua = __double_as_longlong(a), ub = __double_as_longlong(b);
  const lm_u4 v = {(unsigned)ua, (unsigned)(ua >> 32), (unsigned)ub, (unsigned)(ub >> 32)};
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}

__global__ __launch_bounds__(256) void k_lm_dp_exchange_g(const LmDpDesc x, double* __restrict__ red, const int len) {
  __shared__ unsigned s_seq;
  const int tid = threadIdx.x, W = x.world, me = x.rank;
  if (tid == 0) s_seq = __hip_atomic_load(x.counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const unsigned seq = s_seq;
  const int slot = (int)(seq % DP_SLOTS);
  double* const g = red + LM_GBLK_MAX;
  constexpr int NPR = (LM_GREG / 2 + 255) / 256;  // pairs per thread
  double v0[NPR], v1[NPR];
#pragma unroll
  for (int r = 0; r < NPR; ++r) {
    const int e = 2 * (tid + 256 * r);
    v0[r] = v1[r] = 0.0;
    if (e < len) {
      v0[r] = g[e];
      v1[r] = g[e + 1];
      for (int q = 0; q < W; ++q)
        if (q != me) lm_store_sys_b128(x.mbox[q] + ((size_t)slot * W + me) * x.pitch + e, v0[r], v1[r]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its pushes
  __syncthreads();
  if (tid < W && tid != me) {
    unsigned* fo = reinterpret_cast<unsigned*>(x.mbox[tid] + ((size_t)slot * W + me) * x.pitch + LM_RED);
    __hip_atomic_store(fo, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* fi = reinterpret_cast<const unsigned*>(x.mbox[me] + ((size_t)slot * W + tid) * x.pitch + LM_RED);
    unsigned it = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(fi, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
      __builtin_amdgcn_s_sleep(1);
      if ((++it & 255u) == 0u && (__builtin_amdgcn_s_memrealtime() - t0 > DP_SPIN_TICKS ||
                                  __hip_atomic_load(x.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)) {
        __hip_atomic_store(x.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < NPR; ++r) {
    const int e = 2 * (tid + 256 * r);
    if (e >= len) continue;
    double s0 = 0.0, s1 = 0.0;
    for (int q = 0; q < W; ++q) {
      if (q == me) {
        s0 += v0[r];
        s1 += v1[r];
      } else {
        const double* m = x.mbox[me] + ((size_t)slot * W + q) * x.pitch + e;
        s0 += __hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s1 += __hip_atomic_load(m + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    g[e] = s0;
    g[e + 1] = s1;
  }
  if (tid == 0) __hip_atomic_store(x.counter, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// Multi-start selection of a first date (one workgroup).  The exploration
// fits (LmDesc.inst instances on a path prefix of every rank, LmDesc.explore)
// leave their final best loss, damping and best weights in their states.
//  phase 0 (pack): selection block of every candidate c = rank x inst + k:
//    this rank's instances from their states, zeros in the other ranks'
//    segments (summed over the ranks by the LM exchange = an all-gather);
//  phase 1 (pick): the candidate with the lowest final best loss (NaN counts
//    as +inf, ties go to the lowest index; every rank picks the same one):
//    its weights -> the canonical NetWeights (the polish fit's start point),
//    its damping -> main_state[LMS_LAM] (the polish fit carries it).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_lm_select(const TrainDesc d, const LmDesc lm, double* __restrict__ sel,
                                                   double* __restrict__ main_state, const int world, const int rank,
                                                   const int P, const int phase) {
  const int tid = threadIdx.x;
  const int K = lm.inst, NC = world * K;
  if (phase == 0) {
    for (int e = tid; e < NC * LM_SEL_W; e += 256) {
      const int c = e / LM_SEL_W, j = e % LM_SEL_W;
      double v = 0.0;
      if (c / K == rank) {
        const double* st = lm.state + (size_t)(c % K) * LMS_FLOATS;
        const int best = (int)st[LMS_BEST];
        v = j == 0 ? st[LMS_LFIN] : (j == 1 ? st[LMS_LAM] : (j - 2 < P ? st[LMS_W + best * LM_NPMAX + j - 2] : 0.0));
      }
      sel[e] = v;
    }
    return;
  }
  __shared__ int s_pick;
  if (tid < 64) {
    double l = tid < NC ? sel[(size_t)tid * LM_SEL_W] : INFINITY;
    if (!(l == l)) l = INFINITY;
    int idx = tid;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const double l2 = __shfl_xor(l, o, 64);
      const int i2 = __shfl_xor(idx, o, 64);
      if (l2 < l || (l2 == l && i2 < idx)) {
        l = l2;
        idx = i2;
      }
    }
    if (tid == 0) s_pick = idx < NC ? idx : 0;
  }
  __syncthreads();
  const double* c = sel + (size_t)s_pick * LM_SEL_W;
  for (int i = tid; i < P; i += 256) d.wts->w[0][i] = (float)c[2 + i];
  if (tid == 0) main_state[LMS_LAM] = c[1];
}

}  // namespace rph

using namespace rph;

extern "C" int rph_lm_select(const TrainDesc* d, const LmDesc* lm, double* sel, double* main_state, int world,
                             int rank, int P, int phase, void* stream) {
  if (!d || !lm || !sel || !main_state || !lm->state || !d->wts) return rph_report("rph_lm_select", "null pointer");
  if (world < 1 || rank < 0 || rank >= world || lm->inst < 1 || world * lm->inst > LM_SEL_MAX)
    return rph_report("rph_lm_select", "bad world / rank / instance count");
  if (P < 1 || P > LM_NPMAX || (phase != 0 && phase != 1)) return rph_report("rph_lm_select", "bad P / phase");
  hipLaunchKernelGGL(k_lm_select, dim3(1), dim3(256), 0, (hipStream_t)stream, *d, *lm, sel, main_state, world, rank,
                     P, phase);
  return (int)hipGetLastError();
}

extern "C" int rph_lm_dp_exchange(const LmDpDesc* x, double* red, int ng, int p, void* stream) {
  if (!x || !red || x->world < 2 || x->world > 8 || x->rank < 0 || x->rank >= x->world)
    return rph_report("rph_lm_dp_exchange", "bad world / rank");
  if (x->pitch < LM_RED + LM_DP_WGS || ng < 0 || ng > LM_GBLK_MAX || p < 1 || (ng > 0 && p > LM_NPMAX))
    return rph_report("rph_lm_dp_exchange", "bad mailbox pitch / block geometry");
  if ((x->pitch % 2) != 0) return rph_report("rph_lm_dp_exchange", "mailbox rows must be 16-byte aligned");
  for (int q = 0; q < x->world; ++q)
    if (!x->mbox[q]) return rph_report("rph_lm_dp_exchange", "null peer mailbox");
  if (ng == 0) {
    // no Gram entries: the first p doubles of the gradient region [g | stats |
    // output Gram] in one workgroup (16-byte pushes)
    if (p > LM_GREG || (p & 1)) return rph_report("rph_lm_dp_exchange", "bad gradient-region length");
    hipLaunchKernelGGL(k_lm_dp_exchange_g, dim3(1), dim3(256), 0, (hipStream_t)stream, *x, red, p);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(k_lm_dp_exchange, dim3(LM_DP_WGS), dim3(256), 0, (hipStream_t)stream, *x, red, ng, p);
  return (int)hipGetLastError();
}

#define RPH_LM_SHAPES(X)         \
  X(1, 8, 1, HEAD_COMPLEMENT)    \
  X(1, 8, 2, HEAD_FREE)          \
  X(2, 8, 2, HEAD_FREE)          \
  X(3, 8, 2, HEAD_FREE)          \
  X(4, 8, 2, HEAD_FREE)          \
  X(5, 8, 6, HEAD_FREE)          \
  X(6, 8, 7, HEAD_FREE)
// (6, 8, 7): P = 191, 78 tiles of the tile store = 156 KB of the CU's 160 KB
// (lm_chol.h); larger nets have no LM solver and fit with Adam
// (HipBackend.lm_supported() is False)

// Geometry of the LM kernels for a shape: returns 0 and fills (P, R, NBLK)
// or -1 for shapes without an LM solver.
extern "C" int rph_lm_shape(int nin, int h, int nout, int head, int* p, int* r, int* nblk) {
#define X(A, B, C, E)                                                    \
  if (shape_is(nin, h, nout, head, A, B, C, E)) {                        \
    using K = LmKernels<A, B, C, E>;                                     \
    *p = K::S::P;                                                        \
    *r = K::S::R;                                                        \
    *nblk = LmShape<K::S::P>::NBLK;                                      \
    return 0;                                                            \
  }
  RPH_LM_SHAPES(X)
#undef X
  return -1;
}

// Pass workgroups per CU the shape's plain pass body allows (1 or 2): the
// host sizes the pass grid up to 256 x that (engine.lm_pass_wgs).
extern "C" int rph_lm_pass_wps(int nin, int h, int nout, int head) {
#define X(A, B, C, E)                                        \
  if (shape_is(nin, h, nout, head, A, B, C, E)) {            \
    return LmKernels<A, B, C, E>::Body::WAVES_PER_SIMD;      \
  }
  RPH_LM_SHAPES(X)
#undef X
  return 1;
}

// The descriptor of one pass: the output-Gram pass body fits once per CU
// (80 KB of LDS), so where the plain passes run two workgroups per CU (more
// than 256: the cyclic schedule only) that pass takes 256 - one round of
// workgroups instead of two, and a 256-row output-Gram reduction
template <class K>
static LmDesc lm_pass_desc(const LmDesc& lm, const int pass) {
  LmDesc lp = lm;
  const bool og = lm.out_gram && pass > lm.passes - LM_OUTG_TAIL;
  if (og && K::BodyOG::WAVES_PER_SIMD == 1 && lm.leaf_blocks == 0 && lm.gram_base == 0 && lm.num_wgs > 256 &&
      pass == lm.passes)
    lp.num_wgs = 256;
  return lp;
}

// One pass = pass kernel + reduce kernel (into red_new); the caller all-reduces
// red_new when data parallel, then launches rph_lm_solve.
extern "C" int rph_lm_eval(const TrainDesc* d, const LmDesc* lm, double* red_new, int pass, void* stream) {
  hipStream_t s = (hipStream_t)stream;
#define X(A, B, C, E)                                                                           \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E)) {                                  \
    using K = LmKernels<A, B, C, E>;                                                            \
    if (int rc = lm_validate(d, lm, K::S::P, K::S::R, LmShape<K::S::P>::NBLK, K::Body::NU)) return rc; \
    const LmDesc lp = lm_pass_desc<K>(*lm, pass);                                               \
    if (int rc = lm_pass_launch<A, B, C, E>(d, &lp, pass, red_new, s)) return rc;               \
    const int ngw = lm_gram_red_wgs(LmShape<K::S::P>::NBLK * 1024, lp.gram_wgs);                \
    /* the final evaluation built no Gram: its reduce starts past the Gram workgroups */       \
    const int wg0 = pass == lp.passes ? ngw : 0;                                                \
    const int rg = ngw + lm_pk_red_wgs(K::S::R, lp.num_wgs, lp.dp_fused) + lm_og_wgs(K::Body::NU) - wg0; \
    hipLaunchKernelGGL((k_lm_reduce<K::S::P, K::S::R, K::Body::NU>), dim3(rg, lp.inst), dim3(1024), 0, s, \
                       lp, red_new, pass, wg0);                                                 \
    return (int)hipGetLastError();                                                              \
  }
  RPH_LM_SHAPES(X)
#undef X
  return rph_report("rph_lm_eval", "no LM solver for this network shape (8-unit nets only)");
}

extern "C" int rph_lm_solve(const TrainDesc* d, const LmDesc* lm, const double* red_new, int pass, void* stream) {
  hipStream_t s = (hipStream_t)stream;
#define X(A, B, C, E)                                                                                  \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E)) {                                         \
    using K = LmKernels<A, B, C, E>;                                                                   \
    const int bytes = K::smem();                                                                       \
    static bool attr = false;                                                                          \
    if (!attr) {                                                                                       \
      hipError_t e = hipFuncSetAttribute((const void*)k_lm_solve<K::S::P, K::S::R, K::Body::NU>,                   \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, bytes);           \
      if (e != hipSuccess) {                                                                           \
        (void)hipGetLastError(); /* do not leave the error for the next runtime call */                \
        return rph_report("rph_lm_solve", "dynamic LDS request refused");                              \
      }                                                                                                \
      attr = true;                                                                                     \
    }                                                                                                  \
    hipLaunchKernelGGL((k_lm_solve<K::S::P, K::S::R, K::Body::NU>), dim3(LM_SPEC, lm->inst), dim3(256), bytes, s, *d, *lm, \
                       red_new, pass);                                                                 \
    return (int)hipGetLastError();                                                                     \
  }
  RPH_LM_SHAPES(X)
#undef X
  return rph_report("rph_lm_solve", "no LM solver for this network shape");
}

// Whole single-rank fit: passes + 1 evaluations, each followed by a solve.
extern "C" int rph_lm_fit(const TrainDesc* d, const LmDesc* lm, double* red_new, void* stream) {
  for (int k = 0; k <= lm->passes; ++k) {
    if (int rc = rph_lm_eval(d, lm, red_new, k, stream)) return rc;
    if (int rc = rph_lm_solve(d, lm, red_new, k, stream)) return rc;
  }
  return 0;
}
