// rphedge — thread-per-path hedge-MLP training body for the reference's 8-unit
// nets (K8/K9), the ticketed step kernel with the fused Adam/early-stop update
// (K10), the minibatch chunk permutation (K11), the value/holdings/residual
// epilogue (K12) and the C ABI launchers of every training schedule, for gfx950.
//
// Reference semantics (one backward-induction date):
//   model(X1=[state_t, prices_{t+1}]) -> V = holdings(state_t) . prices_{t+1}
//   fit MSE / 99% pinball, Adam(1e-3), batch 512, EarlyStopping(loss)
//   (/root/reference/Replicating_Portfolio.py:149-221).
//
// Design (MI355X-first):
//   * NarrowBody: thread-per-path fp32 forward+backward (the compiler packs the
//     FMAs into v_pk_fma_f32); weights are wave-uniform, staged once in LDS and
//     either hoisted into registers or re-read as ds_read_b128 broadcasts
//     (variants); per-thread register accumulation of the full gradient
//     (R = next pow2 of P+4 floats), one in-wave recursive-halving
//     reduce-scatter (permlane32_swap / ds_swizzle / DPP), one LDS cross-wave sum;
//   * the same body runs under three schedules: k_hedge_step_lag (hedge_lag.h,
//     default above 64 workgroups: the update of step k-1 applied redundantly in
//     every workgroup's prologue, no in-kernel sync), k_hedge_fit (hedge_fit.h,
//     persistent per fit, default for small grids) and k_hedge_train_step below
//     (ticketed: the last-arriving workgroup sums the float-atomic replicas or
//     the deterministic slab, optionally exchanges the packet with the other
//     ranks over xGMI, and applies Keras-Adam + EarlyStopping in the same
//     launch; with an RCCL all-reduce instead, k_hedge_update applies it).
#include "hedge_core.h"
#include "hedge_fit.h"
#include "hedge_lag.h"
#include "hedge_narrow.h"

namespace rph {

// ---------------------------------------------------------------------------
// K9: one optimizer step.  Grid = num_wgs workgroups of 256 threads.
// ---------------------------------------------------------------------------
template <int NIN, int H, int NO, int HEAD>
__global__ __launch_bounds__(256) void k_hedge_train_step(const TrainDesc d, const int step, const int epoch,
                                                          const Perm perm) {
  using B = NarrowBody<NIN, H, NO, HEAD>;
  constexpr int R = B::R;
  constexpr int P = B::P;
  prefetch_kernarg<sizeof(TrainDesc) + 2 * sizeof(int) + sizeof(Perm)>();
  __shared__ __attribute__((aligned(16))) float lds[B::SCRATCH_FLOATS];
  __shared__ __attribute__((aligned(16))) float wl[P + 4];
  __shared__ int s_last;

  // prologue: every independent load is issued up front — early-stop flag,
  // weights, the optimizer state for a possible last-arriver update, and the
  // first path's data (epoch is a launch argument, so the permutation needs no
  // device read).
  RPH_DASSERT(d.batch > 0 && d.n_local >= d.batch && d.num_wgs == (int)gridDim.x);
  RPH_STAMP(0);
  const float stopped = d.fit->stopped;
  const float wv = threadIdx.x < P ? d.wts->w[0][threadIdx.x] : 0.f;
  UpdPre<P> up;
  if (d.fused_update) prefetch_update<P>(up, d.wts, d.opt, d.fit, d.lr_sched, epoch, step);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  typename B::Pre pre;
  pre.valid = false;
  if (B::first(wid) < d.batch) B::load(d, step, perm, B::first(wid), lane, pre);

  if (stopped != 0.f) return;  // early-stopped fit: remaining steps are no-ops
  // Weights are wave-uniform: stage them once in LDS and read them as
  // broadcast ds_read_b128 (keeps the 100+ weights out of the SGPR file).
  if (threadIdx.x < P) wl[threadIdx.x] = wv;
  if (d.fused_update) {  // keep the prefetch here (the compiler would sink it into the last-arriver branch)
    asm volatile("" ::"v"(up.m[0]), "v"(up.v[0]), "v"(up.w[0]), "v"(up.wbest[0]), "s"(up.t), "s"(up.lr), "s"(up.loss_sum),
                 "s"(up.wait), "s"(up.best_loss), "s"(up.lr_sched_e));
  }
  __syncthreads();
  RPH_STAMP(1);
  float vv[1];
  B::partial(d, step, perm, wl, typename B::Frags{}, lds, pre, vv);
  float val = vv[0];
  float* red = lds;  // reuse: red[t] for t < R after the hand-off below
  RPH_STAMP(3);

  if (gridDim.x > 1) {
    // ---- publish the partial write-through (sc1) / float-atomically, then draw
    // the arrival ticket.  No release/acquire fences: every handed-off byte is
    // stored sc1 (or added at the memory side) and every load of it by the last
    // arriver is an sc1 load (MI355X_MICROARCH visibility table, row 1).
    const int G = gridDim.x;
    if (threadIdx.x < R) {
      if (d.deterministic) st_agent(d.slab + (size_t)blockIdx.x * R + threadIdx.x, val);
      else __hip_atomic_fetch_add(d.acc + (blockIdx.x % ACC_REPLICAS) * R + threadIdx.x, val, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains
    __syncthreads();
    RPH_STAMP(4);
    if (threadIdx.x == 0) {
      const uint32_t ticket = __hip_atomic_fetch_add(d.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = (ticket == (uint32_t)G - 1u) ? 1 : 0;
    }
    __syncthreads();
    RPH_STAMP(5);
    if (!s_last) return;
    if (d.deterministic) {
      // fixed row partition + fixed combine order => bitwise reproducible
      constexpr int GROUPS = 256 / R;
      const int col = threadIdx.x % R;
      const int grp = threadIdx.x / R;
      float a = 0.f;
#pragma unroll 8
      for (int r = grp; r < G; r += GROUPS) a += ld_agent(d.slab + (size_t)r * R + col);
      lds[grp * R + col] = a;
      __syncthreads();
      if (threadIdx.x < R) {
        float s2 = 0.f;
        for (int gi = 0; gi < GROUPS; ++gi) s2 += lds[gi * R + threadIdx.x];
        val = s2;
      }
      __syncthreads();
    } else {
      if (threadIdx.x < R) {
        // all 8 replica loads in ONE asm statement with one wait (sc1: every load
        // of the handed-off bytes bypasses the non-coherent L1), then re-arm.
        float* a = d.acc + threadIdx.x;
        float r0, r1, r2, r3, r4, r5, r6, r7;
        if (R == 128) {
          asm volatile(
              "global_load_dword %0, %8, off sc1\n\t"
              "global_load_dword %1, %8, off offset:512 sc1\n\t"
              "global_load_dword %2, %8, off offset:1024 sc1\n\t"
              "global_load_dword %3, %8, off offset:1536 sc1\n\t"
              "global_load_dword %4, %8, off offset:2048 sc1\n\t"
              "global_load_dword %5, %8, off offset:2560 sc1\n\t"
              "global_load_dword %6, %8, off offset:3072 sc1\n\t"
              "global_load_dword %7, %8, off offset:3584 sc1\n\t"
              "s_waitcnt vmcnt(0)"
              : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7)
              : "v"(a)
              : "memory");
        } else {
          float* b = a + 4 * R;
          asm volatile(
              "global_load_dword %0, %8, off sc1\n\t"
              "global_load_dword %1, %8, off offset:1024 sc1\n\t"
              "global_load_dword %2, %8, off offset:2048 sc1\n\t"
              "global_load_dword %3, %8, off offset:3072 sc1\n\t"
              "global_load_dword %4, %9, off sc1\n\t"
              "global_load_dword %5, %9, off offset:1024 sc1\n\t"
              "global_load_dword %6, %9, off offset:2048 sc1\n\t"
              "global_load_dword %7, %9, off offset:3072 sc1\n\t"
              "s_waitcnt vmcnt(0)"
              : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7)
              : "v"(a), "v"(b)
              : "memory");
        }
        val = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
#pragma unroll
        for (int rp = 0; rp < ACC_REPLICAS; ++rp) st_agent(a + rp * R, 0.f);  // re-arm (completes by kernel end)
      }
    }
    if (threadIdx.x == 0) __hip_atomic_store(d.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x < R) red[threadIdx.x] = val;
  __syncthreads();
  RPH_STAMP(6);

  if (d.dp_world > 1) {
    dp_allreduce<R>(d, red);
    RPH_STAMP(7);
  }
  if (d.fused_update) {
    apply_update<P>(red, up, d.wts, d.opt, d.fit, epoch, step, d.steps_per_epoch);
  } else if (threadIdx.x < R) {
    d.grad_out[threadIdx.x] = red[threadIdx.x];
  }
  if (d.dp_world <= 1) RPH_STAMP(7);
}

// ---------------------------------------------------------------------------
// K12: value / holdings / residual epilogue of a backward-induction date.
//   V_t       = h(state_t) . p_t           (Keras predict(X0), RP:212)
//   blend     = g + c (h - g)              (RP:221)
//   residual  = V_{t+1} - h . p_{t+1}       ("VaR", RP:120; Q24)
// Per-workgroup fp64 statistics go to a [num_wgs][EVAL_NSTAT] slab.
// ---------------------------------------------------------------------------
// PA: the traded-asset prices at t ARE the leading features (GBM / basket:
// same tensors, detected by pointer on the host) - loaded once per path.
template <int NIN, int H, int NO, int HEAD, bool PA>
__global__ __launch_bounds__(256) void k_hedge_eval(const EvalDesc d) {
  using S = NetShape<NIN, H, NO, HEAD>;
  constexpr int NHOLD = S::NHOLD;
  static_assert(!PA || NIN >= NHOLD - 1, "price alias needs a feature per traded asset");
  prefetch_kernarg<sizeof(EvalDesc)>();
  RPH_DASSERT(d.n_local > 0 && d.num_wgs == (int)gridDim.x && d.wa != nullptr && d.stats != nullptr);
  __shared__ double sst[4][EVAL_NSTAT];
  constexpr int WBOFF = (S::P + 3) / 4 * 4;  // net B's weights 16-byte aligned (ds_read_b128)
  __shared__ __attribute__((aligned(16))) float wl[WBOFF + S::P + 4];
  const bool has_b = d.wb != nullptr;
  for (int i = threadIdx.x; i < S::P; i += 256) {
    wl[i] = d.wa->w[0][i];
    if (has_b) wl[WBOFF + i] = d.wb->w[0][i];
  }
  __syncthreads();
  if (blockIdx.x == 0) {  // per-date weight snapshots (saved-model format, P&L scan)
    for (int i = threadIdx.x; i < S::P; i += 256) {
      if (d.snap_a) d.snap_a->w[0][i] = wl[i];
      if (d.snap_b) d.snap_b->w[0][i] = has_b ? wl[WBOFF + i] : wl[i];
    }
  }
  const float* __restrict__ WA = wl;
  const float* __restrict__ WB = has_b ? wl + WBOFF : wl;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;

  // per-thread fp32 partials (a thread sees only a handful of paths), one
  // in-wave reduce-scatter, fp64 only across waves / workgroups
  constexpr int NS = 64;
  float st[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) st[i] = 0.f;
  float rmin = INFINITY, rmax = -INFINITY;

  // Inputs of one path; a ring of EPF of them is kept in flight so every
  // iteration's loads were issued EPF-1 iterations earlier (a thread walks
  // n_local / (256 * num_wgs) paths, typically 16: one resident wave per SIMD
  // would otherwise wait a full memory round trip per path).
  struct In {
    float x[NIN], pt[NHOLD], pt1[NHOLD], tgt, gb;
    int p;
    bool valid;
  };
  constexpr int EPF = 4;
  const int stride = (int)gridDim.x * 256;
  const bool has1 = d.price_t1[0] != nullptr;
  auto load_in = [&](int p, In& in) {
    in.p = p;
    in.valid = p < d.n_local;
    const int pp = in.valid ? p : 0;
#pragma unroll
    for (int f = 0; f < NIN; ++f) in.x[f] = d.feat[f][pp];  // raw (ring): standardised where consumed
#pragma unroll
    for (int k = 0; k < NHOLD - 1; ++k) {
      if constexpr (PA) in.pt[k] = in.x[PA ? k : 0];  // (raw feature = raw price)
      else in.pt[k] = d.price_t[k][pp];
      in.pt1[k] = has1 ? d.price_t1[k][pp] : 0.f;
    }
    in.tgt = (has1 && d.target) ? d.target[pp] : 0.f;
    in.gb = d.g_base ? d.g_base[pp] : 0.f;
  };
  In q[EPF];
  const int p_first = blockIdx.x * 256 + threadIdx.x;
#pragma unroll
  for (int i = 0; i < EPF; ++i) load_in(p_first + i * stride, q[i]);

  for (int p0 = blockIdx.x * 256; p0 < d.n_local; p0 += stride) {
    const In cur = q[0];
#pragma unroll
    for (int i = 0; i + 1 < EPF; ++i) q[i] = q[i + 1];
    if (p0 + EPF * stride < d.n_local) load_in(cur.p + EPF * stride, q[EPF - 1]);
    const int p = cur.p;
    const bool valid = cur.valid;
    // opaque zero offset: the weights stay in LDS and are read as broadcasts
    // every iteration instead of being hoisted into (and spilling out of) VGPRs
    uint32_t zo = 0;
    asm volatile("" : "+v"(zo));
    const float* __restrict__ WAi = (const float*)__builtin_assume_aligned(WA + (zo & ~3u), 16);
    const float* __restrict__ WBi = (const float*)__builtin_assume_aligned(WB + (zo & ~3u), 16);
    float z1[H], a1[H], z2[H], a2[H], hold[NHOLD], holdv[NHOLD], xn[NIN];
#pragma unroll
    for (int f = 0; f < NIN; ++f) xn[f] = (cur.x[f] - d.fmu[f]) * d.fisd[f];
    net_forward<NIN, H, NO, HEAD>(WAi, xn, d.alpha, z1, a1, z2, a2, hold);
#pragma unroll
    for (int k = 0; k < NHOLD; ++k) holdv[k] = hold[k];
    if (has_b) {
      // V_t comes from net B (model2.predict, RP:218); reported holdings are
      // the blend hA + hold_c (hB - hA) (get_phi_psi_VaR, RP:114-115).
      net_forward<NIN, H, NO, HEAD>(WBi, xn, d.alpha, z1, a1, z2, a2, holdv);
#pragma unroll
      for (int k = 0; k < NHOLD; ++k) hold[k] = hold[k] + d.hold_c * (holdv[k] - hold[k]);
    }
    float V = 0.f;
#pragma unroll
    for (int k = 0; k < NHOLD - 1; ++k) V = fmaf(holdv[k], cur.pt[k], V);
    V = fmaf(holdv[NHOLD - 1], d.bond_t, V);
    if (d.g_base) V = cur.gb + d.blend_c * (V - cur.gb);
    float res = 0.f, pred1 = 0.f;
    const float tgt = cur.tgt;
    if (has1) {
#pragma unroll
      for (int k = 0; k < NHOLD - 1; ++k) pred1 = fmaf(hold[k], cur.pt1[k], pred1);
      pred1 = fmaf(hold[NHOLD - 1], d.bond_t1, pred1);
      if (d.target) res = tgt - pred1;
    }
    if (valid) {
      if (d.v_out) d.v_out[p] = V;
#pragma unroll
      for (int k = 0; k < NHOLD; ++k)
        if (d.hold_out[k]) d.hold_out[k][p] = hold[k];
      if (d.resid_out) d.resid_out[p] = res;
      if (d.pred1_out) d.pred1_out[p] = pred1;
      st[ES_V] += V;
      st[ES_V2] += V * V;
      st[ES_RES] += res;
      st[ES_RES2] += res * res;
      st[ES_ABSRES] += fabsf(res);
      st[ES_APE] += d.target ? fabsf(res) * __frcp_rn(fmaxf(fabsf(tgt), 1e-7f)) : 0.f;
      st[ES_PRED1] += pred1;
      st[ES_COUNT] += 1.f;
#pragma unroll
      for (int k = 0; k < NHOLD; ++k) {
        st[ES_HOLD + k] += hold[k];
        st[ES_HOLD2 + k] += hold[k] * hold[k];
      }
      rmin = fminf(rmin, res);
      rmax = fmaxf(rmax, res);
    }
  }
  wave_reduce_scatter<NS>(st, lane);  // lane L now holds the wave total of stat L
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    rmin = fminf(rmin, __shfl_xor(rmin, o, 64));
    rmax = fmaxf(rmax, __shfl_xor(rmax, o, 64));
  }
  if (lane < EVAL_NSTAT) sst[wid][lane] = (double)st[0];
  if (lane == 0) {
    sst[wid][ES_RESMIN] = rmin;
    sst[wid][ES_RESMAX] = rmax;
  }
  __syncthreads();
  if (threadIdx.x < EVAL_NSTAT) {
    const int i = threadIdx.x;
    double v;
    if (i == ES_RESMIN) v = fmin(fmin(sst[0][i], sst[1][i]), fmin(sst[2][i], sst[3][i]));
    else if (i == ES_RESMAX) v = fmax(fmax(sst[0][i], sst[1][i]), fmax(sst[2][i], sst[3][i]));
    else v = sst[0][i] + sst[1][i] + sst[2][i] + sst[3][i];
    d.stats[(size_t)blockIdx.x * EVAL_NSTAT + i] = v;
  }
}

// ---------------------------------------------------------------------------
// Self-financing hedge P&L scan (PnlDesc, rph_types.h): one thread per path
// (PPT paths per thread), dates in lockstep per workgroup so each date's
// network(s) are staged once in LDS; the path inputs run one date ahead.  Wealth starts at V_0, holds the traded-
// asset holdings of date t's network and keeps the remainder in the bank
// account; P&L_T = W_T - liability.  Per-workgroup fp64 statistics in the
// eval-stats layout (ES_V = W_T, ES_RES = P&L).  Not a hot path (one pass per
// run, a few hundred VALU flops per path and date); the corrected counterpart
// of the reference's one-step "P&L" (Q24, Replicating_Portfolio.py:120).
// ---------------------------------------------------------------------------
constexpr int PNL_PPT = 4;

template <int NIN, int H, int NO, int HEAD>
__global__ __launch_bounds__(256) void k_hedge_pnl(const PnlDesc d) {
  using S = NetShape<NIN, H, NO, HEAD>;
  constexpr int NHOLD = S::NHOLD;
  constexpr int NA = NHOLD - 1;  // traded assets (the last holding is the bank account)
  constexpr int WBOFF = (S::P + 3) / 4 * 4;
  prefetch_kernarg<sizeof(PnlDesc)>();
  RPH_DASSERT(d.n_local > 0 && d.num_wgs == (int)gridDim.x && d.snap != nullptr && d.stats != nullptr);
  __shared__ __attribute__((aligned(16))) float wl[WBOFF + S::P + 4];
  __shared__ double sred[4][8];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const long long base = (long long)blockIdx.x * 256 * PNL_PPT + tid;
  const bool has_b = d.has_b != 0;
  // per path: wealth, the traded prices at the current date (carried to the
  // next date: each price row is loaded once) and the next date's inputs,
  // all loads of a date issued together before any compute
  float wealth[PNL_PPT], s_cur[PNL_PPT][NA > 0 ? NA : 1];
  long long pidx[PNL_PPT];
#pragma unroll
  for (int j = 0; j < PNL_PPT; ++j) {
    const long long p = base + (long long)j * 256;
    const bool ok = p < d.n_local;
    pidx[j] = ok ? p : 0;  // invalid paths compute on path 0 and are never stored
    wealth[j] = ok ? (d.w0 ? d.w0[p] : d.wealth0) : 0.f;
#pragma unroll
    for (int a = 0; a < NA; ++a) s_cur[j][a] = d.price[a][pidx[j]];
  }
  // date t's inputs are loaded one date ahead (software pipeline): their
  // latency hides under date t-1's network evaluation
  float xr[PNL_PPT][NIN], s_nxt[PNL_PPT][NA > 0 ? NA : 1];
  auto load_date = [&](int t) {
#pragma unroll
    for (int j = 0; j < PNL_PPT; ++j) {
#pragma unroll
      for (int f = 0; f < NIN; ++f) xr[j][f] = d.feat[f][(long long)t * d.feat_ts[f] + pidx[j]];
#pragma unroll
      for (int a = 0; a < NA; ++a) s_nxt[j][a] = d.price[a][(long long)(t + 1) * d.price_ts[a] + pidx[j]];
    }
  };
  if (d.n_dates > 0) load_date(0);
  for (int t = 0; t < d.n_dates; ++t) {
    float xc[PNL_PPT][NIN], sc_nxt[PNL_PPT][NA > 0 ? NA : 1];
#pragma unroll
    for (int j = 0; j < PNL_PPT; ++j) {
#pragma unroll
      for (int f = 0; f < NIN; ++f) xc[j][f] = xr[j][f];
#pragma unroll
      for (int a = 0; a < NA; ++a) sc_nxt[j][a] = s_nxt[j][a];
    }
    if (t + 1 < d.n_dates) load_date(t + 1);
    __syncthreads();  // every thread is done with date t-1's weights
    const NetWeights* wt = d.snap + (size_t)t * 2;
    for (int i = tid; i < S::P; i += 256) {
      wl[i] = wt[0].w[0][i];
      if (has_b) wl[WBOFF + i] = wt[1].w[0][i];
    }
    float mu[NIN], isd[NIN];
#pragma unroll
    for (int f = 0; f < NIN; ++f) {
      mu[f] = d.fmu[t * MAXIN + f];
      isd[f] = d.fisd[t * MAXIN + f];
    }
    const float grow = (float)(d.bond[t + 1] / d.bond[t]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PNL_PPT; ++j) {
      uint32_t zo = 0;  // opaque zero: weights stay in LDS (broadcast reads), not hoisted into VGPRs
      asm volatile("" : "+v"(zo));
      const float* __restrict__ WA = (const float*)__builtin_assume_aligned(wl + (zo & ~3u), 16);
      const float* __restrict__ WB = (const float*)__builtin_assume_aligned(wl + WBOFF + (zo & ~3u), 16);
      float x[NIN];
#pragma unroll
      for (int f = 0; f < NIN; ++f) x[f] = (xc[j][f] - mu[f]) * isd[f];
      float z1[H], a1[H], z2[H], a2[H], hold[NHOLD], hb[NHOLD];
      net_forward<NIN, H, NO, HEAD>(WA, x, d.alpha, z1, a1, z2, a2, hold);
      if (has_b) {
        net_forward<NIN, H, NO, HEAD>(WB, x, d.alpha, z1, a1, z2, a2, hb);
#pragma unroll
        for (int k = 0; k < NHOLD; ++k) hold[k] = hold[k] + d.hold_c * (hb[k] - hold[k]);
      }
      float w = wealth[j] * grow;
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        w = fmaf(hold[a], sc_nxt[j][a] - s_cur[j][a] * grow, w);
        s_cur[j][a] = sc_nxt[j][a];
      }
      wealth[j] = w;
    }
  }
  // P&L and per-workgroup fp64 statistics
  double sv = 0, sv2 = 0, sp = 0, sp2 = 0, sa = 0, cnt = 0;
  float pmin = INFINITY, pmax = -INFINITY;
#pragma unroll
  for (int j = 0; j < PNL_PPT; ++j) {
    const long long p = base + (long long)j * 256;
    if (p >= d.n_local) continue;
    const float pnl = wealth[j] - d.payoff[p];
    if (d.pnl_out) d.pnl_out[p] = pnl;
    sv += wealth[j];
    sv2 += (double)wealth[j] * wealth[j];
    sp += pnl;
    sp2 += (double)pnl * pnl;
    sa += fabsf(pnl);
    cnt += 1.0;
    pmin = fminf(pmin, pnl);
    pmax = fmaxf(pmax, pnl);
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    sv += __shfl_xor(sv, o, 64);
    sv2 += __shfl_xor(sv2, o, 64);
    sp += __shfl_xor(sp, o, 64);
    sp2 += __shfl_xor(sp2, o, 64);
    sa += __shfl_xor(sa, o, 64);
    cnt += __shfl_xor(cnt, o, 64);
    pmin = fminf(pmin, __shfl_xor(pmin, o, 64));
    pmax = fmaxf(pmax, __shfl_xor(pmax, o, 64));
  }
  if (lane == 0) {
    sred[wid][0] = sv; sred[wid][1] = sv2; sred[wid][2] = sp; sred[wid][3] = sp2;
    sred[wid][4] = sa; sred[wid][5] = cnt; sred[wid][6] = pmin; sred[wid][7] = pmax;
  }
  __syncthreads();
  if (tid < EVAL_NSTAT) {
    double v = 0.0;
    auto sum4 = [&](int k) { return (sred[0][k] + sred[1][k]) + (sred[2][k] + sred[3][k]); };
    if (tid == ES_V) v = sum4(0);
    else if (tid == ES_V2) v = sum4(1);
    else if (tid == ES_RES) v = sum4(2);
    else if (tid == ES_RES2) v = sum4(3);
    else if (tid == ES_ABSRES) v = sum4(4);
    else if (tid == ES_COUNT) v = sum4(5);
    else if (tid == ES_RESMIN) v = fmin(fmin(sred[0][6], sred[1][6]), fmin(sred[2][6], sred[3][6]));
    else if (tid == ES_RESMAX) v = fmax(fmax(sred[0][7], sred[1][7]), fmax(sred[2][7], sred[3][7]));
    d.stats[(size_t)blockIdx.x * EVAL_NSTAT + tid] = v;
  }
}

}  // namespace rph

// ---------------------------------------------------------------------------
// Host dispatch over the supported network shapes.
// ---------------------------------------------------------------------------
using namespace rph;

#define RPH_SHAPES(X)            \
  X(1, 8, 1, HEAD_COMPLEMENT)    \
  X(1, 8, 2, HEAD_FREE)          \
  X(2, 8, 2, HEAD_FREE)          \
  X(3, 8, 2, HEAD_FREE)          \
  X(4, 8, 2, HEAD_FREE)          \
  X(5, 8, 6, HEAD_FREE)          \
  X(6, 8, 7, HEAD_FREE)


extern "C" int rph_net_nparams(int nin, int h, int nout, int head, int* p_out, int* r_out) {
#define X(A, B, C, E)                                  \
  if (shape_is(nin, h, nout, head, A, B, C, E)) {      \
    *p_out = NetShape<A, B, C, E>::P;                  \
    *r_out = NetShape<A, B, C, E>::R;                  \
    return 0;                                          \
  }
  RPH_SHAPES(X)
  RPH_WIDE_SHAPES(X)
#undef X
  return -1;
}

extern "C" int rph_train_step(const TrainDesc* d, int step, int epoch, void* stream) {
  if (int rc = validate_train(d, 0, "rph_train_step")) return rc;
  hipStream_t s = (hipStream_t)stream;
  const uint32_t n_chunks = (uint32_t)((d->n_local + (1 << d->chunk_log2) - 1) >> d->chunk_log2);
  const Perm perm = make_perm(n_chunks, d->seed, (uint32_t)epoch, d->shuffle != 0);
#define X(A, B, C, E)                                                                        \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E)) {                               \
    hipLaunchKernelGGL((k_hedge_train_step<A, B, C, E>), dim3(d->num_wgs), dim3(256), 0, s, *d, step, epoch, perm); \
    return (int)hipGetLastError();                                                           \
  }
  RPH_SHAPES(X)
#undef X
  return launch_wide_step(d, step, epoch, perm, s);
}

// One launch per Keras fit() (persistent kernel, hedge_fit.h); world_size 1.
extern "C" int rph_train_fit(const TrainDesc* d, int epochs, void* stream) {
  if (int rc = validate_train(d, 2, "rph_train_fit")) return rc;
  hipStream_t s = (hipStream_t)stream;
#define X(A, B, C, E)                                                \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E))         \
    return launch_fit<NarrowBody<A, B, C, E>>(d, epochs, s);
  RPH_SHAPES(X)
#undef X
  return launch_wide_fit(d, epochs, s);
}

// Lagged-update step kernel k of a fit (hedge_lag.h) and its finalize.
extern "C" int rph_train_lag_step(const TrainDesc* d, int k, int epoch, void* stream) {
  if (int rc = validate_train(d, 1, "rph_train_lag_step")) return rc;
  hipStream_t s = (hipStream_t)stream;
  const uint32_t n_chunks = (uint32_t)((d->n_local + (1 << d->chunk_log2) - 1) >> d->chunk_log2);
  const Perm perm = make_perm(n_chunks, d->seed, (uint32_t)epoch, d->shuffle != 0);
#define X(A, B, C, E)                                                                                 \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E)) {                                        \
    switch (d->variant) {                                                                             \
      case 1: hipLaunchKernelGGL((k_hedge_step_lag<NarrowBody<A, B, C, E, 2>>), dim3(d->num_wgs), dim3(256), 0, s, \
                                 *d, k, epoch, perm); break;                                           \
      case 2: hipLaunchKernelGGL((k_hedge_step_lag<NarrowBody<A, B, C, E, 1, 3>>), dim3(d->num_wgs), dim3(256), 0, \
                                 s, *d, k, epoch, perm); break;                                        \
      case 3: hipLaunchKernelGGL((k_hedge_step_lag<NarrowBody<A, B, C, E, 2, 3>>), dim3(d->num_wgs), dim3(256), 0, \
                                 s, *d, k, epoch, perm); break;                                        \
      case 4: hipLaunchKernelGGL((k_hedge_step_lag<NarrowBody<A, B, C, E, 1, 1, true>>), dim3(d->num_wgs), dim3(256), \
                                 0, s, *d, k, epoch, perm); break;                                     \
      case 5: hipLaunchKernelGGL((k_hedge_step_lag<NarrowBody<A, B, C, E, 1, 1, false, true>>), dim3(d->num_wgs), \
                                 dim3(256), 0, s, *d, k, epoch, perm); break;                          \
      default: hipLaunchKernelGGL((k_hedge_step_lag<NarrowBody<A, B, C, E>>), dim3(d->num_wgs), dim3(256), 0, s, \
                                  *d, k, epoch, perm);                                                 \
    }                                                                                                 \
    return (int)hipGetLastError();                                                                    \
  }
  RPH_SHAPES(X)
#undef X
  return launch_wide_lag_step(d, k, epoch, perm, s);
}

extern "C" int rph_train_lag_finalize(const TrainDesc* d, int K, void* stream);

extern "C" int rph_train_lag_finalize(const TrainDesc* d, int K, void* stream) {
  if (int rc = validate_train(d, 1, "rph_train_lag_finalize")) return rc;
  hipStream_t s = (hipStream_t)stream;
#define X(A, B, C, E)                                                                        \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E)) {                               \
    using S = NetShape<A, B, C, E>;                                                          \
    hipLaunchKernelGGL((k_hedge_lag_finalize<S::P, S::R, NARROW_NREP>), dim3(1), dim3(256), 0, s, *d, K); \
    return (int)hipGetLastError();                                                           \
  }
  RPH_SHAPES(X)
#undef X
#define X(A, B, C, E)                                                                        \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E)) {                               \
    using S = NetShape<A, B, C, E>;                                                          \
    hipLaunchKernelGGL((k_hedge_lag_finalize<S::P, S::R, WIDE_NREP>), dim3(1), dim3(256), 0, s, *d, K); \
    return (int)hipGetLastError();                                                           \
  }
  RPH_WIDE_SHAPES(X)
#undef X
  return -1;
}

// Whole fit on the host side of the native runtime: the epochs x steps launch
// loop (lagged schedule, or ticketed steps with fused update) runs in C++ so an
// eager (non-graph) fit pays one hipLaunchKernel per step instead of a Python
// + ctypes round trip per step.  Graph capture records the same launches.
extern "C" int rph_train_lag_fit(const TrainDesc* d, int epochs, void* stream) {
  if (int rc = validate_train(d, 1, "rph_train_lag_fit")) return rc;
  int k = 0;
  for (int e = 0; e < epochs; ++e)
    for (int s = 0; s < d->steps_per_epoch; ++s, ++k)
      if (int rc = rph_train_lag_step(d, k, e, stream)) return rc;
  return rph_train_lag_finalize(d, k, stream);
}

extern "C" int rph_train_ticket_fit(const TrainDesc* d, int epochs, void* stream) {
  if (int rc = validate_train(d, 0, "rph_train_ticket_fit")) return rc;
  if (!d->fused_update) return rph_report("rph_train_ticket_fit", "needs the fused (in-kernel) update");
  for (int e = 0; e < epochs; ++e)
    for (int s = 0; s < d->steps_per_epoch; ++s)
      if (int rc = rph_train_step(d, s, e, stream)) return rc;
  return 0;
}


extern "C" int rph_train_update(const TrainDesc* d, int step, int epoch, void* stream) {
  if (!d->grad_out || !d->wts || !d->opt || !d->fit) return rph_report("rph_train_update", "null pointer");
  hipStream_t s = (hipStream_t)stream;
#define X(A, B, C, E)                                                                        \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E)) {                               \
    using S = NetShape<A, B, C, E>;                                                          \
    hipLaunchKernelGGL((k_hedge_update<S::P, S::R>), dim3(1), dim3(256), 0, s, *d, step, epoch); \
    return (int)hipGetLastError();                                                           \
  }
  RPH_SHAPES(X)
  RPH_WIDE_SHAPES(X)
#undef X
  return -1;
}

extern "C" int rph_eval(const EvalDesc* d, void* stream) {
  if (!d->wa || !d->stats || d->n_local < 1 || d->num_wgs < 1 || d->nin < 1 || d->nin > MAXIN)
    return rph_report("rph_eval", "bad eval descriptor");
  if (!(d->alpha >= 0.f && d->alpha <= 1.f)) return rph_report("rph_eval", "LeakyReLU slope must be in [0, 1]");
  for (int f = 0; f < d->nin; ++f)
    if (!(d->fisd[f] > 0.f && d->fisd[f] < 3.0e38f && d->fmu[f] == d->fmu[f]))
      return rph_report("rph_eval", "feature standardisation must be finite with fisd > 0");
  for (int f = 0; f < d->nin; ++f)
    if (!d->feat[f]) return rph_report("rph_eval", "null feature pointer");
  hipStream_t s = (hipStream_t)stream;
  const int nhold = d->head == HEAD_COMPLEMENT ? 2 : d->nout;
  bool alias = d->nin >= nhold - 1;
  for (int k = 0; alias && k < nhold - 1; ++k) alias = d->price_t[k] == d->feat[k];
#define X(A, B, C, E)                                                                          \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E)) {                                 \
    if constexpr (A >= NetShape<A, B, C, E>::NHOLD - 1) {                                     \
      if (alias) {                                                                             \
        hipLaunchKernelGGL((k_hedge_eval<A, B, C, E, true>), dim3(d->num_wgs), dim3(256), 0, s, *d); \
        return (int)hipGetLastError();                                                         \
      }                                                                                        \
    }                                                                                          \
    hipLaunchKernelGGL((k_hedge_eval<A, B, C, E, false>), dim3(d->num_wgs), dim3(256), 0, s, *d); \
    return (int)hipGetLastError();                                                             \
  }
  RPH_SHAPES(X)
  RPH_WIDE_SHAPES(X)
#undef X
  return -1;
}

extern "C" int rph_pnl(const PnlDesc* d, void* stream) {
  const int nhold = d->head == HEAD_COMPLEMENT ? 2 : d->nout;
  if (!d->snap || !d->stats || !d->payoff || !d->fmu || !d->fisd || !d->bond || d->n_local < 1 || d->n_dates < 1 ||
      d->nin < 1 || d->nin > MAXIN || nhold < 2 || nhold > MAXHOLD)
    return rph_report("rph_pnl", "bad P&L descriptor");
  if (!(d->alpha >= 0.f && d->alpha <= 1.f)) return rph_report("rph_pnl", "LeakyReLU slope must be in [0, 1]");
  for (int f = 0; f < d->nin; ++f)
    if (!d->feat[f] || d->feat_ts[f] < 0) return rph_report("rph_pnl", "null feature pointer / negative stride");
  for (int k = 0; k < nhold - 1; ++k)
    if (!d->price[k] || d->price_ts[k] < d->n_local) return rph_report("rph_pnl", "null price pointer / bad stride");
  const long long per_wg = 256LL * PNL_PPT;
  if ((long long)d->num_wgs * per_wg < d->n_local || (long long)(d->num_wgs - 1) * per_wg >= d->n_local)
    return rph_report("rph_pnl", "num_wgs does not match n_local / (256 * PNL_PPT)");
  hipStream_t s = (hipStream_t)stream;
#define X(A, B, C, E)                                                                          \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E)) {                                 \
    hipLaunchKernelGGL((k_hedge_pnl<A, B, C, E>), dim3(d->num_wgs), dim3(256), 0, s, *d);     \
    return (int)hipGetLastError();                                                             \
  }
  RPH_SHAPES(X)
  RPH_WIDE_SHAPES(X)
#undef X
  return -1;
}
