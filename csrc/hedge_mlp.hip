// rphedge — fused hedge-MLP training step (K9), Adam/early-stop update (K10),
// minibatch chunk permutation (K11) and the value/holdings/residual epilogue
// (K12) for gfx950.
//
// Reference semantics (one backward-induction date):
//   model(X1=[state_t, prices_{t+1}]) -> V = holdings(state_t) . prices_{t+1}
//   fit MSE / 99% pinball, Adam(1e-3), batch 512, EarlyStopping(loss)
//   (/root/reference/Replicating_Portfolio.py:149-221).
//
// Design (MI355X-first):
//   * thread-per-path fp32 forward+backward; weights are wave-uniform and are
//     read through the scalar unit (s_load -> SGPR operands of v_fma);
//   * per-thread register accumulation of the full gradient (R = next pow2 of
//     P+4 floats), one in-wave recursive-halving reduce-scatter (DPP/swizzle,
//     ~4R VALU), one LDS cross-wave sum, one deterministic [num_wgs][R] slab;
//   * the last-arriving workgroup (agent-scope release/acquire ticket) sums
//     the slab and — for world_size == 1 — applies Keras-Adam, the epoch-end
//     EarlyStopping/LR-schedule bookkeeping and the weight ping-pong in the
//     same launch: ONE kernel per optimizer step, graph-capturable.
//   * world_size > 1: the slab sum goes to grad_out, RCCL all-reduces it on
//     the same stream and k_hedge_update applies the identical update on every
//     rank (bitwise-identical decisions => identical early stopping).
#include "rph_common.h"
#include "rph_types.h"

namespace rph {

// Diagnostic phase stamps (s_memrealtime, 100 MHz): thread 0 of every
// workgroup writes stamp k to d.stamps[blockIdx.x * 8 + k] when d.stamps is set.
#define RPH_STAMP(k)                                                                    \
  do {                                                                                  \
    if (d.stamps != nullptr && threadIdx.x == 0)                                        \
      d.stamps[(size_t)blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();        \
  } while (0)

template <int NIN, int H, int NO, int HEAD>
struct NetShape {
  static constexpr int NHOLD = (HEAD == HEAD_COMPLEMENT) ? 2 : NO;
  static constexpr int OW1 = 0;
  static constexpr int OB1 = OW1 + NIN * H;
  static constexpr int OW2 = OB1 + H;
  static constexpr int OB2 = OW2 + H * H;
  static constexpr int OW3 = OB2 + H;
  static constexpr int OB3 = OW3 + H * NO;
  static constexpr int P = OB3 + NO;
  static constexpr int NSTAT = 4;  // loss, |e|, |e|/|y|, count
  static constexpr int R = (P + NSTAT <= 128) ? 128 : 256;
  static_assert(P <= PMAX, "network too large for PMAX");
  static_assert(NHOLD <= MAXHOLD, "too many holdings");
};

// ---------------------------------------------------------------------------
// K11: bijective chunk permutation for Keras-style per-epoch shuffling.  Paths
// are permuted in chunks of 2^chunk_log2 (64 => one coalesced wave load); the
// permutation is a keyed affine/xorshift bijection on the next power of two
// with cycle-walking, so nothing is materialised.
// ---------------------------------------------------------------------------
struct Perm {
  uint32_t mask, n, k1, a1, b1, a2, b2, sh;
  int on;
  RPH_INLINE uint32_t f(uint32_t x) const {
    x = (((x ^ k1) * a1) + b1) & mask;
    x ^= x >> sh;
    x = ((x * a2) + b2) & mask;
    return x;
  }
  RPH_INLINE uint32_t operator()(uint32_t x) const {
    if (!on) return x;
    x = f(x);
    while (x >= n) x = f(x);
    return x;
  }
};

__host__ __device__ inline Perm make_perm(uint32_t n_chunks, uint32_t seed, uint32_t epoch, bool on) {
  Perm p;
  uint32_t m = 1;
  int bits = 0;
  while (m < n_chunks) { m <<= 1; ++bits; }
  p.mask = m - 1u;
  p.n = n_chunks;
  const u32x4 r = philox4x32_10({epoch, 0x5eedu, 0u, 0u}, seed, 0xC0FFEEu);
  const u32x4 s = philox4x32_10({epoch, 0x5eedu, 1u, 0u}, seed, 0xC0FFEEu);
  p.k1 = r.x & p.mask;
  p.a1 = (r.y | 1u);
  p.b1 = r.z;
  p.a2 = (r.w | 1u);
  p.b2 = s.x;
  p.sh = bits > 1 ? (uint32_t)(bits / 2) : 1u;
  p.on = (on && n_chunks > 1) ? 1 : 0;
  return p;
}

// ---------------------------------------------------------------------------
// Forward pass of one path (fp32).  W is wave-uniform.
// ---------------------------------------------------------------------------
template <int NIN, int H, int NO, int HEAD>
RPH_INLINE void net_forward(const float* __restrict__ W, const float (&x)[NIN], float alpha,
                            float (&z1)[H], float (&a1)[H], float (&z2)[H], float (&a2)[H],
                            float (&hold)[NetShape<NIN, H, NO, HEAD>::NHOLD]) {
  using S = NetShape<NIN, H, NO, HEAD>;
#pragma unroll
  for (int j = 0; j < H; ++j) {
    float acc = W[S::OB1 + j];
#pragma unroll
    for (int f = 0; f < NIN; ++f) acc = fmaf(x[f], W[S::OW1 + f * H + j], acc);
    z1[j] = acc;
    a1[j] = lrelu(acc, alpha);
  }
#pragma unroll
  for (int j = 0; j < H; ++j) {
    float acc = W[S::OB2 + j];
#pragma unroll
    for (int i = 0; i < H; ++i) acc = fmaf(a1[i], W[S::OW2 + i * H + j], acc);
    z2[j] = acc;
    a2[j] = lrelu(acc, alpha);
  }
  float o[NO];
#pragma unroll
  for (int k = 0; k < NO; ++k) {
    float acc = W[S::OB3 + k];
#pragma unroll
    for (int j = 0; j < H; ++j) acc = fmaf(a2[j], W[S::OW3 + j * NO + k], acc);
    o[k] = acc;
  }
  if (HEAD == HEAD_COMPLEMENT) {  // EO: psi = 1 - phi  ("European Options.ipynb" cell 12)
    hold[0] = o[0];
    hold[1] = 1.0f - o[0];
  } else {
#pragma unroll
    for (int k = 0; k < S::NHOLD; ++k) hold[k] = o[k];
  }
}

// ---------------------------------------------------------------------------
// Adam + EarlyStopping + LR schedule (K10).  Runs in ONE workgroup of 256
// threads, weights updated IN PLACE (every other workgroup of the launch has
// already passed the arrival ticket, i.e. finished reading them).  gsum (LDS)
// holds the summed gradient [P] followed by the 4 loss statistics.
// Keras 2.x semantics:
//   lr_t = lr*sqrt(1-b2^t)/(1-b1^t); m += (g-m)(1-b1); v += (g^2-v)(1-b2);
//   w -= lr_t*m/(sqrt(v)+eps)
// EarlyStopping.on_epoch_end: wait+=1; if loss<best: best=loss, save, wait=0;
//   if wait>=patience and epoch>0: stop (+restore best).
// ---------------------------------------------------------------------------
// Optimizer/early-stop state prefetched by EVERY workgroup at kernel start, so
// the last arriver can apply the update without another memory round trip.
struct UpdPre {
  float m, v, w, wbest;                 // this thread's parameter (tid < P)
  float t, lr, b1, b2, eps, nan_steps;
  float loss_sum, abs_sum, ape_sum, loss_cnt;
  float wait, has_best, best_loss, patience, max_epochs, restore_best, restore_at_end;
  float lr_sched_e;                     // lr_sched[epoch] (NaN if none)
};

template <int P>
RPH_INLINE void prefetch_update(UpdPre& u, const NetWeights* wts, const OptState* opt, const FitState* fs,
                                const float* lr_sched, int epoch, int step) {
  const int tid = threadIdx.x;
  if (tid < P) {
    u.m = opt->m[tid];
    u.v = opt->v[tid];
    u.w = wts->w[0][tid];
    u.wbest = fs->w_best[tid];
  } else {
    u.m = u.v = u.w = u.wbest = 0.f;
  }
  u.t = opt->t; u.lr = opt->lr; u.b1 = opt->beta1; u.b2 = opt->beta2; u.eps = opt->eps;
  u.nan_steps = opt->nan_steps;
  u.loss_sum = fs->loss_sum; u.abs_sum = fs->abs_sum; u.ape_sum = fs->ape_sum; u.loss_cnt = fs->loss_cnt;
  u.wait = fs->wait; u.has_best = fs->has_best; u.best_loss = fs->best_loss; u.patience = fs->patience;
  u.max_epochs = fs->max_epochs; u.restore_best = fs->restore_best; u.restore_at_end = fs->restore_at_end;
  u.lr_sched_e = (step == 0 && lr_sched != nullptr) ? lr_sched[epoch] : __builtin_nanf("");
}

// ---------------------------------------------------------------------------
// Adam + EarlyStopping + LR schedule (K10).  Runs in ONE workgroup of 256
// threads, weights updated IN PLACE (every other workgroup of the launch has
// already passed the arrival ticket, i.e. finished reading them).  gsum (LDS)
// holds the summed gradient [P] followed by the 4 loss statistics.
// Keras 2.x semantics:
//   lr_t = lr*sqrt(1-b2^t)/(1-b1^t); m += (g-m)(1-b1); v += (g^2-v)(1-b2);
//   w -= lr_t*m/(sqrt(v)+eps)
// EarlyStopping.on_epoch_end: wait+=1; if loss<best: best=loss, save, wait=0;
//   if wait>=patience and epoch>0: stop (+restore best).
// ---------------------------------------------------------------------------
template <int P>
RPH_INLINE void apply_update(const float* gsum, const UpdPre& u, NetWeights* wts, OptState* opt, FitState* fs,
                             int epoch, int step, int steps_per_epoch) {
  const int tid = threadIdx.x;
  const bool mine = tid < P;
  const float g = mine ? gsum[tid] : 0.f;
  const float lr = (u.lr_sched_e == u.lr_sched_e) ? u.lr_sched_e : u.lr;  // on_epoch_begin (NaN => keep)
  const int finite = __syncthreads_and(mine ? (int)__builtin_isfinite(g) : 1);  // NaN/Inf guard
  const float t = u.t + (finite ? 1.f : 0.f);
  // b^t = exp2(t log2 b) on the transcendental unit (v_log/v_exp, ~1 ulp)
  const float bc1 = 1.f - __builtin_amdgcn_exp2f(t * __builtin_amdgcn_logf(u.b1));
  const float bc2 = 1.f - __builtin_amdgcn_exp2f(t * __builtin_amdgcn_logf(u.b2));
  const float lr_t = lr * sqrtf(bc2) * __frcp_rn(bc1);
  float wnew = u.w;
  if (mine && finite) {
    const float m = u.m + (g - u.m) * (1.f - u.b1);
    const float v = u.v + (g * g - u.v) * (1.f - u.b2);
    opt->m[tid] = m;
    opt->v[tid] = v;
    wnew = u.w - lr_t * m * __frcp_rn(sqrtf(v) + u.eps);
  }
  // epoch bookkeeping: computed redundantly by every thread from the prefetched
  // (uniform) state — no extra barrier; thread 0 persists it.
  const float loss_sum = u.loss_sum + gsum[P + 0];
  const float abs_sum = u.abs_sum + gsum[P + 1];
  const float ape_sum = u.ape_sum + gsum[P + 2];
  const float loss_cnt = u.loss_cnt + gsum[P + 3];
  int act = 0;
  if (step == steps_per_epoch - 1) {
    const float cnt = fmaxf(loss_cnt, 1.f);
    const float L = loss_sum * __frcp_rn(cnt);
    float wait = u.wait + 1.f, best = u.best_loss, stopped = 0.f;
    if (L < best || u.has_best == 0.f) {
      if (L < best) { best = L; wait = 0.f; }
      act = 1;
    }
    if (wait >= u.patience && epoch > 0) {
      stopped = 1.f;
      if (u.restore_best != 0.f) act = 2;
    }
    if ((float)(epoch + 1) >= u.max_epochs && stopped == 0.f) {
      stopped = 1.f;
      if (u.restore_best != 0.f && u.restore_at_end != 0.f) act = 2;
    }
    if (tid == 0) {
      if (epoch < MAXHIST) fs->hist[epoch] = L;
      fs->last_loss = L;
      fs->last_mae = abs_sum * __frcp_rn(cnt);
      fs->last_mape = 100.f * ape_sum * __frcp_rn(cnt);
      fs->loss_sum = fs->abs_sum = fs->ape_sum = fs->loss_cnt = 0.f;
      fs->wait = wait;
      fs->best_loss = best;
      fs->has_best = 1.f;
      fs->epoch = (float)(epoch + 1);
      fs->stopped = stopped;
    }
  } else if (tid == 0) {
    fs->loss_sum = loss_sum;
    fs->abs_sum = abs_sum;
    fs->ape_sum = ape_sum;
    fs->loss_cnt = loss_cnt;
  }
  if (tid == 0) {
    opt->lr = lr;
    opt->t = t;
    if (!finite) opt->nan_steps = u.nan_steps + 1.f;
  }
  if (mine) {
    if (act == 1) fs->w_best[tid] = wnew;
    wts->w[0][tid] = (act == 2) ? u.wbest : wnew;
  }
}

// agent-scope (sc1) 4-byte accesses for the cross-workgroup hand-off
RPH_INLINE void st_agent(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
RPH_INLINE float ld_agent(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int ACC_REPLICAS = 8;  // float-atomic accumulator replicas (contention / 8)

// ---------------------------------------------------------------------------
// Fused one-shot all-reduce of the gradient packet over xGMI (data parallel).
// Runs in the last-arriving workgroup of every rank: push the local packet to
// every rank's mailbox (IPC-mapped peer HBM, system-scope write-through
// stores), raise one flag per peer after every storing wave has drained,
// wait for all peers' flags, then sum the W packets from local HBM in fixed
// rank order — every rank computes the bitwise-identical sum, so the Adam
// update and the early-stopping decision are identical everywhere.  The tag is
// a per-rank device step counter (not a launch argument), so graph replays
// never see stale flags; DP_SLOTS-deep mailboxes let a fast rank run ahead.
// Spins are bounded; a timeout sets dp_error (checked by the host).
// ---------------------------------------------------------------------------
template <int R>
RPH_INLINE void dp_allreduce(const TrainDesc& d, float* red) {
  __shared__ uint32_t s_seq;
  const int tid = threadIdx.x;
  const int W = d.dp_world, me = d.dp_rank;
  if (tid == 0) s_seq = __hip_atomic_load(d.dp_counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const uint32_t seq = s_seq;
  const int slot = (int)(seq % DP_SLOTS);
  if (tid < R) {
    const float v = red[tid];
    for (int p = 0; p < W; ++p)
      __hip_atomic_store(d.dp_mbox[p] + ((size_t)slot * W + me) * R + tid, v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (tid < W) {
    __hip_atomic_store(d.dp_flags[tid] + slot * W + me, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    // wait for rank `tid`'s packet in MY mailbox
    uint32_t* f = d.dp_flags[me] + slot * W + tid;
    unsigned it = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
      __builtin_amdgcn_s_sleep(2);
      if (++it > (1u << 23)) {  // ~seconds: a peer never arrived
        __hip_atomic_store(d.dp_error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
  if (tid < R) {
    float s = 0.f;
    for (int p = 0; p < W; ++p)
      s += __hip_atomic_load(d.dp_mbox[me] + ((size_t)slot * W + p) * R + tid, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    red[tid] = s;
  }
  if (tid == 0) __hip_atomic_store(d.dp_counter, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
}


// ---------------------------------------------------------------------------
// K9: one optimizer step.  Grid = num_wgs workgroups of 256 threads.
// ---------------------------------------------------------------------------
template <int NIN, int H, int NO, int HEAD>
__global__ __launch_bounds__(256) void k_hedge_train_step(const TrainDesc d, const int step, const int epoch,
                                                          const Perm perm) {
  using S = NetShape<NIN, H, NO, HEAD>;
  constexpr int R = S::R;
  constexpr int P = S::P;
  constexpr int NHOLD = S::NHOLD;
  __shared__ __attribute__((aligned(16))) float lds[(4 * R > 1024 ? 4 * R : 1024) + 8];
  __shared__ __attribute__((aligned(16))) float wl[P + 4];
  __shared__ int s_last;

  // prologue: every independent load is issued up front — early-stop flag,
  // weights, the optimizer state for a possible last-arriver update, and the
  // first path's data (epoch is a launch argument, so the permutation needs no
  // device read).
  RPH_STAMP(0);
  const float stopped = d.fit->stopped;
  const float wv = threadIdx.x < P ? d.wts->w[0][threadIdx.x] : 0.f;
  UpdPre up;
  if (d.fused_update) prefetch_update<P>(up, d.wts, d.opt, d.fit, d.lr_sched, epoch, step);

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nwaves = gridDim.x * 4;
  const int gw = blockIdx.x * 4 + wid;

  const uint32_t cmask = (1u << d.chunk_log2) - 1u;  // perm keys come from the host (launch argument)
  const long long base = (long long)step * d.batch;

  // path data of iteration `it` (software-pipelined one iteration ahead)
  auto load_path = [&](long long j0, float (&x)[NIN], float (&pr)[NHOLD], float& y, bool& valid) {
    const long long jl = j0 + lane;
    const long long j = base + jl;
    valid = (jl < d.batch) && (j < d.n_local);
    uint32_t p = 0;
    if (valid) {
      const uint32_t ju = (uint32_t)j;
      p = (perm(ju >> d.chunk_log2) << d.chunk_log2) | (ju & cmask);
      if (p >= (uint32_t)d.n_local) p = ju;  // (only when n_local is not chunk-aligned)
    }
#pragma unroll
    for (int f = 0; f < NIN; ++f) x[f] = valid ? d.feat[f][p] : 0.f;
#pragma unroll
    for (int k = 0; k < NHOLD - 1; ++k) pr[k] = valid ? d.price[k][p] : 0.f;
    pr[NHOLD - 1] = d.bond;
    y = valid ? d.target[p] : 0.f;
  };
  long long j0 = (long long)gw * 64;
  float xn[NIN], prn[NHOLD], yn = 0.f;
  bool validn = false;
  if (j0 < d.batch) load_path(j0, xn, prn, yn, validn);

  if (stopped != 0.f) return;  // early-stopped fit: remaining steps are no-ops
  // Weights are wave-uniform: stage them once in LDS and read them as
  // broadcast ds_read_b128 (keeps the 100+ weights out of the SGPR file).
  if (threadIdx.x < P) wl[threadIdx.x] = wv;
  if (d.fused_update) {  // keep the prefetch here (the compiler would sink it into the last-arriver branch)
    asm volatile("" ::"v"(up.m), "v"(up.v), "v"(up.w), "v"(up.wbest), "s"(up.t), "s"(up.lr), "s"(up.loss_sum),
                 "s"(up.wait), "s"(up.best_loss), "s"(up.lr_sched_e));
  }
  __syncthreads();
  RPH_STAMP(1);
  const float* __restrict__ W = wl;

  float g[R];
#pragma unroll
  for (int i = 0; i < R; ++i) g[i] = 0.f;

  const float alpha = d.alpha;
  for (; j0 < d.batch; j0 += (long long)nwaves * 64) {
    // (loop-invariant LDS weights are hoisted into registers by the compiler;
    // re-reading them per iteration to reach 2 waves/SIMD measured slower)
    const float* __restrict__ Wi = W;
    float x[NIN], pr[NHOLD];
#pragma unroll
    for (int f = 0; f < NIN; ++f) x[f] = xn[f];
#pragma unroll
    for (int k = 0; k < NHOLD; ++k) pr[k] = prn[k];
    const float y = yn;
    const bool valid = validn;
    const long long jnext = j0 + (long long)nwaves * 64;
    if (jnext < d.batch) load_path(jnext, xn, prn, yn, validn);

    float z1[H], a1[H], z2[H], a2[H], hold[NHOLD];
    net_forward<NIN, H, NO, HEAD>(Wi, x, alpha, z1, a1, z2, a2, hold);
    float V = 0.f;
#pragma unroll
    for (int k = 0; k < NHOLD; ++k) V = fmaf(hold[k], pr[k], V);

    // loss + dL/dV (mean over the global batch)
    const float e = V - y;
    float l, dV;
    if (d.loss == LOSS_PINBALL) {
      const float ep = -e;  // y - V
      const float q = d.quantile;
      const bool pos = q * ep >= (q - 1.f) * ep;
      l = pos ? q * ep : (q - 1.f) * ep;
      dV = pos ? -q : (1.f - q);
    } else {
      l = e * e;
      dV = 2.f * e;
    }
    dV = valid ? dV * d.inv_batch : 0.f;
    const float ae = fabsf(e);
    g[P + 0] += valid ? l : 0.f;
    g[P + 1] += valid ? ae : 0.f;
    g[P + 2] += valid ? ae / fmaxf(fabsf(y), 1e-7f) : 0.f;
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
      dz2[j] = da * lrelu_d(z2[j], alpha);
      g[S::OB2 + j] += dz2[j];
    }
#pragma unroll
    for (int i = 0; i < H; ++i) {
      float da = 0.f;
#pragma unroll
      for (int j = 0; j < H; ++j) {
        g[S::OW2 + i * H + j] = fmaf(a1[i], dz2[j], g[S::OW2 + i * H + j]);
        da = fmaf(Wi[S::OW2 + i * H + j], dz2[j], da);
      }
      const float dz1 = da * lrelu_d(z1[i], alpha);
      g[S::OB1 + i] += dz1;
#pragma unroll
      for (int f = 0; f < NIN; ++f) g[S::OW1 + f * H + i] = fmaf(x[f], dz1, g[S::OW1 + f * H + i]);
    }
  }

  RPH_STAMP(2);
  // ---- in-wave reduce-scatter, cross-wave LDS sum --------------------------
  wave_reduce_scatter<R>(g, lane);
  constexpr int PER = R / 64;
#pragma unroll
  for (int i = 0; i < PER; ++i) lds[wid * R + lane * PER + i] = g[i];
  __syncthreads();
  float* red = lds;  // reuse: red[t] for t < R after the sum below
  float val = 0.f;
  if (threadIdx.x < R) val = lds[threadIdx.x] + lds[R + threadIdx.x] + lds[2 * R + threadIdx.x] + lds[3 * R + threadIdx.x];
  __syncthreads();
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

// K10 standalone (world_size > 1): one workgroup applies the all-reduced update.
template <int NIN, int H, int NO, int HEAD>
__global__ __launch_bounds__(256) void k_hedge_update(const TrainDesc d, const int step, const int epoch) {
  using S = NetShape<NIN, H, NO, HEAD>;
  __shared__ float gs[S::R + 8];
  if (d.fit->stopped != 0.f) return;
  UpdPre up;
  prefetch_update<S::P>(up, d.wts, d.opt, d.fit, d.lr_sched, epoch, step);
  for (int i = threadIdx.x; i < S::R; i += blockDim.x) gs[i] = d.grad_out[i];
  __syncthreads();
  apply_update<S::P>(gs, up, d.wts, d.opt, d.fit, epoch, step, d.steps_per_epoch);
}

// ---------------------------------------------------------------------------
// K12: value / holdings / residual epilogue of a backward-induction date.
//   V_t       = h(state_t) . p_t           (Keras predict(X0), RP:212)
//   blend     = g + c (h - g)              (RP:221)
//   residual  = V_{t+1} - h . p_{t+1}       ("VaR", RP:120; Q24)
// Per-workgroup fp64 statistics go to a [num_wgs][EVAL_NSTAT] slab.
// ---------------------------------------------------------------------------
template <int NIN, int H, int NO, int HEAD>
__global__ __launch_bounds__(256) void k_hedge_eval(const EvalDesc d) {
  using S = NetShape<NIN, H, NO, HEAD>;
  constexpr int NHOLD = S::NHOLD;
  __shared__ double sst[4][EVAL_NSTAT];
  __shared__ __attribute__((aligned(16))) float wl[2 * S::P + 8];
  const bool has_b = d.wb != nullptr;
  for (int i = threadIdx.x; i < S::P; i += 256) {
    wl[i] = d.wa->w[0][i];
    if (has_b) wl[S::P + 4 + i] = d.wb->w[0][i];
  }
  __syncthreads();
  const float* __restrict__ WA = wl;
  const float* __restrict__ WB = has_b ? wl + S::P + 4 : wl;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;

  // per-thread fp32 partials (a thread sees only a handful of paths), one
  // in-wave reduce-scatter, fp64 only across waves / workgroups
  constexpr int NS = 64;
  float st[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) st[i] = 0.f;
  float rmin = INFINITY, rmax = -INFINITY;

  for (int p0 = blockIdx.x * 256; p0 < d.n_local; p0 += gridDim.x * 256) {
    const int p = p0 + threadIdx.x;
    const bool valid = p < d.n_local;
    const int pp = valid ? p : 0;
    float x[NIN];
#pragma unroll
    for (int f = 0; f < NIN; ++f) x[f] = d.feat[f][pp];
    float z1[H], a1[H], z2[H], a2[H], hold[NHOLD], holdv[NHOLD];
    net_forward<NIN, H, NO, HEAD>(WA, x, d.alpha, z1, a1, z2, a2, hold);
#pragma unroll
    for (int k = 0; k < NHOLD; ++k) holdv[k] = hold[k];
    if (has_b) {
      // V_t comes from net B (model2.predict, RP:218); reported holdings are
      // the blend hA + hold_c (hB - hA) (get_phi_psi_VaR, RP:114-115).
      net_forward<NIN, H, NO, HEAD>(WB, x, d.alpha, z1, a1, z2, a2, holdv);
#pragma unroll
      for (int k = 0; k < NHOLD; ++k) hold[k] = hold[k] + d.hold_c * (holdv[k] - hold[k]);
    }
    float V = 0.f;
#pragma unroll
    for (int k = 0; k < NHOLD - 1; ++k) V = fmaf(holdv[k], d.price_t[k][pp], V);
    V = fmaf(holdv[NHOLD - 1], d.bond_t, V);
    if (d.g_base) {
      const float gb = d.g_base[pp];
      V = gb + d.blend_c * (V - gb);
    }
    float res = 0.f, pred1 = 0.f, tgt = 0.f;
    const bool has1 = d.price_t1[0] != nullptr;
    if (has1) {
#pragma unroll
      for (int k = 0; k < NHOLD - 1; ++k) pred1 = fmaf(hold[k], d.price_t1[k][pp], pred1);
      pred1 = fmaf(hold[NHOLD - 1], d.bond_t1, pred1);
      if (d.target) {
        tgt = d.target[pp];
        res = tgt - pred1;
      }
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

static inline bool shape_is(int nin, int h, int nout, int head, int a, int b, int c, int e) {
  return nin == a && h == b && nout == c && head == e;
}

extern "C" int rph_net_nparams(int nin, int h, int nout, int head, int* p_out, int* r_out) {
#define X(A, B, C, E)                                  \
  if (shape_is(nin, h, nout, head, A, B, C, E)) {      \
    *p_out = NetShape<A, B, C, E>::P;                  \
    *r_out = NetShape<A, B, C, E>::R;                  \
    return 0;                                          \
  }
  RPH_SHAPES(X)
#undef X
  return -1;
}

extern "C" int rph_train_step(const TrainDesc* d, int step, int epoch, void* stream) {
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
  return -1;
}

extern "C" int rph_train_update(const TrainDesc* d, int step, int epoch, void* stream) {
  hipStream_t s = (hipStream_t)stream;
#define X(A, B, C, E)                                                                        \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E)) {                               \
    hipLaunchKernelGGL((k_hedge_update<A, B, C, E>), dim3(1), dim3(256), 0, s, *d, step, epoch); \
    return (int)hipGetLastError();                                                           \
  }
  RPH_SHAPES(X)
#undef X
  return -1;
}

extern "C" int rph_eval(const EvalDesc* d, void* stream) {
  hipStream_t s = (hipStream_t)stream;
#define X(A, B, C, E)                                                                        \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E)) {                               \
    hipLaunchKernelGGL((k_hedge_eval<A, B, C, E>), dim3(d->num_wgs), dim3(256), 0, s, *d);  \
    return (int)hipGetLastError();                                                           \
  }
  RPH_SHAPES(X)
#undef X
  return -1;
}
