// rphedge — machinery shared by the hedge-MLP training-step kernels
// (hedge_mlp.hip: thread-per-path VALU kernel for the reference's 8-unit nets;
// hedge_mlp_wide.hip: MFMA kernel for 32-unit nets): network shapes, the
// minibatch chunk permutation, the fp32 forward pass, Keras-Adam + early
// stopping applied by the last-arriving workgroup, and the fused xGMI one-shot
// all-reduce of the gradient packet.
//
// Reference semantics: Replicating_Portfolio.py:149-221 (model, compile, fit,
// EarlyStopping, LearningRateScheduler).
#pragma once
#include "rph_common.h"
#include "rph_types.h"

namespace rph {

// Diagnostic phase stamps (s_memrealtime, 100 MHz): thread 0 of every
// workgroup writes stamp k to d.stamps[blockIdx.x * 8 + k] when d.stamps is set.
#define RPH_STAMP(k)                                                                    \
  do {                                                                                  \
    if (d.stamps != nullptr && threadIdx.x == 0)                                        \
      d.stamps[(size_t)blockIdx.x * 8 + (k)] = rph_stamp_clock();                       \
  } while (0)
// the LM pass body's "path loop done" stamp (k_lm_pass's workgroups 0 and 1
// leave stamp rows 0 and 1 to k_lm_solve; the Adam bodies stamp every row)
#define RPH_STAMP_BODY(k)                                                               \
  do {                                                                                  \
    if (blockIdx.x >= 2) RPH_STAMP(k);                                                  \
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
  // gradient-packet width: [P grads | 4 stats | zero pad]
  //   narrow (VALU, P+4 <= 256): the in-wave reduce-scatter width (pow2)
  //   wide (MFMA): a multiple of 256 (one entry per thread per pass)
  static constexpr int R = (P + NSTAT <= 128) ? 128 : (P + NSTAT <= 256) ? 256 : ((P + NSTAT + 255) / 256) * 256;
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

// global path index of minibatch slot j (chunk-permuted)
RPH_INLINE uint32_t perm_path(const Perm& perm, uint32_t j, int chunk_log2, int n_local) {
  const uint32_t cmask = (1u << chunk_log2) - 1u;
  uint32_t p = (perm(j >> chunk_log2) << chunk_log2) | (j & cmask);
  if (p >= (uint32_t)n_local) p = j;  // (only when n_local is not chunk-aligned)
  return p;
}

// ---------------------------------------------------------------------------
// Forward pass of one path (fp32).  W is wave-uniform.
// ---------------------------------------------------------------------------
template <int NIN, int H, int NO, int HEAD>
RPH_INLINE void net_forward(const float* __restrict__ W, const float (&x)[NIN], float alpha,
                            float (&z1)[H], float (&a1)[H], float (&z2)[H], float (&a2)[H],
                            float (&hold)[NetShape<NIN, H, NO, HEAD>::NHOLD],
                            const float* __restrict__ W2 = nullptr /* source of the W2 block (default W) */) {
  using S = NetShape<NIN, H, NO, HEAD>;
  if (W2 == nullptr) W2 = W;
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
    for (int i = 0; i < H; ++i) acc = fmaf(a1[i], W2[S::OW2 + i * H + j], acc);
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

// loss of one path and dL/dV (mean over the global batch folded in by the caller)
RPH_INLINE void path_loss(int loss, float q, float V, float y, float& l, float& dV) {
  const float e = V - y;
  if (loss == LOSS_PINBALL) {
    const float ep = -e;  // y - V
    const bool pos = q * ep >= (q - 1.f) * ep;
    l = pos ? q * ep : (q - 1.f) * ep;
    dV = pos ? -q : (1.f - q);
  } else {
    l = e * e;
    dV = 2.f * e;
  }
}

// ---------------------------------------------------------------------------
// Optimizer/early-stop state prefetched by EVERY workgroup at kernel start, so
// the last arriver can apply the update without another memory round trip.
// Thread t owns parameters t, t+256, ... (NPT of them).
// ---------------------------------------------------------------------------
template <int P>
struct UpdPre {
  static constexpr int NPT = (P + 255) / 256;
  float m[NPT], v[NPT], w[NPT], wbest[NPT];
  float t, lr, b1, b2, eps, nan_steps;
  float loss_sum, abs_sum, ape_sum, loss_cnt;
  float wait, has_best, best_loss, patience, max_epochs, restore_best, restore_at_end;
  float lr_sched_e;                     // lr_sched[epoch] (NaN if none)
};

template <int P>
RPH_INLINE void prefetch_update(UpdPre<P>& u, const NetWeights* wts, const OptState* opt, const FitState* fs,
                                const float* lr_sched, int epoch, int step) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < UpdPre<P>::NPT; ++k) {
    const int i = tid + 256 * k;
    if (i < P) {
      u.m[k] = opt->m[i];
      u.v[k] = opt->v[i];
      u.w[k] = wts->w[0][i];
      u.wbest[k] = fs->w_best[i];
    } else {
      u.m[k] = u.v[k] = u.w[k] = u.wbest[k] = 0.f;
    }
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
// A non-finite gradient skips the whole update (NaN/Inf guard, counted).
// ---------------------------------------------------------------------------
template <int P>
RPH_INLINE void apply_update(const float* gsum, const UpdPre<P>& u, NetWeights* wts, OptState* opt, FitState* fs,
                             int epoch, int step, int steps_per_epoch) {
  constexpr int NPT = UpdPre<P>::NPT;
  const int tid = threadIdx.x;
  float g[NPT];
  int fin = 1;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int i = tid + 256 * k;
    g[k] = (i < P) ? gsum[i] : 0.f;
    fin &= (int)__builtin_isfinite(g[k]);
  }
  const float lr = (u.lr_sched_e == u.lr_sched_e) ? u.lr_sched_e : u.lr;  // on_epoch_begin (NaN => keep)
  const int finite = __syncthreads_and(fin);
  const float t = u.t + (finite ? 1.f : 0.f);
  // b^t = exp2(t log2 b) on the transcendental unit (v_log/v_exp, ~1 ulp)
  const float bc1 = 1.f - __builtin_amdgcn_exp2f(t * __builtin_amdgcn_logf(u.b1));
  const float bc2 = 1.f - __builtin_amdgcn_exp2f(t * __builtin_amdgcn_logf(u.b2));
  const float lr_t = lr * sqrtf(bc2) * __frcp_rn(bc1);
  float wnew[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int i = tid + 256 * k;
    wnew[k] = u.w[k];
    if (i < P && finite) {
      const float m = u.m[k] + (g[k] - u.m[k]) * (1.f - u.b1);
      const float v = u.v[k] + (g[k] * g[k] - u.v[k]) * (1.f - u.b2);
      opt->m[i] = m;
      opt->v[i] = v;
      wnew[k] = u.w[k] - lr_t * m * __frcp_rn(sqrtf(v) + u.eps);
    }
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
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int i = tid + 256 * k;
    if (i < P) {
      if (act == 1) fs->w_best[i] = wnew[k];
      wts->w[0][i] = (act == 2) ? u.wbest[k] : wnew[k];
    }
  }
}

// agent-scope (sc1) 4-byte accesses for the cross-workgroup hand-off
RPH_INLINE void st_agent(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
RPH_INLINE float ld_agent(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bound of one wait for the peers' packets (100 MHz s_memrealtime ticks):
// generous, because ranks may enter their first step seconds apart (graph
// upload, page faults); after a timeout dp_error makes every later wait exit
constexpr unsigned long long DP_SPIN_TICKS = 2000000000ull;  // 20 s

constexpr int ACC_REPLICAS = 8;  // float-atomic accumulator replicas (contention / 8)
// lagged schedule, 32-unit nets: every workgroup re-reads the whole packet of
// the previous step in its prologue, R = 1280+ floats x replicas — fewer
// replicas trade atomic contention for prologue read traffic
// lagged schedule: the narrow nets use RPH_NARROW_NREP of the LAG_SLOTS
// accumulator replica rows (rph_types.h)
#ifndef RPH_NARROW_NREP
#define RPH_NARROW_NREP 16
#endif
constexpr int NARROW_NREP = RPH_NARROW_NREP;
#ifndef RPH_WIDE_NREP
#define RPH_WIDE_NREP 8
#endif
constexpr int WIDE_NREP = RPH_WIDE_NREP;

// sum of the first NREP (<= ACC_REPLICAS, power of two) float-atomic replicas
// of packet entry i, pairwise in fixed order
// AGENT: agent-scope loads (L2 bypass) - needed inside the persistent kernel,
// where the replicas were written by the same launch.  Across a kernel
// boundary (lagged schedule: step k reads step k-1's accumulator) the
// boundary's acquire already invalidated the non-coherent L2, so plain loads
// are correct and let the ~32 workgroups of an XCD share one L2 fill instead
// of each fetching the packet from the memory side.
template <int NREP = ACC_REPLICAS, bool AGENT = true>
RPH_INLINE float sum_replicas(const float* buf, int R, int i) {
  static_assert(NREP >= 1 && NREP <= LAG_SLOTS && (NREP & (NREP - 1)) == 0, "replicas: power of two <= 16");
  float rr[NREP];
#pragma unroll
  for (int rp = 0; rp < NREP; ++rp) rr[rp] = AGENT ? ld_agent(buf + rp * R + i) : buf[rp * R + i];
#pragma unroll
  for (int w = NREP / 2; w >= 1; w /= 2)
#pragma unroll
    for (int j = 0; j < w; ++j) rr[j] = rr[2 * j] + rr[2 * j + 1];
  return rr[0];
}

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
template <int LEN>
RPH_INLINE void dp_allreduce(const TrainDesc& d, float* red) {
  __shared__ uint32_t s_seq;
  const int tid = threadIdx.x;
  const int W = d.dp_world, me = d.dp_rank;
  if (tid == 0) s_seq = __hip_atomic_load(d.dp_counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const uint32_t seq = s_seq;
  const int slot = (int)(seq % DP_SLOTS);
  for (int i = tid; i < LEN; i += 256) {
    const float v = red[i];
    for (int p = 0; p < W; ++p)
      __hip_atomic_store(d.dp_mbox[p] + ((size_t)slot * W + me) * LEN + i, v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (tid < W) {
    __hip_atomic_store(d.dp_flags[tid] + slot * W + me, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    // wait for rank `tid`'s packet in MY mailbox
    uint32_t* f = d.dp_flags[me] + slot * W + tid;
    unsigned it = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
      __builtin_amdgcn_s_sleep(2);
      ++it;
      // a peer never arrived (DP_SPIN_TICKS), or an earlier step already timed
      // out: fail fast instead of spinning again in every later step
      if ((it & 255u) == 0u &&
          (__builtin_amdgcn_s_memrealtime() - t0 > DP_SPIN_TICKS ||
           __hip_atomic_load(d.dp_error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)) {
        __hip_atomic_store(d.dp_error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < LEN; i += 256) {
    float s = 0.f;
    for (int p = 0; p < W; ++p)
      s += __hip_atomic_load(d.dp_mbox[me] + ((size_t)slot * W + p) * LEN + i, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    red[i] = s;
  }
  if (tid == 0) __hip_atomic_store(d.dp_counter, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
}

// K10 standalone (RCCL data parallel / split update): one workgroup applies the
// all-reduced packet grad_out[LEN].
template <int P, int LEN>
__global__ __launch_bounds__(256) void k_hedge_update(const TrainDesc d, const int step, const int epoch) {
  prefetch_kernarg<sizeof(TrainDesc) + 2 * sizeof(int)>();
  __shared__ float gs[LEN + 8];
  if (d.fit->stopped != 0.f) return;
  UpdPre<P> up;
  prefetch_update<P>(up, d.wts, d.opt, d.fit, d.lr_sched, epoch, step);
  for (int i = threadIdx.x; i < LEN; i += blockDim.x) gs[i] = d.grad_out[i];
  __syncthreads();
  apply_update<P>(gs, up, d.wts, d.opt, d.fit, epoch, step, d.steps_per_epoch);
}

// Supported shapes: the reference's 8-unit nets run the VALU thread-per-path
// step kernel; 32-unit nets the MFMA step kernel (hedge_mlp_wide.hip).
#define RPH_SHAPES(X)            \
  X(1, 8, 1, HEAD_COMPLEMENT)    \
  X(1, 8, 2, HEAD_FREE)          \
  X(2, 8, 2, HEAD_FREE)          \
  X(3, 8, 2, HEAD_FREE)          \
  X(4, 8, 2, HEAD_FREE)          \
  X(5, 8, 6, HEAD_FREE)          \
  X(6, 8, 7, HEAD_FREE)

#define RPH_WIDE_SHAPES(X)       \
  X(1, 32, 1, HEAD_COMPLEMENT)   \
  X(1, 32, 2, HEAD_FREE)         \
  X(2, 32, 2, HEAD_FREE)         \
  X(3, 32, 2, HEAD_FREE)         \
  X(5, 32, 6, HEAD_FREE)

static inline bool shape_is(int nin, int h, int nout, int head, int a, int b, int c, int e) {
  return nin == a && h == b && nout == c && head == e;
}

int rph_report(const char* what, const char* msg);  // runtime.cpp: sets rph_last_error, returns -22

// Host-side check of a training descriptor against what the kernels and their
// grids assume (run before every launch: a bad shape must not reach the GPU).
// mode: 0 ticket step, 1 lagged step / finalize, 2 persistent fit.
inline int validate_train(const TrainDesc* d, int mode, const char* who) {
  const int nhold = d->head == HEAD_COMPLEMENT ? 2 : d->nout;
  if (d->nin < 1 || d->nin > MAXIN || nhold < 1 || nhold > MAXHOLD) return rph_report(who, "network shape out of range");
  if (d->num_wgs < 1 || d->num_wgs > 65535) return rph_report(who, "num_wgs out of range");
  if (!(d->alpha >= 0.f && d->alpha <= 1.f)) return rph_report(who, "LeakyReLU slope must be in [0, 1]");
  if (d->batch < 1 || d->n_local < d->batch || d->steps_per_epoch < 1 ||
      (long long)d->batch * d->steps_per_epoch < d->n_local)
    return rph_report(who, "batch / steps_per_epoch do not cover n_local");
  if (d->chunk_log2 < 0 || d->chunk_log2 > 20) return rph_report(who, "chunk_log2 out of range");
  if (!d->wts || !d->opt || !d->fit || !d->target) return rph_report(who, "null state or target pointer");
  for (int f = 0; f < d->nin; ++f) {
    if (!d->feat[f]) return rph_report(who, "null feature pointer");
    if (!(d->fisd[f] > 0.f && d->fisd[f] < 3.0e38f && d->fmu[f] == d->fmu[f]))
      return rph_report(who, "feature standardisation must be finite with fisd > 0");
  }
  for (int k = 0; k < nhold - 1; ++k)
    if (!d->price[k]) return rph_report(who, "null price pointer");
  if (mode == 1 && (!d->lag || !d->acc)) return rph_report(who, "lagged step needs lag and acc buffers");
  if (mode == 2 && (!d->acc || !d->counter)) return rph_report(who, "persistent fit needs acc and counter");
  if (mode == 0) {
    if (!d->counter || (d->deterministic ? !d->slab : !d->acc)) return rph_report(who, "null reduction buffer");
    if (!d->fused_update && !d->grad_out) return rph_report(who, "split update needs grad_out");
  }
  if (d->dp_world > 1) {
    if (d->dp_world > 8 || d->dp_rank < 0 || d->dp_rank >= d->dp_world || !d->dp_counter || !d->dp_error)
      return rph_report(who, "bad data-parallel mailbox description");
    for (int p = 0; p < d->dp_world; ++p)
      if (!d->dp_mbox[p] || !d->dp_flags[p]) return rph_report(who, "null peer mailbox");
  }
  return 0;
}

// Wide (MFMA) training-step launcher (hedge_mlp_wide.hip); returns -1 when the
// shape is not a wide shape.
int launch_wide_step(const TrainDesc* d, int step, int epoch, const Perm& perm, hipStream_t s);

}  // namespace rph
