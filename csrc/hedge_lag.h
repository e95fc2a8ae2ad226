// rphedge — "lagged update" training step: one kernel per optimizer step with
// NO cross-workgroup synchronisation inside the kernel.
//
// Reference semantics: Keras fit() — for each step: forward/backward on the
// minibatch, Adam update; at epoch end EarlyStopping / LearningRateScheduler
// (Replicating_Portfolio.py:200-211).  Identical math, different schedule:
//
//   kernel k (k = e*S + s):
//     prologue  every workgroup loads the optimizer state of slot k&1 and the
//               summed gradient packet of step k-1 (3 rotating float-atomic
//               accumulators), applies the Keras-Adam update of step k-1 — and,
//               if k-1 closed an epoch, EarlyStopping — REDUNDANTLY (identical
//               inputs, identical code, identical results in every workgroup)
//     body      partial packet of step k with the updated weights
//     epilogue  fire-and-forget float atomics into accumulator k%3; workgroup 0
//               writes the updated state to slot (k+1)&1 and zeroes accumulator
//               (k+1)%3 (last read by kernel k-1, next added to by kernel k+1)
//   finalize   one workgroup applies the update of the last step and writes the
//              canonical NetWeights / OptState / FitState.
//
// Versus the ticketed step kernel this removes, per step, the arrival ticket,
// the wait for the slowest workgroup's adds and the serial "last arriver
// updates, next kernel re-reads" chain: the kernel boundary (~1.45 µs,
// MI355X_MICROARCH price list 'boundary') is the only global synchronisation,
// and it is cheaper than any in-kernel grid barrier ('barrier-xcd' ≥ 4.1 µs).
// The double-buffered state slot makes workgroup 0's write-back race-free.
// Early stop: the deciding kernel's workgroup 0 writes the canonical state and
// FitState.stopped; later kernels (and finalize) return at their first load.
#pragma once
#include "hedge_core.h"

namespace rph {

// lag slot layout (floats): w[PMAX] m[PMAX] v[PMAX] scalars[16]
enum LagScalar : int {
  LG_T = 0, LG_LR, LG_NAN, LG_BEST, LG_WAIT, LG_HASBEST, LG_LSUM, LG_ASUM, LG_PSUM, LG_CNT,
  LG_LASTL, LG_LASTMAE, LG_LASTMAPE, LG_SEQ /* DP sequence base, u32 bits */, LG_NSCALAR
};
constexpr int LAG_FLOATS = 3 * PMAX + 16;

RPH_INLINE uint32_t ld_agent_u32c(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int P>
struct LagState {
  static constexpr int NPT = (P + 255) / 256;
  float w[NPT], m[NPT], v[NPT], wb[NPT];
  float sc[LG_NSCALAR];
};

template <int P>
RPH_INLINE void lag_load(LagState<P>& st, const TrainDesc& d, const float* slot /* null: canonical */,
                         const FitState* fit0 /* fit state to start from (canonical load only) */) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < LagState<P>::NPT; ++k) {
    const int i = tid + 256 * k;
    const bool ok = i < P;
    if (slot == nullptr) {
      st.w[k] = ok ? d.wts->w[0][i] : 0.f;
      st.m[k] = ok ? d.opt->m[i] : 0.f;
      st.v[k] = ok ? d.opt->v[i] : 0.f;
    } else {
      st.w[k] = ok ? slot[i] : 0.f;
      st.m[k] = ok ? slot[PMAX + i] : 0.f;
      st.v[k] = ok ? slot[2 * PMAX + i] : 0.f;
    }
    st.wb[k] = ok ? (slot == nullptr ? fit0 : d.fit)->w_best[i] : 0.f;
  }
  if (slot == nullptr) {
    const OptState* o = d.opt;
    const FitState* f = fit0;
    st.sc[LG_T] = o->t; st.sc[LG_LR] = o->lr; st.sc[LG_NAN] = o->nan_steps;
    st.sc[LG_BEST] = f->best_loss; st.sc[LG_WAIT] = f->wait; st.sc[LG_HASBEST] = f->has_best;
    st.sc[LG_LSUM] = f->loss_sum; st.sc[LG_ASUM] = f->abs_sum; st.sc[LG_PSUM] = f->ape_sum;
    st.sc[LG_CNT] = f->loss_cnt; st.sc[LG_LASTL] = f->last_loss; st.sc[LG_LASTMAE] = f->last_mae;
    st.sc[LG_LASTMAPE] = f->last_mape;
    // data parallel: this fit's exchange sequence starts at the rank's device
    // counter (written only at the end of a fit — never by a kernel that
    // also reads it here, i.e. never by kernel 0)
    st.sc[LG_SEQ] = __uint_as_float(d.dp_world > 1 ? ld_agent_u32c(d.dp_counter) : 0u);
  } else {
#pragma unroll
    for (int j = 0; j < LG_NSCALAR; ++j) st.sc[j] = slot[3 * PMAX + j];
  }
}

template <int P>
RPH_INLINE void lag_store(const LagState<P>& st, float* slot) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < LagState<P>::NPT; ++k) {
    const int i = tid + 256 * k;
    if (i < P) {
      slot[i] = st.w[k];
      slot[PMAX + i] = st.m[k];
      slot[2 * PMAX + i] = st.v[k];
    }
  }
  if (tid == 0) {
#pragma unroll
    for (int j = 0; j < LG_NSCALAR; ++j) slot[3 * PMAX + j] = st.sc[j];  // (constant indices: no scratch)
  }
}

// canonical write-back (one workgroup); `stopped`, `ep_done` as decided
template <int P>
RPH_INLINE void lag_store_canonical(const LagState<P>& st, const TrainDesc& d, float stopped, int ep_done) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < LagState<P>::NPT; ++k) {
    const int i = tid + 256 * k;
    if (i < P) {
      d.wts->w[0][i] = st.w[k];
      d.opt->m[i] = st.m[k];
      d.opt->v[i] = st.v[k];
    }
  }
  if (tid == 0) {
    OptState* o = d.opt;
    FitState* f = d.fit;
    o->t = st.sc[LG_T]; o->lr = st.sc[LG_LR]; o->nan_steps = st.sc[LG_NAN];
    f->best_loss = st.sc[LG_BEST]; f->wait = st.sc[LG_WAIT]; f->has_best = st.sc[LG_HASBEST];
    f->loss_sum = st.sc[LG_LSUM]; f->abs_sum = st.sc[LG_ASUM]; f->ape_sum = st.sc[LG_PSUM];
    f->loss_cnt = st.sc[LG_CNT]; f->last_loss = st.sc[LG_LASTL]; f->last_mae = st.sc[LG_LASTMAE];
    f->last_mape = st.sc[LG_LASTMAPE];
    f->epoch = (float)ep_done;
    f->stopped = stopped;
  }
}

// data parallel: the exchanges of a fit used sequence numbers seq_base+1 ..
// seq_base+n; the next fit starts after them
RPH_INLINE void lag_advance_seq(const TrainDesc& d, float seq_base_bits, uint32_t n) {
  if (d.dp_world > 1 && threadIdx.x == 0)
    __hip_atomic_store(d.dp_counter, __float_as_uint(seq_base_bits) + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Cross-rank sum of step k-1's packet (sequence `seq`), fused xGMI one-shot
// with DATA-TAGGED GRANULES: the pusher workgroup of every rank sums its local
// accumulator and writes every entry as one 8-byte {value, seq} granule (a
// single system-scope 64-bit store, single-copy atomic) into every rank's IPC
// mailbox; every workgroup then polls the W granules of each entry until their
// tags equal `seq` and sums the values in fixed rank order (bitwise identical
// on all ranks and workgroups).  No separate flag hop: the load that observes
// the tag also returns the data (MI355X_MICROARCH price list: 'handoff-1to1'
// vs 'handoff-flag').  A rank can be at most one kernel ahead of a peer, so
// slot seq % DP_SLOTS is never overwritten while it is read; a stale granule
// carries an older tag.  Bounded spins; fail fast on dp_error.
template <int R, int NREP>
RPH_INLINE int lag_dp_exchange(const TrainDesc& d, uint32_t seq, const float* local_acc, float* red, bool pusher) {
  const int tid = threadIdx.x;
  const int W = d.dp_world, me = d.dp_rank;
  const int slot = (int)(seq % DP_SLOTS);
  if (pusher) {
    for (int i = tid; i < R; i += 256) {
      const float v = sum_replicas<NREP>(local_acc, R, i);
      const unsigned long long g = ((unsigned long long)seq << 32) | (unsigned long long)__float_as_uint(v);
#pragma unroll
      for (int p = 0; p < 8; ++p)
        if (p < W)
          __hip_atomic_store((unsigned long long*)d.dp_mbox[p] + ((size_t)slot * W + me) * R + i, g,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  int bad = 0;
  const unsigned long long* mb = (const unsigned long long*)d.dp_mbox[me] + (size_t)slot * W * R;
  for (int i = tid; i < R; i += 256) {
    float vals[8];
    unsigned todo = (1u << W) - 1u;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned it = 0;
    while (true) {
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        if ((todo >> p) & 1u) {
          const unsigned long long g = __hip_atomic_load(const_cast<unsigned long long*>(mb + (size_t)p * R + i),
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if ((uint32_t)(g >> 32) == seq) {
            vals[p] = __uint_as_float((uint32_t)g);
            todo &= ~(1u << p);
          }
        }
      }
      if (todo == 0u) break;
      __builtin_amdgcn_s_sleep(1);
      if ((++it & 63u) == 0u &&
          (__builtin_amdgcn_s_memrealtime() - t0 > DP_SPIN_TICKS ||  // a peer never arrived
           __hip_atomic_load(d.dp_error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)) {
        __hip_atomic_store(d.dp_error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        bad = 1;
        break;
      }
    }
    float a = 0.f;
#pragma unroll
    for (int p = 0; p < 8; ++p)
      if (p < W) a += vals[p];
    red[i] = a;
    if (bad) break;
  }
  return __syncthreads_or(bad);
}

template <int P>
RPH_INLINE int lag_apply(LagState<P>& st, const float* red, const TrainDesc& d, int e, int s, bool writer,
                         int& ep_done) {
  constexpr int NPT = LagState<P>::NPT;
  const int tid = threadIdx.x;
  const OptState* o = d.opt;
  const FitState* f = d.fit;
  if (s == 0 && d.lr_sched != nullptr) {  // LearningRateScheduler.on_epoch_begin (NaN => keep)
    const float ls = d.lr_sched[e];
    if (ls == ls) st.sc[LG_LR] = ls;
  }
  float g[NPT];
  int fin = 1;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int i = tid + 256 * k;
    g[k] = (i < P) ? red[i] : 0.f;
    fin &= (int)__builtin_isfinite(g[k]);
  }
  const int finite = __syncthreads_and(fin);
  if (finite) {
    const float b1 = o->beta1, b2 = o->beta2, eps = o->eps;
    const float t = st.sc[LG_T] + 1.f;
    st.sc[LG_T] = t;
    const float bc1 = 1.f - __builtin_amdgcn_exp2f(t * __builtin_amdgcn_logf(b1));
    const float bc2 = 1.f - __builtin_amdgcn_exp2f(t * __builtin_amdgcn_logf(b2));
    const float lr_t = st.sc[LG_LR] * sqrtf(bc2) * __frcp_rn(bc1);
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      st.m[k] = st.m[k] + (g[k] - st.m[k]) * (1.f - b1);
      st.v[k] = st.v[k] + (g[k] * g[k] - st.v[k]) * (1.f - b2);
      if (tid + 256 * k < P) st.w[k] = st.w[k] - lr_t * st.m[k] * __frcp_rn(sqrtf(st.v[k]) + eps);
    }
  } else {
    st.sc[LG_NAN] += 1.f;
  }
  st.sc[LG_LSUM] += red[P + 0];
  st.sc[LG_ASUM] += red[P + 1];
  st.sc[LG_PSUM] += red[P + 2];
  st.sc[LG_CNT] += red[P + 3];
  if (s != d.steps_per_epoch - 1) return 0;
  // ---- EarlyStopping.on_epoch_end ----------------------------------------------
  const float cnt = fmaxf(st.sc[LG_CNT], 1.f);
  const float L = st.sc[LG_LSUM] * __frcp_rn(cnt);
  float wait = st.sc[LG_WAIT] + 1.f, best = st.sc[LG_BEST], stopped = 0.f;
  int act = 0;
  if (L < best || st.sc[LG_HASBEST] == 0.f) {
    if (L < best) {
      best = L;
      wait = 0.f;
    }
    act = 1;
  }
  if (wait >= f->patience && e > 0) {
    stopped = 1.f;
    if (f->restore_best != 0.f) act = 2;
  }
  if ((float)(e + 1) >= f->max_epochs && stopped == 0.f) {
    stopped = 1.f;
    if (f->restore_best != 0.f && f->restore_at_end != 0.f) act = 2;
  }
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int i = tid + 256 * k;
    if (act == 1) {
      st.wb[k] = st.w[k];
      if (writer && i < P) d.fit->w_best[i] = st.w[k];
    }
    if (act == 2) st.w[k] = st.wb[k];
  }
  if (writer && tid == 0 && e < MAXHIST) d.fit->hist[e] = L;
  st.sc[LG_LASTL] = L;
  st.sc[LG_LASTMAE] = st.sc[LG_ASUM] * __frcp_rn(cnt);
  st.sc[LG_LASTMAPE] = 100.f * st.sc[LG_PSUM] * __frcp_rn(cnt);
  st.sc[LG_LSUM] = st.sc[LG_ASUM] = st.sc[LG_PSUM] = st.sc[LG_CNT] = 0.f;
  st.sc[LG_WAIT] = wait;
  st.sc[LG_BEST] = best;
  st.sc[LG_HASBEST] = 1.f;
  ep_done = e + 1;
  return stopped != 0.f ? 1 : 0;
}

// summed packet of accumulator `buf` (NREP replicas) into LDS red[0..R)
// PLAIN: cached loads of the previous launch's accumulator (see sum_replicas);
// measured faster for the 128-float packets of the 8-unit nets, slower for the
// 1280-float packets of the 32-unit nets (profiles/r1/stamp_r1q_acc_loads.jsonl)
template <int R, int NREP, bool PLAIN = false>
RPH_INLINE void lag_sums(const float* buf, float* red) {
  for (int i = threadIdx.x; i < R; i += 256) red[i] = sum_replicas<NREP, !PLAIN>(buf, R, i);
}

template <class B>
__global__ __launch_bounds__(256, B::WAVES_PER_SIMD) void k_hedge_step_lag(const TrainDesc d, const int k, const int epoch,
                                                        const Perm perm) {
  constexpr int P = B::P;
  constexpr int R = B::R;
  constexpr int NR = B::NR;
  constexpr int NREP = B::NREP;  // float-atomic replicas in use (contention vs prologue read traffic)
  const uint32_t kat = prefetch_kernarg_begin<sizeof(TrainDesc) + 2 * sizeof(int) + sizeof(Perm)>();
  __shared__ __attribute__((aligned(16))) float scratch[B::SCRATCH_FLOATS];
  __shared__ __attribute__((aligned(16))) float wl[P + 4];
  __shared__ __attribute__((aligned(16))) float red[NR * 256 + 8];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int S = d.steps_per_epoch;
  const int s = k - epoch * S;

  RPH_DASSERT(d.batch > 0 && k >= 0 && epoch * d.steps_per_epoch <= k && d.lag != nullptr);
  // ---- prologue: every load independent, issued together -----------------------
  RPH_STAMP(0);
  // kernel 0 starts from the fit-state template (and workgroup 0 publishes it
  // as the canonical FitState below); later kernels see that copy
  const FitState* fit0 = (k == 0 && d.fit_init != nullptr) ? d.fit_init : d.fit;
  const float stopped0 = fit0->stopped;
  LagState<P> st;
  lag_load<P>(st, d, k == 0 ? nullptr : d.lag + (size_t)(k & 1) * LAG_FLOATS, fit0);
  typename B::Pre pre;
  B::load(d, s, perm, B::first(wid), lane, pre);
  prefetch_kernarg_end(kat);
  const bool dp = d.dp_world > 1;
  const float* prev = d.acc + (size_t)((k + 2) % 3) * LAG_SLOTS * R;  // accumulator of step k-1
  if (k > 0 && !dp) lag_sums<R, NREP, B::ACC_PLAIN>(prev, red);
  if (stopped0 != 0.f) return;  // early-stopped fit: the remaining steps are no-ops
  __syncthreads();
  const bool w0 = blockIdx.x == 0;
  if (k > 0 && dp && lag_dp_exchange<R, NREP>(d, __float_as_uint(st.sc[LG_SEQ]) + (uint32_t)k, prev, red, w0))
    return;  // a peer timed out (dp_error is set; the host raises)
  RPH_STAMP(1);
  if (k > 0) {
    const int kp = k - 1;
    const int ep = kp / S;
    int ep_done = ep;
    if (lag_apply<P>(st, red, d, ep, kp - ep * S, w0, ep_done)) {
      if (w0) {
        lag_store_canonical<P>(st, d, 1.f, ep_done);
        lag_advance_seq(d, st.sc[LG_SEQ], (uint32_t)k);
      }
      return;
    }
  }
#pragma unroll
  for (int j = 0; j < LagState<P>::NPT; ++j)
    if (tid + 256 * j < P) wl[tid + 256 * j] = st.w[j];
  if (w0) {
    if (k == 0 && d.fit_init != nullptr) {  // canonical FitState := template (read by kernels >= 1)
      const float* src = (const float*)d.fit_init;
      float* dst = (float*)d.fit;
      for (int i = tid; i < FIT_FLOATS; i += 256) dst[i] = src[i];
    }
    // persist the updated state and re-arm the accumulator of step k+1 now, so
    // no optimizer state stays live (in registers) across the partial
    float* z = d.acc + (size_t)((k + 1) % 3) * LAG_SLOTS * R;
    for (int i = tid; i < NREP * R; i += 256) st_agent(z + i, 0.f);
    lag_store<P>(st, d.lag + (size_t)((k + 1) & 1) * LAG_FLOATS);
  }
  __syncthreads();
  RPH_STAMP(2);
  typename B::Frags fr;
  B::make_frags(wl + B::S::OW2, fr);
  float val[NR];
  B::partial(d, s, perm, wl, fr, scratch, pre, val);
  RPH_STAMP(3);

  // ---- epilogue: fire-and-forget adds ----------------------------------------------
  float* buf = d.acc + (size_t)(k % 3) * LAG_SLOTS * R;
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int i = tid + 256 * j;
    if (i < R)
      __hip_atomic_fetch_add(buf + (blockIdx.x % NREP) * R + i, val[j], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
  RPH_STAMP(4);
}

// Update of the last step + canonical write-back.  One workgroup.
template <int P, int R, int NREP>
__global__ __launch_bounds__(256) void k_hedge_lag_finalize(const TrainDesc d, const int K) {
  prefetch_kernarg<sizeof(TrainDesc) + sizeof(int)>();
  __shared__ __attribute__((aligned(16))) float red[((R + 255) / 256) * 256 + 8];
  const bool run = d.fit->stopped == 0.f && K > 0;
  LagState<P> st;
  int bad = 0;
  if (run) {
    lag_load<P>(st, d, d.lag + (size_t)(K & 1) * LAG_FLOATS, d.fit);
    const float* prev = d.acc + (size_t)((K - 1) % 3) * LAG_SLOTS * R;
    if (d.dp_world > 1) {
      bad = lag_dp_exchange<R, NREP>(d, __float_as_uint(st.sc[LG_SEQ]) + (uint32_t)K, prev, red, true);
    } else {
      lag_sums<R, NREP>(prev, red);
    }
  }
  // leave all three accumulators zeroed for the next fit (its kernel 0 adds
  // into accumulator 0 without a memset); every lag kernel of this fit is done
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * LAG_SLOTS * R; i += 256) st_agent(d.acc + i, 0.f);
  if (!run || bad) return;
  // diagnostics (TrainConfig.expose_packet): the summed - and, data parallel,
  // exchanged - packet of the last step, as every rank applies it
  if (d.grad_out != nullptr)
    for (int i = threadIdx.x; i < R; i += 256) d.grad_out[i] = red[i];
  const int S = d.steps_per_epoch;
  const int kp = K - 1, ep = kp / S;
  int ep_done = ep;
  const int stop = lag_apply<P>(st, red, d, ep, kp - ep * S, true, ep_done);
  // (a fit whose last launched step does not close an epoch keeps stopped = 0)
  lag_store_canonical<P>(st, d, stop ? 1.f : 0.f, ep_done);
  lag_advance_seq(d, st.sc[LG_SEQ], (uint32_t)K);
}

}  // namespace rph
