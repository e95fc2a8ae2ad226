// rphedge — persistent training kernel: ONE launch per Keras fit() (K9+K10 fused
// over all epochs and steps).
//
// Reference semantics: model.fit(X1, y, epochs, batch_size, callbacks=[
// EarlyStopping(monitor='loss', patience, restore_best_weights=True),
// LearningRateScheduler]) — Replicating_Portfolio.py:200-209.
//
// Why: the per-step kernel (k_hedge_train_step) pays a kernel boundary per
// optimizer step — dispatch, cache write-back/invalidate, re-loading the
// weights and optimizer state, and a serial "last arriver updates, next
// kernel re-reads" chain.  At the flagship batch that fixed cost is ~2/3 of
// the step.  Here every workgroup stays resident for the whole fit:
//
//   per step:  partial packet (Body::partial, same code as the step kernels)
//              -> float atomics into one of 3 rotating accumulator buffers
//              -> arrival counter (monotonic, agent scope)
//              -> wait until all G workgroups arrived
//              -> EVERY workgroup reads the summed packet and applies the same
//                 Keras-Adam update to its own register/LDS copy of the weights
//                 (identical inputs, identical code => identical weights and
//                 identical early-stopping decisions in every workgroup; no
//                 weight broadcast, no second barrier)
//   buffer (step+2)%3 is re-zeroed by the last arriver of step `step`; every
//   read of it (step-1) precedes every arrival at `step`, and every add into
//   it (step+2) follows the last arriver's arrival at step+1.
//
// Co-residency: the grid is sized to the occupancy-limited number of resident
// workgroups (launcher); every wait is bounded by wall-clock (s_memrealtime)
// and raises ctl[1] (checked by the host), so a non-resident grid ends instead
// of hanging.  Workgroup 0 writes the final weights / optimizer / early-stop
// state back in the layout the step kernels use, so both paths interoperate.
#pragma once
#include "hedge_core.h"

namespace rph {

constexpr unsigned long long FIT_SPIN_TICKS = 200000000ull;  // 2 s at 100 MHz

RPH_INLINE uint32_t ld_agent_u32(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


template <class B>
__global__ __launch_bounds__(256) void k_hedge_fit(const TrainDesc d, const int epochs) {
  constexpr int P = B::P;
  constexpr int R = B::R;
  constexpr int NR = B::NR;
  constexpr int NPT = (P + 255) / 256;
  __shared__ __attribute__((aligned(16))) float scratch[B::SCRATCH_FLOATS];
  __shared__ __attribute__((aligned(16))) float wl[P + 4];
  __shared__ __attribute__((aligned(16))) float red[NR * 256 + 8];
  __shared__ int s_last, s_bad;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const uint32_t G = gridDim.x;
  uint32_t* arrivals = d.counter;   // ctl[0]: zeroed by the host before the launch
  uint32_t* err = d.counter + 1;    // ctl[1]: co-residency / timeout error

  // ---- state -> registers / LDS ----------------------------------------------
  float w[NPT], m[NPT], v[NPT], wb[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int i = tid + 256 * k;
    const bool ok = i < P;
    w[k] = ok ? d.wts->w[0][i] : 0.f;
    m[k] = ok ? d.opt->m[i] : 0.f;
    v[k] = ok ? d.opt->v[i] : 0.f;
    wb[k] = ok ? d.fit->w_best[i] : 0.f;
  }
  const OptState* o = d.opt;
  const FitState* f = d.fit;
  float t = o->t, lr = o->lr, nan_steps = o->nan_steps;
  const float b1 = o->beta1, b2 = o->beta2, eps = o->eps;
  const float lb1 = __builtin_amdgcn_logf(b1), lb2 = __builtin_amdgcn_logf(b2);
  float best = f->best_loss, wait = f->wait, has_best = f->has_best, stopped = f->stopped;
  const float patience = f->patience, max_epochs = f->max_epochs, restore_best = f->restore_best,
              restore_at_end = f->restore_at_end;
  float loss_sum = f->loss_sum, abs_sum = f->abs_sum, ape_sum = f->ape_sum, loss_cnt = f->loss_cnt;
  float last_L = f->last_loss, last_mae = f->last_mae, last_mape = f->last_mape;
  int ep_done = (int)f->epoch;
  const bool dp = d.dp_world > 1;
  // per-rank DP step sequence (read by every workgroup before the first
  // barrier; workgroup 0 advances it after the last one)
  const uint32_t seq0 = dp ? ld_agent_u32(d.dp_counter) : 0u;
  if (stopped != 0.f) return;
#pragma unroll
  for (int k = 0; k < NPT; ++k)
    if (tid + 256 * k < P) wl[tid + 256 * k] = w[k];
  __syncthreads();

  const uint32_t n_chunks = (uint32_t)((d.n_local + (1 << d.chunk_log2) - 1) >> d.chunk_log2);
  const int S = d.steps_per_epoch;
  // diagnostic stamps of the most recent step: 0 start, 1 partial done, 2 adds
  // drained, 3 all arrived (thread 0), 4 sums read, 5 update done
#define FIT_STAMP(k) \
  if (d.stamps != nullptr && tid == 0) d.stamps[(size_t)blockIdx.x * 8 + (k)] = rph_stamp_clock()
  uint32_t gstep = 0;  // steps started (rotating buffers, barrier targets)
  uint32_t done = 0;   // steps completed (DP sequence)
  bool bad = false;
  // first path(s) of the next step are loaded BEFORE the barrier of the
  // current one (they do not depend on the weights), hiding their latency
  typename B::Pre pre;
  {
    const Perm p0 = make_perm(n_chunks, d.seed, (uint32_t)ep_done, d.shuffle != 0);
    B::load(d, 0, p0, B::first(wid), lane, pre);
  }
  for (int e = ep_done; e < epochs && !bad; ++e) {
    const Perm perm = make_perm(n_chunks, d.seed, (uint32_t)e, d.shuffle != 0);
    if (d.lr_sched != nullptr) {  // LearningRateScheduler.on_epoch_begin (NaN => keep)
      const float s = d.lr_sched[e];
      if (s == s) lr = s;
    }
    for (int s = 0; s < S; ++s, ++gstep) {
      FIT_STAMP(0);
      typename B::Frags fr;
      B::make_frags(wl + B::S::OW2, fr);
      float val[NR];
      B::partial(d, s, perm, wl, fr, scratch, pre, val);
      FIT_STAMP(1);
      if (s + 1 < S) {
        B::load(d, s + 1, perm, B::first(wid), lane, pre);
      } else if (e + 1 < epochs) {
        const Perm pn = make_perm(n_chunks, d.seed, (uint32_t)(e + 1), d.shuffle != 0);
        B::load(d, 0, pn, B::first(wid), lane, pre);
      }

      // ---- publish + arrive + wait ---------------------------------------------
      float* buf = d.acc + (size_t)(gstep % 3u) * ACC_REPLICAS * R;
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        const int i = tid + 256 * k;
        if (i < R)
          __hip_atomic_fetch_add(buf + (blockIdx.x % ACC_REPLICAS) * R + i, val[k], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every adding wave drains before the arrival
      __syncthreads();
      FIT_STAMP(2);
      if (tid == 0) {
        const uint32_t target = (gstep + 1u) * G;
        const uint32_t tk = __hip_atomic_fetch_add(arrivals, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
        int b = 0;
        if (tk != target) {
          const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
          unsigned it = 0;
          while (ld_agent_u32(arrivals) < target) {
            __builtin_amdgcn_s_sleep(1);
            if ((++it & 255u) == 0u &&
                (ld_agent_u32(err) != 0u || __builtin_amdgcn_s_memrealtime() - t0 > FIT_SPIN_TICKS)) {
              __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              b = 1;
              break;
            }
          }
        }
        s_last = (tk == target) ? 1 : 0;
        s_bad = b;
      }
      FIT_STAMP(3);
      __syncthreads();
      if (s_bad) {
        bad = true;
        break;
      }

      // ---- summed packet (bitwise identical in every workgroup) ----------------
      if (!dp) {
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          const int i = tid + 256 * k;
          if (i < R) red[i] = sum_replicas(buf, R, i);
        }
      } else {
        // data parallel: this rank's last arriver pushes the local sum into every
        // rank's IPC mailbox (system-scope stores over xGMI) and raises one flag
        // per peer; EVERY workgroup of every rank then waits for the W flags of
        // this step and sums the W packets in fixed rank order (identical
        // everywhere).  A peer can be at most one step ahead, so the DP_SLOTS-deep
        // slot of `seq` is never overwritten while it is read.
        const uint32_t seq = seq0 + gstep + 1u;
        const int slot = (int)(seq % DP_SLOTS);
        const int W = d.dp_world, me = d.dp_rank;
        if (s_last) {
#pragma unroll
          for (int k = 0; k < NR; ++k) {
            const int i = tid + 256 * k;
            if (i < R) {
              const float vloc = sum_replicas(buf, R, i);
              for (int p = 0; p < W; ++p)
                __hip_atomic_store(d.dp_mbox[p] + ((size_t)slot * W + me) * R + i, vloc, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            }
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          if (tid < W)
            __hip_atomic_store(d.dp_flags[tid] + slot * W + me, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        int b = 0;
        if (tid < W) {
          const uint32_t* fl = d.dp_flags[me] + slot * W + tid;
          const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
          unsigned it = 0;
          while (__hip_atomic_load(const_cast<uint32_t*>(fl), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
            __builtin_amdgcn_s_sleep(1);
            if ((++it & 255u) == 0u && __builtin_amdgcn_s_memrealtime() - t0 > FIT_SPIN_TICKS) {
              __hip_atomic_store(d.dp_error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              b = 1;
              break;
            }
          }
        }
        if (__syncthreads_or(b)) {
          bad = true;
          break;
        }
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          const int i = tid + 256 * k;
          if (i < R) {
            float a = 0.f;
            for (int p = 0; p < W; ++p)
              a += __hip_atomic_load(d.dp_mbox[me] + ((size_t)slot * W + p) * R + i, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_SYSTEM);
            red[i] = a;
          }
        }
      }
      if (s_last) {  // re-zero the buffer of step gstep+2 (last read at gstep-1)
        float* z = d.acc + (size_t)((gstep + 2u) % 3u) * ACC_REPLICAS * R;
        for (int i = tid; i < ACC_REPLICAS * R; i += 256) st_agent(z + i, 0.f);
      }
      __syncthreads();
      FIT_STAMP(4);

      // ---- Keras Adam (NaN/Inf guard) -----------------------------------------
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
        t += 1.f;
        const float bc1 = 1.f - __builtin_amdgcn_exp2f(t * lb1);
        const float bc2 = 1.f - __builtin_amdgcn_exp2f(t * lb2);
        const float lr_t = lr * sqrtf(bc2) * __frcp_rn(bc1);
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          m[k] = m[k] + (g[k] - m[k]) * (1.f - b1);
          v[k] = v[k] + (g[k] * g[k] - v[k]) * (1.f - b2);
          if (tid + 256 * k < P) w[k] = w[k] - lr_t * m[k] * __frcp_rn(sqrtf(v[k]) + eps);
        }
      } else {
        nan_steps += 1.f;
      }
      loss_sum += red[P + 0];
      abs_sum += red[P + 1];
      ape_sum += red[P + 2];
      loss_cnt += red[P + 3];

      // ---- EarlyStopping.on_epoch_end -----------------------------------------
      if (s == S - 1) {
        const float cnt = fmaxf(loss_cnt, 1.f);
        const float L = loss_sum * __frcp_rn(cnt);
        int act = 0;
        wait += 1.f;
        if (L < best || has_best == 0.f) {
          if (L < best) {
            best = L;
            wait = 0.f;
          }
          act = 1;
        }
        if (wait >= patience && e > 0) {
          stopped = 1.f;
          if (restore_best != 0.f) act = 2;
        }
        if ((float)(e + 1) >= max_epochs && stopped == 0.f) {
          stopped = 1.f;
          if (restore_best != 0.f && restore_at_end != 0.f) act = 2;
        }
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          if (act == 1) wb[k] = w[k];
          if (act == 2) w[k] = wb[k];
        }
        if (blockIdx.x == 0 && tid == 0 && e < MAXHIST) d.fit->hist[e] = L;
        last_L = L;
        last_mae = abs_sum * __frcp_rn(cnt);
        last_mape = 100.f * ape_sum * __frcp_rn(cnt);
        loss_sum = abs_sum = ape_sum = loss_cnt = 0.f;
        has_best = 1.f;
        ep_done = e + 1;
      }
#pragma unroll
      for (int k = 0; k < NPT; ++k)
        if (tid + 256 * k < P) wl[tid + 256 * k] = w[k];
      __syncthreads();
      ++done;
      FIT_STAMP(5);
      if (stopped != 0.f) break;
    }
    if (stopped != 0.f) break;
  }
#undef FIT_STAMP

  // ---- write back (workgroup 0): the layout the step kernels read --------------
  if (blockIdx.x != 0 || bad) return;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int i = tid + 256 * k;
    if (i < P) {
      d.wts->w[0][i] = w[k];
      d.opt->m[i] = m[k];
      d.opt->v[i] = v[k];
      d.fit->w_best[i] = wb[k];
    }
  }
  if (tid == 0) {
    if (dp) __hip_atomic_store(d.dp_counter, seq0 + done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    d.opt->t = t;
    d.opt->lr = lr;
    d.opt->nan_steps = nan_steps;
    FitState* fs = d.fit;
    fs->best_loss = best;
    fs->wait = wait;
    fs->has_best = has_best;
    fs->stopped = stopped;
    fs->epoch = (float)ep_done;
    fs->loss_sum = loss_sum;
    fs->abs_sum = abs_sum;
    fs->ape_sum = ape_sum;
    fs->loss_cnt = loss_cnt;
    fs->last_loss = last_L;
    fs->last_mae = last_mae;
    fs->last_mape = last_mape;
  }
}

// Launch with the grid clamped to the resident capacity of the device.
template <class B>
int launch_fit(const TrainDesc* d, int epochs, hipStream_t s) {
  static int cap = 0;
  if (cap == 0) {
    int dev = 0, cus = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -2;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -2;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_hedge_fit<B>, 256, 0) != hipSuccess) return -2;
    cap = (nb > 0 ? nb : 1) * cus;
  }
  const int G = d->num_wgs < cap ? d->num_wgs : cap;
  hipLaunchKernelGGL((k_hedge_fit<B>), dim3(G), dim3(256), 0, s, *d, epochs);
  return (int)hipGetLastError();
}

int launch_wide_fit(const TrainDesc* d, int epochs, hipStream_t s);
int launch_wide_lag_step(const TrainDesc* d, int k, int epoch, const Perm& perm, hipStream_t s);

}  // namespace rph
