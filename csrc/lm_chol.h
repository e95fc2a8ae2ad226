// rphedge — fp64 Cholesky solve of the Levenberg-Marquardt system on ONE
// workgroup of gfx950 (k_lm_solve): tile store + panel wave + owner waves.
//
// The augmented matrix M = [[A, .], [b^T, 1]] (A = 2G + damping, P x P; b = -g
// as row P) is cut into 16 x 16 tiles (lower triangle, NT x NT tile grid
// padded with identity rows).  Its Cholesky factor's last row is y = L^-1 b,
// so the forward solve rides along; the backward solve L^T d = y follows.
//
//  * owner waves 1..3 keep every lower tile in fp64 MFMA accumulator
//    registers (tile t -> wave 1 + t % 3, column-major order: the tiles still
//    active at panel K are a suffix, so the owners stay balanced) and apply
//    the rank-16 trailing update of panel K with v_mfma_f64_16x16x4_f64
//    (4 per tile), the next panel's column block FIRST (look-ahead), which
//    they publish to the LDS tile store before updating the rest;
//  * the panel wave 0 takes each published 16-column panel (one or more rows
//    per lane), factors it column by column (the pivot by v_readlane, its
//    reciprocal square root from v_rsq_f64 + one Newton step, the column
//    broadcast through LDS), writes L back to the store and signals.
// Panel and owner waves hand off through LDS counters (workgroup-scope
// release / acquire, bounded spins): no workgroup barrier inside the loop.
// The store swizzles the columns of each tile row by 2 * (row >> 1), so the
// owners' MFMA fragment reads (16 rows x 2 columns per half-wave) and the
// panel wave's row reads (ds_read_b128) are free of bank conflicts.
#pragma once
#include "rph_common.h"

namespace rph {

typedef double lmc_d4 __attribute__((ext_vector_type(4)));

template <int P>
struct TileGrid {
  static constexpr int PR = P + 1;              // rows: the system + the right-hand side
  static constexpr int NT = (PR + 15) / 16;     // tile rows / columns
  static constexpr int PT = 16 * NT;
  static constexpr int NK = (P + 15) / 16;      // panels (columns < P are factored)
  static constexpr int NTILE = NT * (NT + 1) / 2;
  static constexpr int NSLOT = (PT + 63) / 64;  // panel rows per lane of the panel wave
  static constexpr int NOWN = 3;                // owner waves
  static constexpr int TPW = (NTILE + NOWN - 1) / NOWN;
  static constexpr int NBG = (P + 31) / 32;     // 32 x 32 Gram blocks per row (k_lm_reduce layout)
  // dynamic LDS (doubles): tile store | d [PT] | 1/L_kk [PT] | column broadcast [2][16]; the damped
  // diagonal shares d's slot (read by the owners' initial loads only, d written by the backward
  // solve after the last panel), so the 6-asset net (P = 191, 78 tiles) fits the 160 KB
  static constexpr int OFF_D = NTILE * 256;
  static constexpr int OFF_DIAG = OFF_D;
  static constexpr int OFF_RDG = OFF_D + PT;
  static constexpr int OFF_BC = OFF_RDG + PT;
  // the inverses of the diagonal blocks 0..NK-2 of L (owners, after their
  // last update), for the backward solve - the nets with up to 48 tiles
  static constexpr int NX = NTILE <= 48 ? NK - 1 : 0;
  static constexpr int OFF_X = OFF_BC + 32;
  static constexpr int OFF_FLAGS = OFF_X + NX * 256;  // (as unsigned) pub[NT + 1], fac[NT + 1], xdone
  static constexpr int LDS_BYTES = OFF_FLAGS * 8 + 2 * (NT + 1) * 4 + 16;
  // lower tile t (column-major) <-> (row block, column block)
  static constexpr int tidx(int ib, int jb) { return jb * NT - jb * (jb - 1) / 2 + (ib - jb); }
  static constexpr int tcol(int t) {
    int b = 0;
    while (t >= NT - b) t -= NT - b++;
    return b;
  }
  static constexpr int trow(int t) {
    int b = 0;
    while (t >= NT - b) t -= NT - b++;
    return b + t;
  }
};

// element (r, c) of a tile -> double offset inside the tile
RPH_INLINE int tg_off(int r, int c) { return r * 16 + (c ^ ((r >> 1) << 1)); }

// fp64 reciprocal square root: v_rsq_f64 (rel. err 5.2e-8) + one Newton step
RPH_INLINE double lmc_rsq(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  return y * __builtin_fma(-0.5 * x * y, y, 1.5);
}

RPH_INLINE double lmc_readlane(double v, int l) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// Gram entry G[i][j] (symmetric) from the reduced block: upper-triangular
// 32 x 32 blocks in MFMA register order (k_lm_reduce / k_lm_pass layout)
template <int NBG>
RPH_INLINE double lmc_gram(const double* src, int i, int j) {
  const int lo = i < j ? i : j, hi = i < j ? j : i;  // row lo, column hi of the upper triangle
  const int mb = lo >> 5, nb = hi >> 5;
  const int b = mb * NBG - (mb * (mb - 1)) / 2 + (nb - mb);
  const int jj = lo & 31;
  const int q = (jj & 3) + 4 * (jj >> 3), h = (jj >> 2) & 1;
  return src[(size_t)b * 1024 + q * 64 + h * 32 + (hi & 31)];
}

RPH_INLINE void lmc_signal(unsigned* flag) {
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// LDS hand-off between the lanes of ONE wave (a lane reads what other lanes
// just stored): no instruction is needed (a wave's LDS operations complete in
// order), but the compiler must not forward a value loaded before the stores
// to a load after them - for the lanes that did not store, its single-thread
// view says the memory is unchanged.  A wavefront-scope fence forbids that.
RPH_INLINE void lmc_wave_sync() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }

// bounded wait for *flag >= target (one wave); false on timeout
RPH_INLINE bool lmc_wait(const unsigned* flag, unsigned target) {
  for (unsigned it = 0; it < (1u << 24); ++it) {
    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) return true;
    __builtin_amdgcn_s_sleep(0);
  }
  return false;
}

// The whole workgroup copies the strictly lower Gram entries (x2) into the
// tile store before the setup barrier (the rhs row follows it): the Gram block is read
// in its own order (each 64-lane load one contiguous 512-byte run), where the
// owners' accumulator-order loads touch 16 cache lines per instruction
template <int P>
RPH_INLINE void lmc_stage(double* T, const double* src) {
  using TG = TileGrid<P>;
  constexpr int NBG = TG::NBG, NBLK = NBG * (NBG + 1) / 2;
  constexpr int NIT = NBLK * 4;  // 256 threads x 4 = one 32 x 32 block
  constexpr int CH = NIT;        // every load in flight before the first store (one round trip)
  const int tid = threadIdx.x;
  lm_static_for<(NIT + CH - 1) / CH>([&](auto cc) {
    constexpr int I0 = decltype(cc)::value * CH;
    double v[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (I0 + u < NIT) v[u] = src[(I0 + u) * 256 + tid];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int it = I0 + u;
      if (it < NIT) {
        const int b = it >> 2, e = (it & 3) * 256 + tid;
        int mb = 0, rem = b;  // block b -> (mb, nb), upper triangle row-major (lmc_gram)
        while (rem >= NBG - mb) rem -= NBG - mb++;
        const int nb = mb + rem;
        const int q = e >> 6, h = (e >> 5) & 1;
        const int lo = 32 * mb + (q & 3) + 4 * h + 8 * (q >> 2), hi = 32 * nb + (e & 31);
        if (lo < hi && hi < P) T[TG::tidx(hi >> 4, lo >> 4) * 256 + tg_off(hi & 15, lo & 15)] = 2.0 * v[u];
      }
    }
  });
}

// Owner wave O (0..2): its tiles are t = O + 3 j (compile-time), so every
// register index is static.
template <int P, int O>
struct LmcOwner {
  using TG = TileGrid<P>;
  static constexpr int TPW = TG::TPW;

  // initial tiles from the Gram block (x2), damped diagonal, rhs row, identity padding
  RPH_INLINE static void load(lmc_d4* C, const double* src, const double* diag, const double* g, int lr, int lq) {
    lm_static_for<TPW>([&](auto jc) {
      constexpr int j = decltype(jc)::value, t = O + 3 * j;
      if constexpr (t < TG::NTILE) {
        constexpr int ib = TG::trow(t), jb = TG::tcol(t);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * ib + lq + 4 * r, c = 16 * jb + lr;
          // every load unconditional (clamped, in bounds): a per-element
          // branch around the load would wait out each one separately
          const int ic = i < P ? i : P - 1, cc = c < P ? c : P - 1;
          const double gv = lmc_gram<TG::NBG>(src, ic, cc), gr = g[cc], dg = diag[ic];
          double v;
          if (i < P && c < P) v = i == c ? dg : (c < i ? 2.0 * gv : 0.0);
          else if (i == P && c < P) v = -gr;
          else v = i == c ? 1.0 : 0.0;
          C[j][r] = v;
        }
      }
    });
  }

  // the same tiles from the store, where lmc_stage put the strictly lower
  // Gram entries (x2) and the rhs row: LDS reads only
  RPH_INLINE static void load_staged(lmc_d4* C, const double* T, const double* diag, int lr, int lq) {
    lm_static_for<TPW>([&](auto jc) {
      constexpr int j = decltype(jc)::value, t = O + 3 * j;
      if constexpr (t < TG::NTILE) {
        constexpr int ib = TG::trow(t), jb = TG::tcol(t);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * ib + lq + 4 * r, c = 16 * jb + lr;
          const int ic = i < P ? i : P - 1;
          const double tv = T[t * 256 + tg_off(lq + 4 * r, lr)], dg = diag[ic];
          double v;
          if (i < P && c < P) v = i == c ? dg : (c < i ? tv : 0.0);
          else if (i == P && c < P) v = tv;
          else v = i == c ? 1.0 : 0.0;
          C[j][r] = v;
        }
      }
    });
  }

  // publish the tiles of column block jb (their current values) to the store
  RPH_INLINE static void publish(const lmc_d4* C, double* T, int jbk, int lr, int lq) {
    lm_static_for<TPW>([&](auto jc) {
      constexpr int j = decltype(jc)::value, t = O + 3 * j;
      if constexpr (t < TG::NTILE) {
        constexpr int jb = TG::tcol(t);
        if (jb == jbk) {
#pragma unroll
          for (int r = 0; r < 4; ++r) T[t * 256 + tg_off(lq + 4 * r, lr)] = C[j][r];
        }
      }
    });
  }

  // C -= L(ib, K) L(jb, K)^T for the tiles with column block in [jlo, jhi]
  RPH_INLINE static void update(lmc_d4* C, const double* T, int K, int jlo, int jhi, int lr, int lq) {
    lm_static_for<TPW>([&](auto jc) {
      constexpr int j = decltype(jc)::value, t = O + 3 * j;
      if constexpr (t < TG::NTILE) {
        constexpr int ib = TG::trow(t), jb = TG::tcol(t);
        if (jb >= jlo && jb <= jhi) {
          const double* Ta = T + TG::tidx(ib, K) * 256;
          const double* Tb = T + TG::tidx(jb, K) * 256;
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const int o = tg_off(lr, 4 * s + lq);
            C[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(-Ta[o], Tb[o], C[j], 0, 0, 0);
          }
        }
      }
    });
  }

  // the inverse of the diagonal blocks K = O + 3 s (< NX) of L: lanes 16 s + c
  // compute column c by forward substitution (in-lane chains, the L entries
  // as LDS broadcasts) -> X[K][i][c]
  RPH_INLINE static void invert(const double* T, const double* rdg, double* X, int lane) {
#pragma clang fp contract(off)
    const int s = lane >> 4, c = lane & 15, K = O + 3 * s;
    if (K < TG::NX) {
      const double* Lt = T + TG::tidx(K, K) * 256;
      double x[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        double s0 = i == c ? 1.0 : 0.0, s1 = 0.0;
#pragma unroll
        for (int k = 0; k < i; ++k) {
          const double l = Lt[tg_off(i, k)];
          if (k & 1) s1 = __builtin_fma(-l, x[k], s1);
          else s0 = __builtin_fma(-l, x[k], s0);
        }
        x[i] = (s0 + s1) * rdg[16 * K + i];
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) X[K * 256 + i * 16 + c] = x[i];
    }
  }

  // STAGED: the tiles from the store (lmc_stage), else from the Gram block
  template <bool STAGED>
  RPH_INLINE static void run(const double* src, const double* diag, const double* g, double* T, unsigned* pub,
                             const unsigned* fac, int* s_fail, const double* rdg, double* X, unsigned* xdone) {
    const int lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
    lmc_d4 C[TPW];
    if constexpr (STAGED) load_staged(C, T, diag, lr, lq);
    else load(C, src, diag, g, lr, lq);
    publish(C, T, 0, lr, lq);
    lmc_signal(&pub[0]);
    bool ok = true;
    for (int K = 0; K + 1 < TG::NK; ++K) {
      if (!lmc_wait(&fac[K], 1u)) {
        *s_fail = 2;
        ok = false;
        break;
      }
      update(C, T, K, K + 1, K + 1, lr, lq);  // look-ahead: the next panel's column block
      publish(C, T, K + 1, lr, lq);
      lmc_signal(&pub[K + 1]);
      update(C, T, K, K + 2, TG::NT - 1, lr, lq);
    }
    // idle from here (the last panel is the panel wave's): the diagonal blocks'
    // inverses for the backward solve (signalled even after a failure, so the
    // backward never waits out its bound)
    if constexpr (TG::NX > 0) {
      if (ok) invert(T, rdg, X, lane);
      lmc_signal(xdone);
    }
  }
};

// Panel wave: factor the NK panels; L (lower, zero above the diagonal) to
// the store, 1 / L_kk to rdg.
// diagnostic stamps (row of d.stamps, thread 0 = lane 0 of the panel wave;
// tools/stamp_lm.py): 0/1 panel 0 wait passed / written back, 2/3 panel 1,
// 4/5 last panel, 6 its rows loaded, 7 its columns factored
#define LMC_STAMP(k)                                                                    \
  do {                                                                                  \
    if (stamps != nullptr && lane == 0) stamps[k] = rph_stamp_clock();               \
  } while (0)

// row_newbcast:J (gfx90a+ 64-bit DPP): every lane of each 16-lane row gets
// lane J of that row's v - one v_mov_b64_dpp, no SGPR or LDS round trip
template <int J>
RPH_INLINE double lmc_bcast(double v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + J, 0xF, 0xF, true);
}

// acc += row_newbcast:J(s0) * (-s1): v_fmac_f64_dpp (gfx90a+ DPP on a 64-bit
// VOP2 op) - the broadcast rides in the fma, one instruction per update and no
// dependent mov.  The same single rounding as fma(-s1, bcast(s0), acc).  (The
// compiler's hazard recognizer sees the inline DPP: it pads a VALU write of
// s0 right before it.)
template <int J>
RPH_INLINE void lmc_fmac_bcast(double& acc, double s0, double s1) {
  asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(acc)
               : "v"(s0), "v"(s1), "i"(J));
}

// A 16-row tile row (16 doubles) from the store / to the store (swizzled columns)
RPH_INLINE void lmc_load_row(double (&a)[16], const double* tr, int r) {
  const int sw = (r >> 1) << 1;
#pragma unroll
  for (int c = 0; c < 16; c += 2) {
    const double2 v = *reinterpret_cast<const double2*>(tr + (c ^ sw));
    a[c] = v.x;
    a[c + 1] = v.y;
  }
}

template <int P>
RPH_INLINE void lmc_panels(double* T, double* rdg, double* bc, const unsigned* pub, unsigned* fac, int* s_fail,
                           unsigned long long* stamps) {
#pragma clang fp contract(off)
  using TG = TileGrid<P>;
  const int lane = threadIdx.x & 63, li = lane & 15;
  (void)bc;
  bool ok = true, alive = true;
  // Register layout of panel K: every 16-lane DPP row holds a replica of the
  // diagonal tile (lane 16 r + i: its row i in dk[]), and the panel rows
  // below it are spread over all 64 lanes (row 16K + 16 + lane + 64 s in
  // a[s][]).  Column c's entries L[16K + j][16K + c] of the diagonal tile are
  // then one row_newbcast:j away from every lane (lmc_bcast): the pivot, the
  // column scale and every trailing update of the panel are in-register -
  // no v_readlane / SGPR hazard and no LDS round trip per column.  The fma
  // sequence applied to every entry is the same as a serial right-looking
  // Cholesky (bitwise the previous readlane / LDS-broadcast panel).
  // Every panel is its own straight-line code (static column count, static
  // row slots): the column chain of one panel is a single basic block, so the
  // next column's pivot chain overlaps this column's trailing updates.
  lm_static_for<TG::NK>([&](auto kc) {
    constexpr int K = decltype(kc)::value;
    constexpr int NC = P - 16 * K < 16 ? P - 16 * K : 16;  // factored columns
    constexpr int OFF = TG::PT - 16 * K - 16;              // panel rows below the diagonal tile
    constexpr int NS = (OFF + 63) / 64;                    // their row slots per lane
    if (!alive) return;
    if (!lmc_wait(&pub[K], 3u)) {
      *s_fail = 2;
      alive = false;
      return;
    }
    if constexpr (K < 2) LMC_STAMP(2 * K);
    else if constexpr (K == TG::NK - 1) LMC_STAMP(4);
    double dk[16];
    lmc_load_row(dk, T + TG::tidx(K, K) * 256 + li * 16, li);
    // (a lane past the last panel row duplicates row o % OFF: it computes and
    // stores exactly that row's values, so loads and stores need no branch -
    // a conditional store would let the compiler sink the row updates into
    // it, keeping every broadcast alive until then)
    double a[NS > 0 ? NS : 1][16];
    int arow[NS > 0 ? NS : 1];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int o = lane + 64 * s;
      arow[s] = 16 * K + 16 + (o < OFF ? o : o % (OFF > 0 ? OFF : 1));
      lmc_load_row(a[s], T + TG::tidx(arow[s] >> 4, K) * 256 + (arow[s] & 15) * 16, arow[s] & 15);
    }
    if constexpr (K == TG::NK - 1) LMC_STAMP(6);
    // column c's block: scale column c, then the dependent chain of column
    // c + 1 (its update by column c, its pivot, v_rsq_f64 + the Newton step:
    // seven dependent fp64 operations) in seven stages, each followed by a
    // share of column c's remaining updates (independent of the chain) and a
    // scheduling barrier - the wave issues in order, so the updates fill the
    // chain's latencies instead of following it; only one column's broadcasts
    // are live at a time (no spills).  Same operations as lmc_rsq.
    double piv = lmc_bcast<0>(dk[0]);
    double rl = lmc_rsq(piv);
    double myrl = 0.0;  // lane i < NC of every DPP row: 1 / L[16K + i][16K + i]
    lm_static_for<NC>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      constexpr int NU = NC - c - 2 > 0 ? NC - c - 2 : 0;  // remaining updates j = c + 2 .. NC - 1
      constexpr int NST = 7;                                // chain stages
      ok = ok && piv > 0.0;
      dk[c] *= rl;  // lane i: L[16K + i][16K + c] (i >= c)
#pragma unroll
      for (int s = 0; s < NS; ++s) a[s][c] *= rl;
      myrl = li == c ? rl : myrl;
      // the inline v_fmac_f64_dpp below read dk[c] through DPP: two wait
      // states after its VALU write whatever the hazard recognizer assumes
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_nop 1");
      // updates of columns c + 2 + [lo, hi) by column c
      auto updates = [&](auto lo_c, auto hi_c) {
        constexpr int LO = decltype(lo_c)::value, HI = decltype(hi_c)::value;
        lm_static_for<NC>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          if constexpr (j >= c + 2 + LO && j < c + 2 + HI) {
            // x -= L[16K + j][16K + c] x_c: the broadcast of lane j's dk[c] inside the fma
            lmc_fmac_bcast<j>(dk[j], dk[c], dk[c]);
#pragma unroll
            for (int s = 0; s < NS; ++s) lmc_fmac_bcast<j>(a[s][j], dk[c], a[s][c]);
          }
        });
      };
      double piv_n = 1.0, rl_n = 1.0, l1 = 0.0, hn = 0.0, yn = 0.0, tn = 0.0;
      lm_static_for<NST>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if constexpr (c + 1 < NC) {
          if constexpr (k == 0) {
            l1 = lmc_bcast<c + 1>(dk[c]);  // L[16K + c + 1][16K + c]
          } else if constexpr (k == 1) {
            dk[c + 1] = __builtin_fma(-dk[c], l1, dk[c + 1]);
#pragma unroll
            for (int s = 0; s < NS; ++s) a[s][c + 1] = __builtin_fma(-a[s][c], l1, a[s][c + 1]);
          } else if constexpr (k == 2) {
            piv_n = lmc_bcast<c + 1>(dk[c + 1]);  // the next pivot: lane c + 1's diagonal, now final
          } else if constexpr (k == 3) {
            yn = __builtin_amdgcn_rsq(piv_n);
            hn = -0.5 * piv_n;
          } else if constexpr (k == 4) {
            tn = hn * yn;
          } else if constexpr (k == 5) {
            tn = __builtin_fma(tn, yn, 1.5);
          } else {
            rl_n = yn * tn;
          }
        }
        updates(std::integral_constant<int, k * NU / NST>{}, std::integral_constant<int, (k + 1) * NU / NST>{});
        __builtin_amdgcn_sched_barrier(0);
      });
      piv = piv_n;
      rl = rl_n;
    });
    rdg[16 * K + li] = myrl;  // (every DPP row the same value; entries >= P unused)
    if constexpr (K == TG::NK - 1) LMC_STAMP(7);
    // write L back: the rows below the diagonal tile first (same basic block
    // as their updates), then the diagonal tile
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int row = arow[s];
      double* tr = T + TG::tidx(row >> 4, K) * 256 + (row & 15) * 16;
      const int sw = ((row & 15) >> 1) << 1;
#pragma unroll
      for (int c = 0; c < 16; c += 2) {
        double2 v;
        v.x = a[s][c];
        v.y = a[s][c + 1];
        *reinterpret_cast<double2*>(tr + (c ^ sw)) = v;
      }
    }
    {
      // the diagonal tile, its upper triangle as zeros (every DPP row stores
      // the same values to the same places: no branch)
      double* tr = T + TG::tidx(K, K) * 256 + li * 16;
      const int sw = (li >> 1) << 1;
#pragma unroll
      for (int c = 0; c < 16; c += 2) {
        double2 v;
        v.x = c > li ? 0.0 : dk[c];
        v.y = c + 1 > li ? 0.0 : dk[c + 1];
        *reinterpret_cast<double2*>(tr + (c ^ sw)) = v;
      }
    }
    lmc_signal(&fac[K]);
    if constexpr (K < 2) LMC_STAMP(2 * K + 1);
    else if constexpr (K == TG::NK - 1) LMC_STAMP(5);
  });
  if (!ok && lane == 0) *s_fail = 1;
}
#undef LMC_STAMP

// Backward solve L^T d = y (y = row P of L) by the panel wave, blocks of 16
// columns from the last: z = y_K - sum_{i >= 16(K+1)} L[i][K-block] d_i (lane
// = (column, row residue mod 4), reduced by shuffles), then the 16 x 16
// triangular block by a readlane chain.  d -> dv[0, P).
template <int P>
RPH_INLINE void lmc_backward(const double* T, const double* rdg, double* dv, const double* X, const unsigned* xdone,
                             int* s_fail) {
#pragma clang fp contract(off)
  using TG = TileGrid<P>;
  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
  // static blocks (last first): every load of a block is issued before its sums
  lm_static_for<TG::NK>([&](auto kc) {
    constexpr int K = TG::NK - 1 - decltype(kc)::value;
    constexpr int NC = P - 16 * K < 16 ? P - 16 * K : 16;
    constexpr int I0 = 16 * (K + 1);
    constexpr int NI = P > I0 ? (P - I0 + 3) / 4 : 0;  // rows i = I0 + q + 4 t of this lane
    const int col = 16 * K + c;
    double z0 = 0.0, z1 = 0.0;  // two chains: half the fma latency
#pragma unroll
    for (int t = 0; t < NI; ++t) {
      const int i = I0 + q + 4 * t;
      if (i < P) {
        const double l = T[TG::tidx(i >> 4, K) * 256 + tg_off(i & 15, c)];
        if (t & 1) z1 = __builtin_fma(l, dv[i], z1);
        else z0 = __builtin_fma(l, dv[i], z0);
      }
    }
    double z = z0 + z1;
    z += __shfl_xor(z, 16, 64);
    z += __shfl_xor(z, 32, 64);
    const double y = col < P ? T[TG::tidx(P >> 4, K) * 256 + tg_off(P & 15, c)] : 0.0;
    z = y - z;
    double dk = 0.0;
    if constexpr (K < TG::NX) {
      // an inverted block (owners): d = X^T z, X = L_KK^-1 - independent
      // broadcasts instead of a dependent 16-step chain
      if constexpr (K == TG::NX - 1)
        if (!lmc_wait(xdone, 3u)) *s_fail = 2;
      // (z is the same in every DPP row: z_i = row_newbcast:i, no SGPR round trip)
      const double* xk = X + K * 256 + c;
      double a0 = 0.0, a1 = 0.0;
      lm_static_for<16>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const double zi = lmc_bcast<i>(z);
        if (i & 1) a1 = __builtin_fma(xk[i * 16], zi, a1);
        else a0 = __builtin_fma(xk[i * 16], zi, a0);
      });
      dk = a0 + a1;
    } else {
      // column c of the diagonal tile: L[16K + j][16K + c], j = 0..15
      double lc[16];
      const double* td = T + TG::tidx(K, K) * 256;
#pragma unroll
      for (int j = 0; j < 16; ++j) lc[j] = td[tg_off(j, c)];
      const double rd = col < P ? rdg[col] : 0.0;
      lm_static_for<NC>([&](auto jc) {
        constexpr int j = NC - 1 - decltype(jc)::value;
        const double dj = lmc_bcast<j>(z * rd);  // d[16K + j] (final in lane j of every DPP row)
        if (c == j) dk = dj;
        z = __builtin_fma(-lc[j], dj, z);  // lanes c < j
      });
    }
    if (q == 0 && col < P) dv[col] = dk;
    lmc_wave_sync();
  });
}

}  // namespace rph
