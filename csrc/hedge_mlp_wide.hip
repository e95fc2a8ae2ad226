// rphedge — fused training step for 32-unit hedge MLPs on the matrix cores
// (K9-wide, gfx950).
//
// Same contract as k_hedge_train_step (hedge_mlp.hip): one launch = one Keras
// optimizer step (forward + loss + backward + gradient reduction + Adam +
// EarlyStopping bookkeeping in the last-arriving workgroup), reference
// semantics Replicating_Portfolio.py:149-221.  With 32 hidden units the
// 32x32 middle layer is GEMM-shaped — three products per minibatch tile:
//
//   Z2ᵀ  = W2ᵀ · A1ᵀ     forward           (32 units x 32 paths, K = 32 units)
//   dA1ᵀ = W2  · dZ2ᵀ    backward          (32 units x 32 paths, K = 32 units)
//   dW2  = A1ᵀ · dZ2     weight gradient   (32 x 32, K = 32 paths per tile)
//
// all on v_mfma_f32_32x32x16_bf16 (2 MFMAs each, fp32 accumulate) or, with
// d.mfma_fp32, on v_mfma_f32_32x32x2_f32 (exact fp32, 16 MFMAs each).
//
// Layout (one wave = one 32-path tile at a time; lane l: path r = l&31 of the
// tile, lane half h = l>>5):
//   * every activation lives in the 32x32 MFMA accumulator layout: lane (r,h)
//     register q holds unit  unit_of(q,h) = (q&3) + 8(q>>2) + 4h  of path r.
//     Layer 1 (K = nin) is computed by VALU directly in that layout, so the
//     forward and backward layer-2 products take their B operand straight
//     from registers (bf16 k-order = the permuted unit order; the W2 operand
//     fragments are built once per launch in the matching order) — no LDS;
//   * dW2 sums over PATHS (the lane index), so a1 and dz2 go through a per-wave
//     LDS transpose image ([unit][path], 80-byte rows) read back as ds_read_b128
//     MFMA fragments, accumulating in 16 registers across all tiles;
//   * the small gradients (W1, b1, b2, W3, b3) and the loss statistics are
//     accumulated per lane in registers and reduced once per launch with a
//     32-lane reduce-scatter (the two lane halves hold different units);
//   * the per-workgroup packet [P grads | 4 stats | pad] (R = multiple of 256
//     floats) goes through the same ticketed hand-off as the narrow kernel
//     (float-atomic replicas or deterministic slab), optional fused xGMI
//     all-reduce, and Adam applied in place by the last arriver.
#include "hedge_core.h"
#include "hedge_fit.h"
#include "hedge_lag.h"

namespace rph {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int WH = 32;         // hidden width handled by this kernel
constexpr int IMG_PITCH = 40;  // bf16 per row of the transpose images (80 B rows)
constexpr int IMG_PITCH32 = 33;

// unit held in accumulator register q by lane half h (32x32 C/D layout)
RPH_INLINE constexpr int unit_of(int q, int h) { return (q & 3) + 8 * (q >> 2) + 4 * h; }

template <bool F32>
struct WFrag;
template <>
struct WFrag<false> { bf16x8 f[2]; };
template <>
struct WFrag<true> { float f[16]; };

// A-operand fragments of a 32x32 layer product whose k index runs over units
// in accumulator order.  TR=false: element(row r, unit u) = W2[u][r] (W2ᵀ);
// TR=true: W2[r][u].
template <bool F32, bool TR>
RPH_INLINE void load_wfrag(WFrag<F32>& w, const float* __restrict__ W2, int r, int h) {
  if constexpr (F32) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int u = unit_of(q, h);
      w.f[q] = TR ? W2[r * WH + u] : W2[u * WH + r];
    }
  } else {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int u = unit_of(8 * s + j, h);
        w.f[s][j] = (__bf16)(TR ? W2[r * WH + u] : W2[u * WH + r]);
      }
  }
}

// Y[row][path] = Σ_u A[row][u] X[u][path] with X in accumulator layout
// (x[q] = X[unit_of(q,h)][r]); the result is again in accumulator layout.
template <bool F32>
RPH_INLINE f32x16 layer_mfma(const WFrag<F32>& w, const float (&x)[16]) {
  f32x16 acc = {};
  if constexpr (F32) {
#pragma unroll
    for (int q = 0; q < 16; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w.f[q], x[q], acc, 0, 0, 0);
  } else {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 b;
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = (__bf16)x[8 * s + j];
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w.f[s], b, acc, 0, 0, 0);
    }
  }
  return acc;
}

// dW2 += A1ᵀ · dZ2 over the 32 paths of the tile (transpose through LDS).
template <bool F32>
RPH_INLINE void outer_mfma(void* img, const float (&a1)[16], const float (&dz2)[16], int r, int h, f32x16& acc) {
  if constexpr (F32) {
    float* IA = (float*)img;
    float* IB = IA + WH * IMG_PITCH32;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      IA[unit_of(q, h) * IMG_PITCH32 + r] = a1[q];
      IB[unit_of(q, h) * IMG_PITCH32 + r] = dz2[q];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int s = 0; s < 16; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(IA[r * IMG_PITCH32 + 2 * s + h], IB[r * IMG_PITCH32 + 2 * s + h],
                                                 acc, 0, 0, 0);
  } else {
    __bf16* IA = (__bf16*)img;
    __bf16* IB = IA + WH * IMG_PITCH;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      IA[unit_of(q, h) * IMG_PITCH + r] = (__bf16)a1[q];
      IB[unit_of(q, h) * IMG_PITCH + r] = (__bf16)dz2[q];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 a = *(const bf16x8*)(IA + r * IMG_PITCH + 16 * s + 8 * h);
      const bf16x8 b = *(const bf16x8*)(IB + r * IMG_PITCH + 16 * s + 8 * h);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    }
  }
  // the next tile rewrites the images: its writes must follow these reads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- bf16 path: one conversion per activation, shared by the layer MFMA and
// the dW2 transpose image.  Registers 8s..8s+7 of an accumulator-layout tile
// are packed pairwise (v_cvt_pk_bf16_f32) into fragment s = the B operand of
// a product over the unit index (k order = accumulator order).
RPH_INLINE void pack_bf16(const float (&x)[16], bf16x8 (&b)[2]) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) b[s][j] = (__bf16)x[8 * s + j];
}

RPH_INLINE f32x16 layer_mfma_bf16(const WFrag<false>& w, const bf16x8 (&b)[2]) {
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w.f[0], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w.f[1], b[1], acc, 0, 0, 0);
  return acc;
}

// dW2 += A1ᵀ·dZ2 over the 32 paths of the tile, bf16.  Each lane stores its
// packed registers 4g..4g+3 (units 8g+4h..+3 of path r, 8 bytes) into a
// [path][unit] image (TR_PITCH-byte rows, padded against write conflicts) and
// the MFMA operands (unit r, 8 consecutive paths) come back with the gfx950
// transposing read ds_read_b64_tr_b16 (cdna_hip_programming.md T10): lane 4q+p
// of each 16-lane group addresses image row r0+q, units c0+4p..+3, and lane i
// of the group receives unit c0+i of rows r0..r0+3.  EXEC is all ones here
// (the tile loop is wave-uniform), as the transposing read requires.
constexpr int TR_PITCH = 72;  // bytes per image row (32 bf16 + 8 B pad)
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

RPH_INLINE void outer_mfma_tr(unsigned char* img, const bf16x8 (&a1b)[2], const bf16x8 (&dzb)[2], int r, int h,
                              int lane, f32x16& acc) {
  unsigned char* IA = img;
  unsigned char* IB = img + 32 * TR_PITCH;
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const int off = r * TR_PITCH + (8 * g4 + 4 * h) * 2;
    const bf16x8& sa = a1b[g4 >> 1];
    const bf16x8& sb = dzb[g4 >> 1];
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const bf16x4 va = {sa[4 * (g4 & 1) + 0], sa[4 * (g4 & 1) + 1], sa[4 * (g4 & 1) + 2], sa[4 * (g4 & 1) + 3]};
    const bf16x4 vb = {sb[4 * (g4 & 1) + 0], sb[4 * (g4 & 1) + 1], sb[4 * (g4 & 1) + 2], sb[4 * (g4 & 1) + 3]};
    *(bf16x4*)(IA + off) = va;
    *(bf16x4*)(IB + off) = vb;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int grp = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int c0 = 16 * (grp & 1), hh = grp >> 1;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int off = (16 * s + 8 * hh + q) * TR_PITCH + (c0 + 4 * p) * 2;
    const s16x4 ra0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(IA + off));
    const s16x4 ra1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(IA + off + 4 * TR_PITCH));
    const s16x4 rb0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(IB + off));
    const s16x4 rb1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(IB + off + 4 * TR_PITCH));
    // whole-vector bit casts (element-wise bit_cast<__bf16> inserts were
    // miscompiled into splats of element 0 in the narrow body's twin)
    const bf16x8 fa = __builtin_bit_cast(bf16x8, __builtin_shufflevector(ra0, ra1, 0, 1, 2, 3, 4, 5, 6, 7));
    const bf16x8 fb = __builtin_bit_cast(bf16x8, __builtin_shufflevector(rb0, rb1, 0, 1, 2, 3, 4, 5, 6, 7));
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc, 0, 0, 0);
  }
  // the next tile rewrites the images: its writes must follow these reads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// o[k] = part[k](lane half 0) + part[k](lane half 1), in every lane, for k < NO.
// Pairs (2m, 2m+1): one v_permlane32_swap leaves the sum of output 2m in the
// low half and of 2m+1 in the high half, a second swap of that sum with itself
// hands each half the other's; an odd last output takes one self-swap.
template <int NO>
RPH_INLINE void half_sum_outputs(const float (&part)[NO], float (&o)[NO]) {
#pragma unroll
  for (int m = 0; m + 1 < NO; m += 2) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(part[m]), __float_as_uint(part[m + 1]), false,
                                                    false);
    const float sm = __uint_as_float(r[0]) + __uint_as_float(r[1]);  // lo: o[m], hi: o[m+1]
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(sm), __float_as_uint(sm), false, false);
    o[m] = __uint_as_float(b[0]);
    o[m + 1] = __uint_as_float(b[1]);
  }
  if constexpr (NO & 1) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(part[NO - 1]), __float_as_uint(part[NO - 1]),
                                                    false, false);
    o[NO - 1] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
}

// Per-lane register vector of the small gradients (units of this lane half)
template <int NIN, int NO>
struct SmallGrad {
  static constexpr int DW1 = 0;
  static constexpr int DB1 = DW1 + 16 * NIN;
  static constexpr int DB2 = DB1 + 16;
  static constexpr int DW3 = DB2 + 16;
  static constexpr int DB3 = DW3 + 16 * NO;
  static constexpr int ST = DB3 + NO;
  static constexpr int NV = ST + 4;
  static constexpr int RV = NV <= 64 ? 64 : NV <= 128 ? 128 : 256;
  static_assert(NV <= 256, "small-gradient vector too long");
};

// packet index of small-gradient entry idx held by lane half h (-1: none)
template <int NIN, int NO, int P>
RPH_INLINE int small_param(int idx, int h) {
  using G = SmallGrad<NIN, NO>;
  using S = NetShape<NIN, WH, NO, HEAD_FREE>;  // offsets do not depend on the head
  if (idx < G::DB1) return S::OW1 + (idx / 16) * WH + unit_of(idx % 16, h);
  if (idx < G::DB2) return S::OB1 + unit_of(idx - G::DB1, h);
  if (idx < G::DW3) return S::OB2 + unit_of(idx - G::DB2, h);
  if (idx < G::DB3) {
    const int t = idx - G::DW3;
    return S::OW3 + unit_of(t / NO, h) * NO + (t % NO);
  }
  if (h != 0) return -1;  // path-level entries are accumulated by lane half 0 only
  if (idx < G::ST) return S::OB3 + (idx - G::DB3);
  if (idx < G::NV) return P + (idx - G::ST);
  return -1;
}

// 32-lane reduce-scatter (bits 4..0): lane (r, h) ends with the half-wave sum
// of entries [r*RV/32, (r+1)*RV/32) in v[0 .. RV/32).
template <int RV>
RPH_INLINE void half_reduce_scatter(float* v, int lane) {
  halve_step<RV, 4>(v, lane);
  halve_step<RV / 2, 3>(v, lane);
  halve_step<RV / 4, 2>(v, lane);
  halve_step<RV / 8, 1>(v, lane);
  halve_step<RV / 16, 0>(v, lane);
}

// Per-workgroup gradient packet of one minibatch step on the matrix cores.
// Used by the per-step kernel below and by the persistent per-fit kernel.
template <int NIN, int NO, int HEAD, bool F32>
struct WideBody {
  static constexpr int WAVES_PER_SIMD = 1;
  using S = NetShape<NIN, WH, NO, HEAD>;
  using G = SmallGrad<NIN, NO>;
  static constexpr int P = S::P;
  static constexpr int R = S::R;  // packet width, multiple of 256
  static constexpr int NR = R / 256;
  static constexpr int NREP = WIDE_NREP;  // lagged schedule: float-atomic replicas
  static constexpr bool ACC_PLAIN = false;  // lagged prologue: agent-scope accumulator loads (faster here)
  static constexpr int NHOLD = S::NHOLD;
  static constexpr int RV = G::RV;
  static constexpr int IMG_BYTES = F32 ? 2 * WH * IMG_PITCH32 * 4 : 2 * WH * TR_PITCH;
  static constexpr int SCRATCH_FLOATS = ((4 * IMG_BYTES > 4 * R * 4) ? 4 * IMG_BYTES : 4 * R * 4) / 4 + 8;
  static_assert(R % 256 == 0, "wide packet must be a multiple of 256");
  struct Frags {
    WFrag<F32> w2t, w2;
  };
  struct Pre {  // this lane's path of the first tile, loaded ahead by the caller
    float x[NIN], pr[NHOLD], y;
    bool valid;
  };

  // W2src: the 32x32 W2 block (global memory or LDS)
  RPH_INLINE static void make_frags(const float* __restrict__ W2src, Frags& f) {
    const int lane = threadIdx.x & 63;
    load_wfrag<F32, false>(f.w2t, W2src, lane & 31, lane >> 5);
    load_wfrag<F32, true>(f.w2, W2src, lane & 31, lane >> 5);
  }

  RPH_INLINE static int first(int wid) { return blockIdx.x * 4 + wid; }  // first tile of this wave

  RPH_INLINE static void load(const TrainDesc& d, int step, const Perm& perm, int T, int lane, Pre& p) {
    const long long jl = (long long)T * 32 + (lane & 31);
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

  // wl: weights in LDS; scratch: SCRATCH_FLOATS of LDS; pre: first tile (loaded).
  // Returns in val[k] the workgroup sum of packet entry tid + 256 k.
  RPH_INLINE static void partial(const TrainDesc& d, int step, const Perm& perm, const float* __restrict__ wl_in,
                                 const Frags& fr, float* scratch, Pre& pre, float (&val)[NR]) {
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int nwaves = gridDim.x * 4;
    const int ntiles = (d.batch + 31) >> 5;
    void* img = (unsigned char*)scratch + wid * IMG_BYTES;
    float g[RV];
#pragma unroll
    for (int i = 0; i < RV; ++i) g[i] = 0.f;
    f32x16 gw2 = {};
    const float alpha = d.alpha;
    const float hv0 = (h == 0) ? 1.f : 0.f;

    for (int T = first(wid); T < ntiles; T += nwaves) {
      float x[NIN], pr[NHOLD];
#pragma unroll
      for (int f = 0; f < NIN; ++f) x[f] = (pre.x[f] - d.fmu[f]) * d.fisd[f];
#pragma unroll
      for (int k = 0; k < NHOLD; ++k) pr[k] = pre.pr[k];
      const float y = pre.y;
      const bool valid = pre.valid;
      if (T + nwaves < ntiles) load(d, step, perm, T + nwaves, lane, pre);  // software pipelining

      // weights are re-read from LDS every tile through an opaque zero offset:
      // hoisted, the ~100 per-lane layer-1/2/3 weights overflowed into AGPRs and
      // came back with v_accvgpr_read every tile
      const float* __restrict__ wl = wl_in;
      {
        uint32_t zo = 0;
        asm volatile("" : "+v"(zo));
        wl = (const float*)__builtin_assume_aligned(wl_in + (zo & ~3u), 16);
      }
      // ---- forward --------------------------------------------------------
      // (z1, z2 are not kept: for 0 <= alpha <= 1, lrelu'(z) = [a > 0 ? 1 : alpha]
      // with a = lrelu(z), so the activations alone carry the backward mask)
      float a1[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int u = unit_of(q, h);
        float acc = wl[S::OB1 + u];
#pragma unroll
        for (int f = 0; f < NIN; ++f) acc = fmaf(x[f], wl[S::OW1 + f * WH + u], acc);
        a1[q] = lrelu(acc, alpha);
      }
      bf16x8 a1b[2];
      f32x16 z2acc;
      if constexpr (F32) {
        z2acc = layer_mfma<F32>(fr.w2t, a1);
      } else {
        pack_bf16(a1, a1b);
        z2acc = layer_mfma_bf16(fr.w2t, a1b);
      }
      float a2[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) a2[q] = lrelu(z2acc[q] + wl[S::OB2 + unit_of(q, h)], alpha);
      float o[NO];
      {
        float part[NO];  // this lane half's 16 units
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          float acc = 0.f;
#pragma unroll
          for (int q = 0; q < 16; ++q) acc = fmaf(a2[q], wl[S::OW3 + unit_of(q, h) * NO + k], acc);
          part[k] = acc;
        }
        // full sums over the two lane halves with v_permlane32_swap (VALU, on
        // the forward->loss->backward critical path) instead of ds_bpermute
        half_sum_outputs<NO>(part, o);
#pragma unroll
        for (int k = 0; k < NO; ++k) o[k] += wl[S::OB3 + k];
      }
      float hold[NHOLD];
      if (HEAD == HEAD_COMPLEMENT) {
        hold[0] = o[0];
        hold[1] = 1.f - o[0];
      } else {
#pragma unroll
        for (int k = 0; k < NHOLD; ++k) hold[k] = o[k];
      }
      float V = 0.f;
#pragma unroll
      for (int k = 0; k < NHOLD; ++k) V = fmaf(hold[k], pr[k], V);
      float l, dV;
      path_loss(d.loss, d.quantile, V, y, l, dV);
      dV = valid ? dV * d.inv_batch : 0.f;
      const float hv = valid ? hv0 : 0.f;  // path-level statistics: lane half 0 only
      const float ae = fabsf(V - y);
      g[G::ST + 0] = fmaf(hv, l, g[G::ST + 0]);
      g[G::ST + 1] = fmaf(hv, ae, g[G::ST + 1]);
      g[G::ST + 2] = fmaf(hv, ae * __frcp_rn(fmaxf(fabsf(y), 1e-7f)), g[G::ST + 2]);
      g[G::ST + 3] += hv;

      // ---- backward -------------------------------------------------------
      float dout[NO];
      if (HEAD == HEAD_COMPLEMENT) {
        dout[0] = dV * (pr[0] - pr[1]);
      } else {
#pragma unroll
        for (int k = 0; k < NO; ++k) dout[k] = dV * pr[k];
      }
#pragma unroll
      for (int k = 0; k < NO; ++k) g[G::DB3 + k] = fmaf(hv0, dout[k], g[G::DB3 + k]);
      float dz2[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int u = unit_of(q, h);
        float da = 0.f;
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          g[G::DW3 + q * NO + k] = fmaf(a2[q], dout[k], g[G::DW3 + q * NO + k]);
          da = fmaf(wl[S::OW3 + u * NO + k], dout[k], da);
        }
        dz2[q] = a2[q] > 0.f ? da : alpha * da;
        g[G::DB2 + q] += dz2[q];
      }
      bf16x8 dzb[2];
      f32x16 da1;
      if constexpr (F32) {
        da1 = layer_mfma<F32>(fr.w2, dz2);
      } else {
        pack_bf16(dz2, dzb);
        da1 = layer_mfma_bf16(fr.w2, dzb);
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float dz1 = a1[q] > 0.f ? da1[q] : alpha * da1[q];
        g[G::DB1 + q] += dz1;
#pragma unroll
        for (int f = 0; f < NIN; ++f) g[G::DW1 + f * 16 + q] = fmaf(x[f], dz1, g[G::DW1 + f * 16 + q]);
      }
      if constexpr (F32) {
        outer_mfma<F32>(img, a1, dz2, r, h, gw2);
      } else {
        outer_mfma_tr((unsigned char*)img, a1b, dzb, r, h, lane, gw2);
      }
    }
    RPH_STAMP(5);  // path loop done (Adam fits: every workgroup's own row)

    // ---- per-wave packet -> LDS, cross-wave sum -----------------------------
    half_reduce_scatter<RV>(g, lane);
    __syncthreads();  // every wave is done with its transpose image (aliases the packet)
    float* pk = scratch;
    float* pkw = pk + wid * R;
    for (int i = P + 4 + lane; i < R; i += 64) pkw[i] = 0.f;
    constexpr int PER = RV / 32;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int prm = small_param<NIN, NO, P>(r * PER + i, h);
      if (prm >= 0) pkw[prm] = g[i];
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) pkw[S::OW2 + unit_of(q, h) * WH + r] = gw2[q];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int i = tid + 256 * k;
      val[k] = (pk[i] + pk[R + i]) + (pk[2 * R + i] + pk[3 * R + i]);
    }
    __syncthreads();
  }
};

template <int NIN, int NO, int HEAD, bool F32>
__global__ __launch_bounds__(256) void k_hedge_train_step_wide(const TrainDesc d, const int step, const int epoch,
                                                               const Perm perm) {
  using B = WideBody<NIN, NO, HEAD, F32>;
  constexpr int P = B::P;
  constexpr int R = B::R;
  constexpr int NR = B::NR;
  prefetch_kernarg<sizeof(TrainDesc) + 2 * sizeof(int) + sizeof(Perm)>();
  __shared__ __attribute__((aligned(16))) float scratch[B::SCRATCH_FLOATS];
  __shared__ __attribute__((aligned(16))) float wl[P + 4];
  __shared__ int s_last;

  RPH_STAMP(0);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const float stopped = d.fit->stopped;
  const float* __restrict__ Wg = d.wts->w[0];
  UpdPre<P> up;
  if (d.fused_update) prefetch_update<P>(up, d.wts, d.opt, d.fit, d.lr_sched, epoch, step);
  typename B::Frags fr;
  B::make_frags(Wg + B::S::OW2, fr);
  for (int i = tid; i < P; i += 256) wl[i] = Wg[i];
  typename B::Pre pre;
  pre.valid = false;
  if (B::first(wid) < ((d.batch + 31) >> 5)) B::load(d, step, perm, B::first(wid), lane, pre);

  if (stopped != 0.f) return;  // early-stopped fit: remaining steps are no-ops
  if (d.fused_update) {
    asm volatile("" ::"v"(up.m[0]), "v"(up.v[0]), "v"(up.w[0]), "v"(up.wbest[0]), "s"(up.t), "s"(up.lr),
                 "s"(up.loss_sum), "s"(up.wait), "s"(up.best_loss), "s"(up.lr_sched_e));
  }
  __syncthreads();
  RPH_STAMP(1);
  float val[NR];
  B::partial(d, step, perm, wl, fr, scratch, pre, val);
  float* pk = scratch;
  RPH_STAMP(3);

  if (gridDim.x > 1) {
    const int Gn = gridDim.x;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int i = tid + 256 * k;
      if (d.deterministic) st_agent(d.slab + (size_t)blockIdx.x * R + i, val[k]);
      else __hip_atomic_fetch_add(d.acc + (blockIdx.x % ACC_REPLICAS) * R + i, val[k], __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains
    __syncthreads();
    RPH_STAMP(4);
    if (tid == 0) {
      const uint32_t ticket = __hip_atomic_fetch_add(d.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = (ticket == (uint32_t)Gn - 1u) ? 1 : 0;
    }
    __syncthreads();
    RPH_STAMP(5);
    if (!s_last) return;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int i = tid + 256 * k;
      float a = 0.f;
      if (d.deterministic) {
        // fixed combine order => bitwise reproducible
        for (int row = 0; row < Gn; ++row) a += ld_agent(d.slab + (size_t)row * R + i);
      } else {
        float rr[ACC_REPLICAS];
#pragma unroll
        for (int rp = 0; rp < ACC_REPLICAS; ++rp) rr[rp] = ld_agent(d.acc + rp * R + i);
        a = ((rr[0] + rr[1]) + (rr[2] + rr[3])) + ((rr[4] + rr[5]) + (rr[6] + rr[7]));
#pragma unroll
        for (int rp = 0; rp < ACC_REPLICAS; ++rp) st_agent(d.acc + rp * R + i, 0.f);  // re-arm
      }
      val[k] = a;
    }
    if (tid == 0) __hip_atomic_store(d.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  float* red = pk;
#pragma unroll
  for (int k = 0; k < NR; ++k) red[tid + 256 * k] = val[k];
  __syncthreads();
  RPH_STAMP(6);
  if (d.dp_world > 1) dp_allreduce<R>(d, red);
  if (d.fused_update) {
    apply_update<P>(red, up, d.wts, d.opt, d.fit, epoch, step, d.steps_per_epoch);
  } else {
#pragma unroll
    for (int k = 0; k < NR; ++k) d.grad_out[tid + 256 * k] = red[tid + 256 * k];
  }
  RPH_STAMP(7);
}

int launch_wide_step(const TrainDesc* d, int step, int epoch, const Perm& perm, hipStream_t s) {
#define X(A, B, C, E)                                                                                   \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E)) {                                          \
    if (d->mfma_fp32)                                                                                   \
      hipLaunchKernelGGL((k_hedge_train_step_wide<A, C, E, true>), dim3(d->num_wgs), dim3(256), 0, s, *d, \
                         step, epoch, perm);                                                            \
    else                                                                                                \
      hipLaunchKernelGGL((k_hedge_train_step_wide<A, C, E, false>), dim3(d->num_wgs), dim3(256), 0, s, *d, \
                         step, epoch, perm);                                                            \
    return (int)hipGetLastError();                                                                      \
  }
  RPH_WIDE_SHAPES(X)
#undef X
  return -1;
}

// Persistent per-fit kernel for the wide nets.  The 5-32-6 basket net is not
// offered: its optimizer state (6 parameters per thread x w/m/v/best) on top of
// the MFMA tile state spills ~1.4 KB/lane and the spilled variant gave wrong
// results on gfx950 — that shape runs the lagged/ticketed step kernels.
#define RPH_WIDE_FIT_SHAPES(X)   \
  X(1, 32, 1, HEAD_COMPLEMENT)   \
  X(1, 32, 2, HEAD_FREE)         \
  X(2, 32, 2, HEAD_FREE)         \
  X(3, 32, 2, HEAD_FREE)

int launch_wide_fit(const TrainDesc* d, int epochs, hipStream_t s) {
#define X(A, B, C, E)                                                          \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E)) {                 \
    if (d->mfma_fp32) return launch_fit<WideBody<A, C, E, true>>(d, epochs, s); \
    return launch_fit<WideBody<A, C, E, false>>(d, epochs, s);                 \
  }
  RPH_WIDE_FIT_SHAPES(X)
#undef X
  return rph_report("rph_train_fit", "no persistent fit kernel for this network shape (use lag/ticket)");
}

int launch_wide_lag_step(const TrainDesc* d, int k, int epoch, const Perm& perm, hipStream_t s) {
#define X(A, B, C, E)                                                                                         \
  if (shape_is(d->nin, d->h, d->nout, d->head, A, B, C, E)) {                                                \
    if (d->mfma_fp32)                                                                                         \
      hipLaunchKernelGGL((k_hedge_step_lag<WideBody<A, C, E, true>>), dim3(d->num_wgs), dim3(256), 0, s, *d, k, \
                         epoch, perm);                                                                        \
    else                                                                                                      \
      hipLaunchKernelGGL((k_hedge_step_lag<WideBody<A, C, E, false>>), dim3(d->num_wgs), dim3(256), 0, s, *d,  \
                         k, epoch, perm);                                                                     \
    return (int)hipGetLastError();                                                                            \
  }
  RPH_WIDE_SHAPES(X)
#undef X
  return -1;
}

}  // namespace rph
