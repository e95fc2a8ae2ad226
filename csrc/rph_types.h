// rphedge — host/device shared plain-old-data structures.
//
// Every device-resident state block is a flat float32 array so the Python side
// (rphedge/ops/native.py) can allocate it as a torch tensor and read fields by
// index.  The field indices below are mirrored in rphedge/ops/layout.py and
// checked by rph_layout_check() at import time.
#pragma once
#include <stdint.h>

namespace rph {

constexpr int PMAX = 2048;     // max flat parameters per hedge network
constexpr int MAXIN = 8;       // max input features
constexpr int MAXHOLD = 8;     // max hedging instruments (assets + bond)
constexpr int MAXHIST = 1024;  // per-fit epoch-loss history
constexpr int EVAL_NSTAT = 32; // doubles per workgroup in the eval stats slab
constexpr int LAG_SLOTS = 16;  // lagged schedule: replica rows per rotating accumulator buffer

enum Head : int { HEAD_FREE = 0, HEAD_COMPLEMENT = 1 };
enum Loss : int { LOSS_MSE = 0, LOSS_PINBALL = 1 };

// Network weights.  Updated in place by the last-arriving workgroup of a step
// (all readers of the launch have finished by then); w[1]/cur are reserved.
struct NetWeights {
  float w[2][PMAX];
  float cur;
  float pad[3];
};

// Keras-semantics Adam state (one per compiled optimizer; Q1 parity shares one
// NetWeights between two OptStates — Replicating_Portfolio.py:172, :175-180).
struct OptState {
  float m[PMAX];
  float v[PMAX];
  float t;          // iteration counter (persists across fits like a Keras optimizer)
  float lr;         // current learning rate (LearningRateScheduler writes it)
  float beta1, beta2, eps;
  float nan_steps;  // NaN/Inf guard: number of skipped updates
  float pad0, pad1;
};

// EarlyStopping(monitor='loss') + epoch bookkeeping; reset by the host per fit
// (Replicating_Portfolio.py:174, :203-209).
struct FitState {
  float w_best[PMAX];
  float best_loss;     // +inf at fit start
  float wait;
  float stopped;       // 1 => remaining launched steps are no-ops
  float epoch;         // epochs completed in this fit
  float patience;
  float max_epochs;
  float restore_best;  // Keras restore_best_weights
  float has_best;
  float loss_sum, loss_cnt, abs_sum, ape_sum;  // running sums over the epoch
  float last_loss, last_mae, last_mape;
  float restore_at_end;  // Keras-3 semantics: also restore when max_epochs reached
  float hist[MAXHIST];   // epoch loss history
};

constexpr int NETW_FLOATS = (int)(sizeof(NetWeights) / 4);
constexpr int OPT_FLOATS = (int)(sizeof(OptState) / 4);
constexpr int FIT_FLOATS = (int)(sizeof(FitState) / 4);

// ---------------------------------------------------------------------------
// Launch descriptors (passed by pointer from ctypes, by value to kernels).
// ---------------------------------------------------------------------------
struct TrainDesc {
  const float* feat[MAXIN];      // features at t, [n_local] each
  const float* price[MAXHOLD];   // traded-asset prices at t+1 (bond excluded)
  const float* target;           // V_{t+1}, [n_local]
  NetWeights* wts;
  OptState* opt;
  FitState* fit;
  const float* lr_sched;         // [max_epochs] or null; NaN entry => keep lr
  float* slab;                   // [max_wgs][R] partials
  uint32_t* counter;             // arrival ticket (zeroed at alloc, reset by last arriver)
  float* grad_out;               // [R] summed gradient (multi-rank path), may be null
  float bond;                    // B_{t+1} (normalised), same for all paths
  float alpha;                   // LeakyReLU slope
  float quantile;                // pinball q
  float inv_batch;               // 1 / global batch size
  int loss;                      // Loss
  int n_local;                   // local paths
  int batch;                     // local batch per step
  int steps_per_epoch;
  int chunk_log2;                // shuffle granularity (0 = per path, 6 = 64-path chunks)
  int shuffle;                   // Keras fit(shuffle=True)
  uint32_t seed;
  int fused_update;              // 1: last arriver applies Adam (world_size==1)
  int num_wgs;
  int nin, h, nout, head;        // network shape (dispatch)
  float* acc;                    // [8][R] float-atomic accumulator (zeroed; re-armed by last arriver)
  int deterministic;             // 1: fixed-order slab reduction (bitwise reproducible)
  unsigned long long* stamps;    // diagnostic phase stamps [num_wgs][8] (null in production)
  // Fused data-parallel all-reduce over xGMI peer memory (dp_world > 1):
  // mailbox of rank p = dp_mbox[p]: [DP_SLOTS][dp_world][R] floats, flags
  // dp_flags[p]: [DP_SLOTS][dp_world] u32 (IPC-mapped, system-scope accesses).
  int dp_world;
  int dp_rank;
  float* dp_mbox[8];
  uint32_t* dp_flags[8];
  uint32_t* dp_counter;          // this rank's step sequence counter (device)
  uint32_t* dp_error;            // set on a peer timeout (host checks after the run)
  int mfma_fp32;                 // 32-unit nets: exact fp32 MFMA (32x32x2) instead of bf16 (32x32x16)
  float* lag;                    // lagged-update state slots [2][LAG_FLOATS] (hedge_lag.h)
  int variant;                   // kernel variant (narrow: 1 = 2 waves/SIMD, weights re-read from LDS)
  const FitState* fit_init;      // lagged schedule: fit-state template read by kernel 0, which also
                                 // writes it to `fit` (no separate template copy per fit); may be null
  float fmu[MAXIN];              // input standardisation x' = (x - fmu) * fisd, fused into the feature
  float fisd[MAXIN];             // loads (identity: 0 / 1; the host folds it into layer 1 on export)
};

constexpr int DP_SLOTS = 4;

struct EvalDesc {
  const float* feat[MAXIN];      // features at t
  const float* price_t[MAXHOLD]; // traded assets at t
  const float* price_t1[MAXHOLD];// traded assets at t+1 (may be null => no residual)
  const float* target;           // V_{t+1} (may be null)
  const NetWeights* wa;
  const NetWeights* wb;          // optional second network (holdings blend)
  const float* g_base;           // optional: V_t = g + blend_c * (h - g)
  float* v_out;                  // V_t (may be null)
  float* hold_out[MAXHOLD];      // holdings (may be null)
  float* resid_out;              // V_{t+1} - h . p_{t+1} (may be null)
  float* pred1_out;              // h . p_{t+1} (may be null)
  double* stats;                 // [num_wgs][EVAL_NSTAT]
  float bond_t, bond_t1;
  float alpha;
  float blend_c;
  float hold_c;                  // holdings = hA + hold_c * (hB - hA)
  int n_local;
  int num_wgs;
  int nin, h, nout, head;
  float fmu[MAXIN];              // input standardisation x' = (x - fmu) * fisd (identity: 0 / 1)
  float fisd[MAXIN];
  // per-date weight snapshots for the saved-model format and the P&L scan:
  // workgroup 0 copies the P current weights of wa / wb into w[0] of these
  // NetWeights blocks (may be null) - no separate copy launch per date
  NetWeights* snap_a;
  NetWeights* snap_b;
};

// Self-financing hedge P&L scan (k_hedge_pnl): one forward pass over the
// rebalancing dates with the per-date networks.  Wealth starts at V_0 (the
// fitted date-0 value), holds phi_t (the traded-asset holdings of date t's
// network, blended hA + hold_c (hB - hA) when a second network is given) and
// keeps the rest in the bank account:
//   W_{t+1} = sum_a phi_a,t S_a,t+1 + (W_t - sum_a phi_a,t S_a,t) B_{t+1} / B_t
//   P&L_T   = W_T - V_T(payoff)
// Element (t, p) of feature f lives at feat[f][t * feat_ts[f] + p] (the
// time-major coarse grids), likewise for the traded prices.
struct PnlDesc {
  const float* feat[MAXIN];
  long long feat_ts[MAXIN];
  const float* price[MAXHOLD];   // traded assets (bond excluded)
  long long price_ts[MAXHOLD];
  const NetWeights* snap;        // [n_dates][2] per-date networks (A at [t][0], B at [t][1])
  const float* fmu;              // [n_dates][MAXIN] per-date standardisation
  const float* fisd;
  const double* bond;            // [n_dates + 1] B_t on the coarse grid
  const float* w0;               // initial wealth per path (values[0]); null: wealth0 scalar
  const float* payoff;           // terminal liability per path (values[n_dates])
  float* pnl_out;                // per-path P&L (may be null)
  double* stats;                 // [num_wgs][EVAL_NSTAT]: ES_V = W_T, ES_RES = P&L, ...
  float alpha, hold_c, wealth0;
  int has_b;
  int n_local, n_dates, num_wgs;
  int nin, h, nout, head;
};

// Levenberg-Marquardt fit (hedge_lm.hip): full-batch MSE fits of the 8-unit
// nets by damped Gauss-Newton steps.  One PASS = k_lm_pass (loss + gradient
// over every local path, VALU; Gram matrix J^T J of a path subsample on the
// matrix cores) -> k_lm_reduce (fixed-order sums of the per-workgroup slabs) ->
// [data parallel: all-reduce of the reduced block] -> k_lm_solve (one
// workgroup: accept / reject the trial point, damping, fp64 Cholesky solve of
// (G + lam diag G) d = -g, next trial point).  Deterministic: no float atomics.
constexpr int LM_NPMAX = 192;        // padded parameter count (6 x 32)
constexpr int LM_TILE = 64;          // Gram subsample paths per gram workgroup (one MFMA K tile)
// reduced block (doubles) of one trial point: [G blocks | g | stats]
//   G: NB(NB+1)/2 upper-triangular 32x32 blocks in MFMA register order
//   g: gradient of mean((V - y)^2) [LM_NPMAX]; stats: loss sum, |e| sum, ape sum, count
constexpr int LM_GBLK_MAX = 21 * 1024;
// + the output-layer Gram matrix over EVERY path (the value is linear in the
// output layer's NU <= 64 parameters, so the loss is exactly quadratic in
// them): G_oo = mean_p u_p u_p^T, u = dV/dtheta_o, packed upper triangle
// (i <= j, row-major) at LM_RED_OUTG, accumulated on the matrix cores by the
// last LM_OUTG_TAIL evaluations of an lm_out_fix fit (NarrowPairBody OG)
constexpr int LM_OUTG = 64 * 65 / 2;
constexpr int LM_OUTG_TAIL = 1;  // evaluations of an lm_out_fix fit that carry it: the last one (passes)
constexpr int LM_RED_OUTG = LM_GBLK_MAX + LM_NPMAX + 8;
constexpr int LM_RED = LM_RED_OUTG + LM_OUTG;
constexpr int LM_PASS_WGS_MAX = 512;  // LM pass workgroups (two per CU for the small nets; k_lm_reduce trees)
constexpr int LM_OG_MAX = 64;    // output-layer parameters of the full-batch Gram (two 32-row MFMA blocks)
// k_lm_solve workgroups of a full solve: workgroup m factorises the system at
// the damping that m consecutive rejections would reach, so a rejection's
// solve only publishes a step computed ahead (speculative reject branch)
constexpr int LM_SPEC = 4;
// solver state (doubles)
enum LmState : int {
  LMS_W = 0,                         // [2][LM_NPMAX] weights of the two slots (trial / best)
  LMS_RED = 2 * LM_NPMAX,            // [2][LM_RED] reduced blocks (the best point's at LMS_RED)
  LMS_BEST = LMS_RED + 2 * LM_RED,   // host mirror: index of the best weight slot (last solve)
  LMS_LAM,                           // host mirror: damping after the last solve
  LMS_NACC,                          // accepted steps of the current fit
  LMS_FAIL,                          // Cholesky failures (non-positive pivot)
  LMS_LFIN,                          // the fit's final best loss (written by the last solve)
  LMS_FAILTOT,                       // Cholesky failures of every fit on this state (never reset)
  LMS_SPEC_LAM = LMS_FAIL + 8,       // [LM_SPEC] damping of precomputed reject-branch step m
  LMS_SPEC_PRED = LMS_SPEC_LAM + LM_SPEC,  // [LM_SPEC] its predicted reduction
  LMS_SPEC_OK = LMS_SPEC_PRED + LM_SPEC,   // [LM_SPEC] 1: positive definite (step valid)
  LMS_SPEC_W = LMS_SPEC_OK + LM_SPEC,       // [LM_SPEC][LM_NPMAX] trial weights best + d_m
  // [2][LM_SLOT] solver scalars by pass parity: the pass and solve kernels of
  // pass p read slot p & 1, the solve writes slot (p + 1) & 1 - so no
  // workgroup of a solve ever reads a scalar another one is writing
  LMS_SLOTS = LMS_SPEC_W + LM_SPEC * LM_NPMAX,
  LMS_FLOATS = LMS_SLOTS + 16
};
constexpr int LM_SLOT = 8;
enum LmSlot : int {
  LSS_BEST = 0,    // index of the best weight slot
  LSS_LAM,         // damping
  LSS_NU,          // Nielsen damping: growth factor of the next rejection
  LSS_PRED,        // predicted loss reduction of the pending trial (quadratic model)
  LSS_COPY,        // 1: that solve accepted; the next pass kernel copies the trial's reduced
                   // block into the best block (deferred off the solve's path)
  LSS_SPEC_IDX,    // next precomputed reject-branch step (>= LM_SPEC: none)
  LSS_LBEST,       // the best point's loss
  LSS_STOP,        // > 0: the fit stopped at the solve of this pass (adaptive budget)
};

// Data-parallel exchange of the LM reduced block over IPC-mapped peer
// mailboxes (k_lm_dp_exchange): LM_DP_WGS workgroups, each owning a chunk of
// the block; per (slot, sender) row `pitch` 8-byte entries = LM_RED data +
// LM_DP_WGS per-workgroup flags.
constexpr int LM_DP_WGS = 16;
// fused exchange (LmDesc.dp_fused): k_lm_reduce's gradient-packet and
// output-Gram workgroups push their entries of the gradient region themselves,
// each with its own flag (<= LM_DP_FLAGS of them) after the LM_RED data entries
constexpr int LM_DP_FLAGS = 128;
constexpr int LM_DP_PITCH = LM_RED + LM_DP_FLAGS;  // mailbox row pitch (8-byte entries)
struct LmDpDesc {
  double* mbox[8];               // every rank's mailbox [DP_SLOTS][world][pitch] (own = mbox[rank])
  unsigned* counter;             // [0] exchanges completed by this rank, [1] workgroup arrival ticket
  unsigned* error;               // [0] set on a peer timeout
  int world, rank;
  int pitch;                     // entries per (slot, sender) row (>= LM_DP_PITCH)
  // fault injection (transport-probe tests only; 0 in every run): 1 = the
  // fused exchange in k_lm_reduce drops rank W-1's contribution on EVERY rank
  // - a wrong sum that is still bitwise identical across ranks, so only a
  // comparison with an independent all-reduce can catch it
  int fault;
};

struct LmDesc {
  double* state;                 // [LMS_FLOATS]
  float* slab_b;                 // [num_wgs][R] per-workgroup gradient packets
  float* slab_g;                 // [gram_wgs][NBLK * 1024] per-workgroup Gram blocks
  int num_wgs;                   // pass-kernel grid
  int gram_wgs;                  // workgroups [0, gram_wgs) add the Gram tile of subsample slots [64 wg, 64 wg + 64)
  int red_wgs;                   // reduce-kernel grid
  int passes;                    // trial points evaluated after the start point
  // Gram subsample: the global path range is cut into 8 aligned blocks and
  // the first gram_blk paths of each block are used (aligned prefixes of a
  // Sobol sequence are nets; the same global subsample at world size 1, 2,
  // 4, 8): slot j of this rank = local path (j / gram_blk) * gram_blk_stride + j % gram_blk
  int gram_blk;
  int gram_blk_stride;
  float inv_ns;                  // 1 / (global Gram subsample size)
  float inv_n;                   // 1 / (global path count)
  float lam0, lam_up, lam_down, lam_min, lam_max, ridge;
  // after the last pass, the parameter bias_index (the bond holding's output
  // bias) takes an exact 1-D Newton step: the value fit's residual mean over
  // all paths becomes zero, so no drift accumulates over the dates; -1: off
  int bias_index;
  int weights_only;              // 1: publish the weights only (no FitState / loss history: a bias refit
                                 // after an Adam fit, passes = 0)
  int damping;                   // 0: lam x lam_down / x lam_up on accept / reject; 1: Nielsen (gain ratio)
  // adaptive pass budget: from the solve of pass stop_min on, an accepted
  // pass that lowers the best loss by less than stop_tol (relative) ends the
  // fit (a rejection never does); the
  // remaining launches of the fit return at once (stop_tol = 0: off)
  int stop_min;
  float stop_tol;
  // pass kernel: the waves of the gram_wgs Gram workgroups take gram_skip
  // path blocks fewer than an even split (their Gram tile follows the paths)
  int gram_skip;
  // independent fits in one launch (grid y = instance k; k's state at
  // state + k LMS_FLOATS, reduced block at red + k LM_RED, slabs at k x one
  // instance's slab size): the multi-start exploration of a first date
  int inst;
  // 1: exploration fits - the last solve publishes nothing to the NetWeights /
  // FitState (k_lm_select picks the start point of the polish fit)
  int explore;
  // > 0: the fit's initial damping is max(state[LMS_LAM] x lam_carry, lam_min)
  // (the previous fit's final damping on this state), else lam0
  float lam_carry;
  float diag_floor;              // damping diagonal max(2 G_ii, diag_floor x mean 2 G_ii) (Marquardt scaling floor)
  const float* w0;               // [inst][LM_NPMAX] start weights (nullptr: the canonical NetWeights)
  // 1: the start weights were fitted on inputs standardised with (ren_mu,
  // ren_isd); the first layer is re-expressed for this fit's (fmu, fisd), so
  // the warm start is the previous date's hedge as a function of the RAW state
  // (the reference's warm start: raw features)
  int renorm;
  int pad1;
  float ren_mu[MAXIN];
  float ren_isd[MAXIN];
  // > 0: after the last pass the output layer's out_n parameters (the last
  // ones) take the exact Newton step 2 G_oo d = -g_o (the value is linear in
  // them); 0: only the bond bias (bias_index) does
  int out_n;
  float out_mu;                  // its Marquardt damping: A_ii = 2 G_ii (1 + out_mu) + ridge x mean diagonal
  // 1: the last LM_OUTG_TAIL passes accumulate the full-batch output-layer
  // Gram matrix (slab_o -> red[LM_RED_OUTG]); the output step then uses it
  int out_gram;
  // > 0: trust region of the output step - ||d|| <= out_tr x max(||w_o||,
  // 1e-3 sqrt(out_n)) (w_o the output weights it starts from); a longer step
  // is scaled back onto the boundary (its exact loss change follows: the
  // loss is quadratic along d).  0: off
  float out_tr;
  float* slab_o;                 // [num_wgs][3][1024] per-workgroup output-layer Gram tiles (MFMA layout)
  // 1: the Gram subsample is read from gfeat / gprice ([ns] per feature /
  // traded asset, slot order = the global subsample, simulated identically on
  // every rank), so every rank builds the same Gram matrix and the data-
  // parallel exchange carries only [g | stats | output Gram]; 0: slot j reads
  // local path (j / gram_blk) * gram_blk_stride + j % gram_blk of the shard
  // (this rank's part of the subsample; the Gram is then summed over ranks)
  const float* gfeat[MAXIN];
  const float* gprice[MAXIN];
  int gram_side;
  // pinball fits (TrainDesc.loss == LOSS_PINBALL): IRLS Gram weights
  // 1 / (2 max(|r|, delta)), delta = max(q_delta, q_kappa x the mean |r| of
  // the path's 64-path Gram tile) (target units)
  float q_delta;
  float q_kappa;
  // data parallel, every rank building the same Gram (gram_side): the
  // gradient region [g | stats | output Gram] is summed over the ranks INSIDE
  // k_lm_reduce (its packet / output-Gram workgroups push to the peers'
  // mailboxes, raise one flag each, wait for the peers' same flag and sum in
  // rank order; the pass kernel advances the exchange counter): no extra
  // launch per pass.  0: single rank, or the separate exchange kernels
  LmDpDesc dp;
  int dp_fused;
  // > 0: wave w of the pass grid takes the contiguous path blocks
  // [w leaf_blocks, (w + 1) leaf_blocks) (128 paths each; gram_skip unused):
  // the per-wave partial sums are then the same "leaves" of the global path
  // range at every world size (a rank's shard is a contiguous run of whole
  // leaves), and with the reduce's contiguous-halves trees the summed
  // gradient is bitwise independent of the world size.  0: cyclic blocks
  int leaf_blocks;
  // pinball fits on the simulated global subsample (gram_side): the targets
  // of its paths ([gram_wgs x 64]: V_{t+1} evaluated on the subsample at the
  // date boundary, driver.BackwardInduction), so the IRLS weights - and the
  // Gram - are the same on every rank; nullptr for MSE fits (J needs no target)
  const float* gtarget;
  // first workgroup of the Gram tiles: 0 = the first gram_wgs path workgroups
  // build them (after their share of the paths, gram_skip balancing);
  // num_wgs = Gram-only workgroups after the path grid, which a second
  // workgroup slot of the path workgroups' CUs runs beside them (the pass
  // kernel fits two workgroups per CU), so every path workgroup takes the
  // same share of the paths (the contiguous-leaf schedule's balance)
  int gram_base;
  int pad4;
};

// Multi-start selection block (k_lm_select): candidate c = (rank, instance)
// holds [final best loss, final damping, weights (LM_NPMAX)] at c * LM_SEL_W;
// packed by every rank into its own segment, summed over the ranks (the LM
// exchange), then every rank picks the same candidate.
constexpr int LM_SEL_W = LM_NPMAX + 2;
constexpr int LM_SEL_MAX = 64;          // candidates (world x instances)


// Eval stats slab columns
enum EvalStat : int {
  ES_V = 0, ES_V2 = 1, ES_RES = 2, ES_RES2 = 3, ES_ABSRES = 4, ES_APE = 5, ES_PRED1 = 6,
  ES_COUNT = 7, ES_HOLD = 8 /* 8 entries */, ES_HOLD2 = 16 /* 8 entries */, ES_RESMIN = 24,
  ES_RESMAX = 25
};

struct SimDesc {
  int model;                     // SimModel
  int n_local;
  long long path_offset;         // global index of local path 0 (Sobol index)
  int n_fine;                    // fine grid points incl. t=0
  int reduction;                 // store every `reduction` fine steps
  int n_coarse;                  // stored points
  int na;                        // assets (basket)
  int fp64;                      // recursion in double
  int parity;                    // reference quirks (SV sqrt of negative -> NaN, Q3 lambda index)
  const uint32_t* sv1; const uint32_t* shift1; int dims1;   // Sobol table A
  const uint32_t* sv2; const uint32_t* shift2; int dims2;   // Sobol table B (SV / mortality)
  double s0[MAXIN], mu[MAXIN], sigma[MAXIN];
  double chol[MAXIN * MAXIN];
  double dt;
  double inv_norm[MAXIN];
  // SV / Heston
  double v0, a, b, c, kappa, theta, xi, rho;
  // mortality
  double l0, lc, eta; int n0; uint32_t seed;
  float* out;                    // [n_coarse][na][n_local]
  float* out2;                   // second coarse output (vol / N-fraction)  [n_coarse][n_local]
  float* out3;                   // third coarse output (lambda)             [n_coarse][n_local]
  float* final_out;              // terminal fine value(s) [na][n_local]
  float* final2_out;             // terminal fine N-fraction [n_local]
  // SV_REF: time scale of the calibrated (a, b, c) in fine steps; 0 = the
  // reference recursion (no dt on the mean reversion, Q5), > 0 = corrected
  // CIR-on-sigma with every rate in calibration-day units: a(b-v) dt*tscale,
  // c sqrt(v dt*tscale) (tscale = 252 trading days per year)
  double sv_tscale;
  int scheme;                    // HESTON: 0 full-truncation Euler, 1 Andersen QE (martingale-corrected)
  int pad0;
  // path-index map (the LM Gram subsample simulated on every rank): local path
  // p is global path path_offset + (p / map_blk) * map_stride + p % map_blk;
  // map_blk = 0: contiguous (path_offset + p)
  long long map_blk;
  long long map_stride;
};

enum HestonScheme : int { HESTON_EULER = 0, HESTON_QE = 1 };

enum SimModel : int {
  SIM_GBM_ARITH = 0,   // Y_t = Y_{t-1}(1 + mu dt + sigma sqrt(dt) Z)   (RP:64-65)
  SIM_GBM_LOG = 1,     // log-Euler / exact GBM                          (EO:161-165)
  SIM_SV_REF = 2,      // reference "CIR-on-sigma" SV                    (RP:282-289)
  SIM_HESTON = 3,      // full-truncation Heston, rho-correlated
  SIM_BASKET = 4,      // correlated log-GBM basket (Cholesky)
  SIM_MORTALITY = 5,   // lambda Euler + binomial survivors             (RP:71-84)
};

}  // namespace rph
