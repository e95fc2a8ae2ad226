"""Float-index layout of the device state blocks (mirror of csrc/rph_types.h).

Checked against the native library at load time (``rph_layout``)."""
PMAX = 2048
MAXHIST = 1024
EVAL_NSTAT = 32

# NetWeights: float w[2][PMAX]; float cur; pad[3]
NETW_FLOATS = 2 * PMAX + 4

# lagged-update state slot (csrc/hedge_lag.h): w, m, v [PMAX] + 16 scalars
LAG_FLOATS = 3 * PMAX + 16
# lagged-update accumulators: 3 rotating buffers x LAG_SLOTS replica rows x R
LAG_SLOTS = 16
W_CUR = 2 * PMAX

# OptState: m[PMAX], v[PMAX], t, lr, beta1, beta2, eps, nan_steps, pad0, pad1
OPT_FLOATS = 2 * PMAX + 8
O_M = 0
O_V = PMAX
O_T = 2 * PMAX
O_LR = O_T + 1
O_B1 = O_T + 2
O_B2 = O_T + 3
O_EPS = O_T + 4
O_NAN = O_T + 5

# FitState
F_WBEST = 0
F_BEST = PMAX
F_WAIT = PMAX + 1
F_STOPPED = PMAX + 2
F_EPOCH = PMAX + 3
F_PATIENCE = PMAX + 4
F_MAXEP = PMAX + 5
F_RESTORE = PMAX + 6
F_HASBEST = PMAX + 7
F_LOSS_SUM = PMAX + 8
F_LOSS_CNT = PMAX + 9
F_ABS_SUM = PMAX + 10
F_APE_SUM = PMAX + 11
F_LAST_LOSS = PMAX + 12
F_LAST_MAE = PMAX + 13
F_LAST_MAPE = PMAX + 14
F_RESTORE_END = PMAX + 15
F_HIST = PMAX + 16
FIT_FLOATS = F_HIST + MAXHIST

# eval stats columns
ES_V, ES_V2, ES_RES, ES_RES2, ES_ABSRES, ES_APE, ES_PRED1, ES_COUNT = range(8)
ES_HOLD = 8
ES_HOLD2 = 16
ES_RESMIN = 24
ES_RESMAX = 25

HEAD_FREE, HEAD_COMPLEMENT = 0, 1
LOSS_MSE, LOSS_PINBALL = 0, 1

SIM_GBM_ARITH, SIM_GBM_LOG, SIM_SV_REF, SIM_HESTON, SIM_BASKET, SIM_MORTALITY = range(6)
HESTON_EULER, HESTON_QE = 0, 1   # SimDesc.scheme (csrc/rph_types.h HestonScheme)

# Levenberg-Marquardt solver (csrc/rph_types.h LmState)
LM_NPMAX = 192
LM_TILE = 64
LM_GBLK_MAX = 21 * 1024
LM_OUTG = 64 * 65 // 2               # full-batch output-layer Gram, packed upper triangle (NU <= 64)
LM_OUTG_TAIL = 1                     # the last evaluation of an lm_out_fix fit carries it
LM_RED_OUTG = LM_GBLK_MAX + LM_NPMAX + 8
LM_RED = LM_RED_OUTG + LM_OUTG
LM_PASS_WGS_MAX = 512               # LM pass workgroups (csrc/rph_types.h)
LM_OG_MAX = 64
LMS_W = 0
LMS_RED = 2 * LM_NPMAX
LMS_BEST = LMS_RED + 2 * LM_RED      # host mirrors of the last solve
LMS_LAM = LMS_BEST + 1
LMS_NACC = LMS_BEST + 2
LMS_FAIL = LMS_BEST + 3
LMS_LFIN = LMS_BEST + 4             # the fit's final best loss (last solve)
LMS_FAILTOT = LMS_BEST + 5          # Cholesky failures of every fit on this state (never reset)
LM_SEL_W = LM_NPMAX + 2             # multi-start selection block: [loss, damping, weights] per candidate
LM_SEL_MAX = 64
LM_DP_WGS = 16
LM_DP_FLAGS = 128                   # fused exchange: per-workgroup flags after the LM_RED data entries
LM_DP_PITCH = LM_RED + LM_DP_FLAGS  # LM mailbox row pitch
LM_SPEC = 4
LMS_SPEC_LAM = LMS_FAIL + 8
LMS_SPEC_PRED = LMS_SPEC_LAM + LM_SPEC
LMS_SPEC_OK = LMS_SPEC_PRED + LM_SPEC
LMS_SPEC_W = LMS_SPEC_OK + LM_SPEC
LMS_SLOTS = LMS_SPEC_W + LM_SPEC * LM_NPMAX  # [2][LM_SLOT] scalars by pass parity
LMS_FLOATS = LMS_SLOTS + 16
LM_SLOT = 8
LSS_BEST, LSS_LAM, LSS_NU, LSS_PRED, LSS_COPY, LSS_SPEC_IDX, LSS_LBEST, LSS_STOP = range(8)


def lm_slot(pass_: int) -> int:
    """State index of the scalar slot the pass / solve kernels of pass ``pass_`` read."""
    return LMS_SLOTS + LM_SLOT * (int(pass_) & 1)
