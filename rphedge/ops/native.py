"""ctypes bindings to the in-tree native library ``rphedge/_lib/librphedge.so``.

The library (HIP kernels for gfx950 + C++ runtime: hipGraph capture, RCCL
communicator) exposes a plain C ABI.  ``torch`` is imported first so that the
HIP runtime (``libamdhip64.so.7``) and RCCL (``librccl.so.1``) already loaded
by torch are reused by the dynamic loader — one HIP runtime per process,
device pointers from torch tensors are valid in our kernels.

On a machine with a GPU the native library is mandatory: every op raises if it
is missing (no silent eager fallback).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch  # noqa: F401  (must be loaded before librphedge.so)

from . import layout as L

# RPH_NATIVE_LIB=debug|asan selects the variant built by `python -m rphedge.build --debug|--asan`;
# a path ending in .so loads that exact library (A/B of two builds, tools/ab_presets.sh)
_LIB_ENV = os.environ.get("RPH_NATIVE_LIB", "")
_LIB_PATH = Path(_LIB_ENV).resolve() if _LIB_ENV.endswith(".so") else Path(__file__).resolve().parent.parent / "_lib" / (
    {"debug": "librphedge_debug.so", "asan": "librphedge_asan.so"}.get(_LIB_ENV, "librphedge.so"))
_lib = None
_load_error: str | None = None

MAXIN, MAXHOLD = 8, 8
VP = C.c_void_p


class TrainDesc(C.Structure):
    _fields_ = [
        ("feat", VP * MAXIN), ("price", VP * MAXHOLD), ("target", VP),
        ("wts", VP), ("opt", VP), ("fit", VP), ("lr_sched", VP),
        ("slab", VP), ("counter", VP), ("grad_out", VP),
        ("bond", C.c_float), ("alpha", C.c_float), ("quantile", C.c_float), ("inv_batch", C.c_float),
        ("loss", C.c_int), ("n_local", C.c_int), ("batch", C.c_int), ("steps_per_epoch", C.c_int),
        ("chunk_log2", C.c_int), ("shuffle", C.c_int), ("seed", C.c_uint32), ("fused_update", C.c_int),
        ("num_wgs", C.c_int), ("nin", C.c_int), ("h", C.c_int), ("nout", C.c_int), ("head", C.c_int),
        ("acc", VP), ("deterministic", C.c_int), ("stamps", VP),
        ("dp_world", C.c_int), ("dp_rank", C.c_int), ("dp_mbox", VP * 8), ("dp_flags", VP * 8),
        ("dp_counter", VP), ("dp_error", VP), ("mfma_fp32", C.c_int), ("lag", VP), ("variant", C.c_int),
        ("fit_init", VP), ("fmu", C.c_float * MAXIN), ("fisd", C.c_float * MAXIN),
    ]

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        for f in range(MAXIN):  # identity standardisation unless the backend sets one
            self.fisd[f] = 1.0


class EvalDesc(C.Structure):
    _fields_ = [
        ("feat", VP * MAXIN), ("price_t", VP * MAXHOLD), ("price_t1", VP * MAXHOLD), ("target", VP),
        ("wa", VP), ("wb", VP), ("g_base", VP), ("v_out", VP), ("hold_out", VP * MAXHOLD),
        ("resid_out", VP), ("pred1_out", VP), ("stats", VP),
        ("bond_t", C.c_float), ("bond_t1", C.c_float), ("alpha", C.c_float), ("blend_c", C.c_float),
        ("hold_c", C.c_float),
        ("n_local", C.c_int), ("num_wgs", C.c_int), ("nin", C.c_int), ("h", C.c_int), ("nout", C.c_int),
        ("head", C.c_int), ("fmu", C.c_float * MAXIN), ("fisd", C.c_float * MAXIN),
        ("snap_a", VP), ("snap_b", VP),
    ]

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        for f in range(MAXIN):
            self.fisd[f] = 1.0


class PnlDesc(C.Structure):
    _fields_ = [
        ("feat", VP * MAXIN), ("feat_ts", C.c_longlong * MAXIN), ("price", VP * MAXHOLD),
        ("price_ts", C.c_longlong * MAXHOLD), ("snap", VP), ("fmu", VP), ("fisd", VP), ("bond", VP),
        ("w0", VP), ("payoff", VP), ("pnl_out", VP), ("stats", VP),
        ("alpha", C.c_float), ("hold_c", C.c_float), ("wealth0", C.c_float), ("has_b", C.c_int),
        ("n_local", C.c_int), ("n_dates", C.c_int), ("num_wgs", C.c_int),
        ("nin", C.c_int), ("h", C.c_int), ("nout", C.c_int), ("head", C.c_int),
    ]


class LmDpDesc(C.Structure):
    _fields_ = [
        ("mbox", VP * 8), ("counter", VP), ("error", VP),
        ("world", C.c_int), ("rank", C.c_int), ("pitch", C.c_int), ("fault", C.c_int),
    ]


class LmDesc(C.Structure):
    _fields_ = [
        ("state", VP), ("slab_b", VP), ("slab_g", VP),
        ("num_wgs", C.c_int), ("gram_wgs", C.c_int), ("red_wgs", C.c_int), ("passes", C.c_int),
        ("gram_blk", C.c_int), ("gram_blk_stride", C.c_int), ("inv_ns", C.c_float), ("inv_n", C.c_float),
        ("lam0", C.c_float), ("lam_up", C.c_float), ("lam_down", C.c_float), ("lam_min", C.c_float),
        ("lam_max", C.c_float), ("ridge", C.c_float), ("bias_index", C.c_int), ("weights_only", C.c_int),
        ("damping", C.c_int), ("stop_min", C.c_int), ("stop_tol", C.c_float), ("gram_skip", C.c_int),
        ("inst", C.c_int), ("explore", C.c_int), ("lam_carry", C.c_float), ("diag_floor", C.c_float), ("w0", VP),
        ("renorm", C.c_int), ("pad1", C.c_int), ("ren_mu", C.c_float * MAXIN), ("ren_isd", C.c_float * MAXIN),
        ("out_n", C.c_int), ("out_mu", C.c_float), ("out_gram", C.c_int), ("out_tr", C.c_float),
        ("slab_o", VP),
        ("gfeat", VP * MAXIN), ("gprice", VP * MAXIN), ("gram_side", C.c_int), ("q_delta", C.c_float), ("q_kappa", C.c_float),
        ("dp", LmDpDesc), ("dp_fused", C.c_int), ("leaf_blocks", C.c_int), ("gtarget", VP),
        ("gram_base", C.c_int), ("pad4", C.c_int),
    ]

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.inst = 1  # one fit per launch unless a multi-start exploration sets more


class SimDesc(C.Structure):
    _fields_ = [
        ("model", C.c_int), ("n_local", C.c_int), ("path_offset", C.c_longlong),
        ("n_fine", C.c_int), ("reduction", C.c_int), ("n_coarse", C.c_int), ("na", C.c_int),
        ("fp64", C.c_int), ("parity", C.c_int),
        ("sv1", VP), ("shift1", VP), ("dims1", C.c_int),
        ("sv2", VP), ("shift2", VP), ("dims2", C.c_int),
        ("s0", C.c_double * MAXIN), ("mu", C.c_double * MAXIN), ("sigma", C.c_double * MAXIN),
        ("chol", C.c_double * (MAXIN * MAXIN)), ("dt", C.c_double), ("inv_norm", C.c_double * MAXIN),
        ("v0", C.c_double), ("a", C.c_double), ("b", C.c_double), ("c", C.c_double),
        ("kappa", C.c_double), ("theta", C.c_double), ("xi", C.c_double), ("rho", C.c_double),
        ("l0", C.c_double), ("lc", C.c_double), ("eta", C.c_double), ("n0", C.c_int), ("seed", C.c_uint32),
        ("out", VP), ("out2", VP), ("out3", VP), ("final_out", VP), ("final2_out", VP),
        ("sv_tscale", C.c_double), ("scheme", C.c_int), ("pad0", C.c_int),
        ("map_blk", C.c_longlong), ("map_stride", C.c_longlong),
    ]


def _expected_layout() -> list[int]:
    f = 4
    T, E, S = TrainDesc, EvalDesc, SimDesc
    return [
        L.NETW_FLOATS * f, L.OPT_FLOATS * f, L.FIT_FLOATS * f,
        L.W_CUR * f, L.O_T * f, L.O_LR * f, L.O_NAN * f,
        L.F_BEST * f, L.F_STOPPED * f, L.F_EPOCH * f, L.F_LAST_LOSS * f, L.F_RESTORE_END * f, L.F_HIST * f,
        C.sizeof(T), T.price.offset, T.target.offset, T.wts.offset, T.lr_sched.offset, T.slab.offset,
        T.counter.offset, T.grad_out.offset, T.bond.offset, T.inv_batch.offset, T.loss.offset, T.seed.offset,
        T.num_wgs.offset, T.head.offset, T.acc.offset, T.deterministic.offset, T.stamps.offset,
        T.dp_world.offset, T.dp_mbox.offset, T.dp_flags.offset, T.dp_counter.offset, T.dp_error.offset,
        T.fit_init.offset, T.fmu.offset, T.fisd.offset,
        C.sizeof(E), E.price_t.offset, E.price_t1.offset, E.target.offset, E.wa.offset, E.g_base.offset,
        E.v_out.offset, E.hold_out.offset, E.resid_out.offset, E.pred1_out.offset, E.stats.offset,
        E.bond_t.offset, E.hold_c.offset, E.n_local.offset, E.head.offset, E.fmu.offset, E.fisd.offset,
        E.snap_a.offset, E.snap_b.offset,
        C.sizeof(PnlDesc), PnlDesc.feat_ts.offset, PnlDesc.price.offset, PnlDesc.price_ts.offset,
        PnlDesc.snap.offset, PnlDesc.bond.offset, PnlDesc.pnl_out.offset, PnlDesc.stats.offset,
        PnlDesc.alpha.offset, PnlDesc.has_b.offset, PnlDesc.n_dates.offset, PnlDesc.head.offset,
        C.sizeof(LmDesc), LmDesc.slab_b.offset, LmDesc.slab_g.offset, LmDesc.num_wgs.offset,
        LmDesc.passes.offset, LmDesc.gram_blk.offset, LmDesc.inv_ns.offset, LmDesc.lam0.offset,
        LmDesc.ridge.offset, LmDesc.bias_index.offset, LmDesc.weights_only.offset, LmDesc.damping.offset, LmDesc.stop_tol.offset, LmDesc.gram_skip.offset,
        LmDesc.inst.offset, LmDesc.lam_carry.offset, LmDesc.w0.offset, LmDesc.renorm.offset,
        LmDesc.ren_isd.offset, LmDesc.out_n.offset, LmDesc.gfeat.offset, LmDesc.gprice.offset,
        LmDesc.gram_side.offset, LmDesc.q_delta.offset, LmDesc.dp.offset, LmDesc.dp_fused.offset, LmDesc.gtarget.offset, LmDesc.gram_base.offset, C.sizeof(LmDesc),
        L.LMS_LFIN, L.LMS_FAILTOT, L.LM_SEL_W, L.LM_DP_PITCH,
        C.sizeof(LmDpDesc), LmDpDesc.counter.offset, LmDpDesc.world.offset, LmDpDesc.pitch.offset,
        L.LM_NPMAX, L.LM_RED, L.LMS_BEST, L.LMS_FLOATS,
        L.LM_SPEC, L.LMS_SPEC_W, L.LMS_SLOTS, L.LM_SLOT, L.LSS_LBEST, L.LSS_STOP,
        C.sizeof(S), S.path_offset.offset, S.sv1.offset, S.dims1.offset, S.sv2.offset, S.dims2.offset,
        S.s0.offset, S.chol.offset, S.dt.offset, S.inv_norm.offset, S.v0.offset, S.rho.offset, S.l0.offset,
        S.n0.offset, S.seed.offset, S.out.offset, S.final2_out.offset, S.sv_tscale.offset, S.scheme.offset,
        S.map_blk.offset, S.map_stride.offset,
        L.LAG_SLOTS,
    ]


def _bind(lib):
    sig = {
        "rph_last_error": (C.c_char_p, []),
        "rph_layout": (C.c_int, [C.POINTER(C.c_longlong), C.c_int]),
        "rph_device_info": (C.c_int, [C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_longlong),
                                      C.c_char_p, C.c_int]),
        "rph_memset_async": (C.c_int, [VP, C.c_int, C.c_longlong, VP]),
        "rph_stream_sync": (C.c_int, [VP]),
        "rph_graph_begin": (C.c_int, [VP]),
        "rph_graph_end": (C.c_int, [VP, C.POINTER(VP), C.POINTER(C.c_longlong)]),
        "rph_graph_launch": (C.c_int, [VP, VP]),
        "rph_graph_destroy": (C.c_int, [VP]),
        "rph_nccl_unique_id": (C.c_int, [C.c_char_p]),
        "rph_nccl_init": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.POINTER(VP)]),
        "rph_nccl_allreduce_f32": (C.c_int, [VP, VP, C.c_longlong, VP]),
        "rph_nccl_allreduce_f64": (C.c_int, [VP, VP, C.c_longlong, VP]),
        "rph_nccl_allreduce_u32": (C.c_int, [VP, VP, C.c_longlong, VP]),
        "rph_nccl_destroy": (C.c_int, [VP]),
        "rph_net_nparams": (C.c_int, [C.c_int] * 4 + [C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "rph_train_step": (C.c_int, [C.POINTER(TrainDesc), C.c_int, C.c_int, VP]),
        "rph_train_update": (C.c_int, [C.POINTER(TrainDesc), C.c_int, C.c_int, VP]),
        "rph_train_fit": (C.c_int, [C.POINTER(TrainDesc), C.c_int, VP]),
        "rph_train_lag_step": (C.c_int, [C.POINTER(TrainDesc), C.c_int, C.c_int, VP]),
        "rph_train_lag_finalize": (C.c_int, [C.POINTER(TrainDesc), C.c_int, VP]),
        "rph_train_lag_fit": (C.c_int, [C.POINTER(TrainDesc), C.c_int, VP]),
        "rph_train_ticket_fit": (C.c_int, [C.POINTER(TrainDesc), C.c_int, VP]),
        "rph_eval": (C.c_int, [C.POINTER(EvalDesc), VP]),
        "rph_pnl": (C.c_int, [C.POINTER(PnlDesc), VP]),
        "rph_lm_shape": (C.c_int, [C.c_int] * 4 + [C.POINTER(C.c_int)] * 3),
        "rph_lm_pass_wps": (C.c_int, [C.c_int] * 4),
        "rph_lm_eval": (C.c_int, [C.POINTER(TrainDesc), C.POINTER(LmDesc), VP, C.c_int, VP]),
        "rph_lm_solve": (C.c_int, [C.POINTER(TrainDesc), C.POINTER(LmDesc), VP, C.c_int, VP]),
        "rph_lm_fit": (C.c_int, [C.POINTER(TrainDesc), C.POINTER(LmDesc), VP, VP]),
        "rph_lm_dp_exchange": (C.c_int, [C.POINTER(LmDpDesc), VP, C.c_int, C.c_int, VP]),
        "rph_lm_select": (C.c_int, [C.POINTER(TrainDesc), C.POINTER(LmDesc), VP, VP, C.c_int, C.c_int, C.c_int,
                                    C.c_int, VP]),
        "rph_sobol_normal": (C.c_int, [VP, C.c_int, C.c_int, VP, VP, C.c_longlong, C.c_int, C.c_int, VP]),
        "rph_simulate": (C.c_int, [C.POINTER(SimDesc), VP]),
        "rph_payoff": (C.c_int, [C.c_int, C.c_int, C.c_int, VP, VP, C.c_float, VP, VP, VP]),
        "rph_radix_hist": (C.c_int, [VP, C.c_longlong, C.c_uint32, C.c_uint32, C.c_int, C.c_int, VP, VP]),
        "rph_ipc_alloc": (C.c_int, [C.c_longlong, C.POINTER(VP), C.c_char_p]),
        "rph_ipc_open": (C.c_int, [C.c_char_p, C.POINTER(VP)]),
        "rph_ipc_close": (C.c_int, [VP]),
        "rph_free": (C.c_int, [VP]),
        "rph_ipc_handle_size": (C.c_int, []),
        "rph_ipc_is_finegrained": (C.c_int, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def load(required: bool | None = None):
    """Load (building if needed) the native library.  ``required`` defaults to
    True whenever a GPU is visible."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if required is None:
        required = torch.cuda.is_available()
    try:
        if _LIB_ENV.endswith(".so") and not _LIB_PATH.exists():
            raise FileNotFoundError(f"RPH_NATIVE_LIB={_LIB_ENV} does not exist (it is never built implicitly)")
        if not _LIB_PATH.exists() or os.environ.get("RPH_REBUILD"):
            from .. import build as _build

            v = os.environ.get("RPH_NATIVE_LIB", "")
            _build.build(debug=v == "debug", asan=v == "asan")
        lib = C.CDLL(str(_LIB_PATH), mode=C.RTLD_GLOBAL)
        _bind(lib)
        cap = 256
        buf = (C.c_longlong * cap)()
        n = lib.rph_layout(buf, cap)
        got = list(buf[:n])
        exp = _expected_layout()
        if got != exp:
            raise RuntimeError(f"native/ctypes layout mismatch:\n native={got}\n python={exp}")
        _lib = lib
        return lib
    except Exception as e:  # pragma: no cover - exercised on broken installs only
        _load_error = f"{type(e).__name__}: {e}"
        if required:
            raise RuntimeError(f"rphedge native library unavailable on a GPU machine: {_load_error}") from e
        return None


def available() -> bool:
    return load(required=False) is not None


def _check(rc: int, what: str):
    if rc != 0:
        msg = _lib.rph_last_error().decode() if _lib is not None else ""
        raise RuntimeError(f"{what} failed with code {rc}: {msg}")


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(stream=None) -> int:
    """HIP stream handle of a torch stream (None: the current stream; an int is
    taken as a raw handle, 0 = the null stream)."""
    if isinstance(stream, int):
        return stream
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


# ---------------------------------------------------------------------------
# thin wrappers
# ---------------------------------------------------------------------------
def net_nparams(nin: int, h: int, nout: int, head: int) -> tuple[int, int]:
    lib = load(required=True)
    p, r = C.c_int(), C.c_int()
    if lib.rph_net_nparams(nin, h, nout, head, C.byref(p), C.byref(r)) != 0:
        raise ValueError(f"unsupported hedge network shape nin={nin} h={h} nout={nout} head={head}")
    return p.value, r.value


def sobol_normal(out: torch.Tensor, table, offset: int = 0, raw: bool = False, stream=None):
    lib = load(required=True)
    sv, sh, dims = table
    n, d = out.shape
    assert d <= dims
    fp64 = 1 if out.dtype == torch.float64 else 0
    _check(lib.rph_sobol_normal(ptr(out), n, d, ptr(sv), ptr(sh), int(offset), fp64, int(raw),
                                stream_handle(stream)), "rph_sobol_normal")


def simulate(desc: SimDesc, stream=None):
    lib = load(required=True)
    _check(lib.rph_simulate(C.byref(desc), stream_handle(stream)), "rph_simulate")


def train_step(desc: TrainDesc, step: int, epoch: int, stream=None):
    _check(_lib.rph_train_step(C.byref(desc), int(step), int(epoch), stream_handle(stream)), "rph_train_step")


def train_fit(desc: TrainDesc, epochs: int, stream=None):
    """One persistent launch for a whole fit (csrc/hedge_fit.h); desc.counter
    (>= 2 u32) and desc.acc (3 x 8 x R floats) must be zeroed before it."""
    _check(_lib.rph_train_fit(C.byref(desc), int(epochs), stream_handle(stream)), "rph_train_fit")


def train_lag_step(desc: TrainDesc, k: int, epoch: int, stream=None):
    """Lagged-update step kernel k of a fit (csrc/hedge_lag.h)."""
    _check(_lib.rph_train_lag_step(C.byref(desc), int(k), int(epoch), stream_handle(stream)), "rph_train_lag_step")


def train_lag_fit(desc: TrainDesc, epochs: int, stream=None):
    """All steps + finalize of a lagged-schedule fit, launched from C++."""
    load(required=True)
    _check(_lib.rph_train_lag_fit(C.byref(desc), int(epochs), stream_handle(stream)), "rph_train_lag_fit")


def train_ticket_fit(desc: TrainDesc, epochs: int, stream=None):
    """All steps of a ticketed fit (fused update), launched from C++."""
    load(required=True)
    _check(_lib.rph_train_ticket_fit(C.byref(desc), int(epochs), stream_handle(stream)), "rph_train_ticket_fit")


def train_lag_finalize(desc: TrainDesc, K: int, stream=None):
    _check(_lib.rph_train_lag_finalize(C.byref(desc), int(K), stream_handle(stream)), "rph_train_lag_finalize")


def train_update(desc: TrainDesc, step: int, epoch: int, stream=None):
    _check(_lib.rph_train_update(C.byref(desc), int(step), int(epoch), stream_handle(stream)), "rph_train_update")


def eval_(desc: EvalDesc, stream=None):
    _check(_lib.rph_eval(C.byref(desc), stream_handle(stream)), "rph_eval")


def lm_shape(nin: int, h: int, nout: int, head: int):
    """(P, R, Gram blocks) of the LM kernels, or None."""
    lib = load(required=True)
    v = [C.c_int() for _ in range(3)]
    if lib.rph_lm_shape(nin, h, nout, head, *[C.byref(x) for x in v]) != 0:
        return None
    return tuple(int(x.value) for x in v)


def lm_pass_wps(nin: int, h: int, nout: int, head: int) -> int:
    """Pass workgroups per CU of the shape's plain LM pass body (1 or 2;
    csrc/hedge_narrow.h NarrowPairBody::WAVES_PER_SIMD)."""
    return int(load(required=True).rph_lm_pass_wps(nin, h, nout, head))


def lm_eval(desc: TrainDesc, lm: LmDesc, red_new: torch.Tensor, pass_: int, stream=None):
    _check(_lib.rph_lm_eval(C.byref(desc), C.byref(lm), ptr(red_new), int(pass_), stream_handle(stream)),
           "rph_lm_eval")


def lm_solve(desc: TrainDesc, lm: LmDesc, red_new: torch.Tensor, pass_: int, stream=None):
    _check(_lib.rph_lm_solve(C.byref(desc), C.byref(lm), ptr(red_new), int(pass_), stream_handle(stream)),
           "rph_lm_solve")


def lm_fit(desc: TrainDesc, lm: LmDesc, red_new: torch.Tensor, stream=None):
    """Whole single-rank Levenberg-Marquardt fit (csrc/hedge_lm.hip), launched from C++."""
    load(required=True)
    _check(_lib.rph_lm_fit(C.byref(desc), C.byref(lm), ptr(red_new), stream_handle(stream)), "rph_lm_fit")


def lm_select(desc: TrainDesc, lm: LmDesc, sel: torch.Tensor, main_state: torch.Tensor, world: int, rank: int,
              p: int, phase: int, stream=None):
    """Multi-start selection (k_lm_select): phase 0 packs this rank's exploration
    results into ``sel``, phase 1 picks the best candidate into the NetWeights
    and ``main_state``'s damping."""
    _check(_lib.rph_lm_select(C.byref(desc), C.byref(lm), ptr(sel), ptr(main_state), int(world), int(rank), int(p),
                              int(phase), stream_handle(stream)), "rph_lm_select")


def lm_dp_exchange(x: LmDpDesc, red: torch.Tensor, ng: int, p: int, stream=None):
    """All-reduce of the LM reduced block over the IPC mailboxes (k_lm_dp_exchange)."""
    load(required=True)
    _check(_lib.rph_lm_dp_exchange(C.byref(x), ptr(red), int(ng), int(p), stream_handle(stream)),
           "rph_lm_dp_exchange")


def pnl(desc: PnlDesc, stream=None):
    """Self-financing hedge P&L scan over the rebalancing dates (k_hedge_pnl)."""
    load(required=True)
    _check(_lib.rph_pnl(C.byref(desc), stream_handle(stream)), "rph_pnl")


def payoff(kind: int, s: torch.Tensor, out: torch.Tensor, strike: float, nfrac=None, wts=None, na: int = 1,
           stream=None):
    lib = load(required=True)
    n = out.numel()
    _check(lib.rph_payoff(kind, n, na, ptr(s), ptr(nfrac), float(strike), ptr(wts), ptr(out),
                          stream_handle(stream)), "rph_payoff")


def radix_hist(x: torch.Tensor, pmask: int, prefix: int, shift: int, nbins: int, hist: torch.Tensor, stream=None):
    lib = load(required=True)
    _check(lib.rph_radix_hist(ptr(x), x.numel(), pmask & 0xFFFFFFFF, prefix & 0xFFFFFFFF, shift, nbins, ptr(hist),
                              stream_handle(stream)), "rph_radix_hist")


def memset_async(t: torch.Tensor, value: int = 0, stream=None):
    lib = load(required=True)
    _check(lib.rph_memset_async(ptr(t), value, t.numel() * t.element_size(), stream_handle(stream)),
           "rph_memset_async")


def device_info(dev: int = 0) -> dict:
    lib = load(required=True)
    cus, lds = C.c_int(), C.c_int()
    hbm = C.c_longlong()
    name = C.create_string_buffer(128)
    _check(lib.rph_device_info(dev, C.byref(cus), C.byref(lds), C.byref(hbm), name, 128), "rph_device_info")
    return {"cus": cus.value, "lds_per_cu": lds.value, "hbm_bytes": hbm.value, "arch": name.value.decode()}


class Graph:
    """hipGraph captured from a stream with the native runtime."""

    def __init__(self):
        self.exec = None
        self.num_nodes = 0

    def capture_begin(self, stream=None):
        lib = load(required=True)
        self._stream = stream_handle(stream)
        _check(lib.rph_graph_begin(self._stream), "rph_graph_begin")

    def capture_end(self):
        ex = VP()
        nn = C.c_longlong()
        _check(_lib.rph_graph_end(self._stream, C.byref(ex), C.byref(nn)), "rph_graph_end")
        self.exec = ex.value
        self.num_nodes = nn.value

    def replay(self, stream=None):
        _check(_lib.rph_graph_launch(self.exec, stream_handle(stream)), "rph_graph_launch")

    def __del__(self):
        if self.exec is not None and _lib is not None:
            try:
                _lib.rph_graph_destroy(self.exec)
            except Exception:
                pass
            self.exec = None


class NcclComm:
    """RCCL communicator owned by the native runtime (one per process/GPU).

    The 128-byte unique id is created on rank 0 and broadcast via the
    torch.distributed store, then every rank calls ``ncclCommInitRank``.
    """

    def __init__(self, rank: int, world: int, store, tag: str = "rph_nccl"):
        lib = load(required=True)
        key = f"{tag}_uid"
        if rank == 0:
            buf = C.create_string_buffer(128)
            n = lib.rph_nccl_unique_id(buf)
            if n <= 0:
                _check(-1, "rph_nccl_unique_id")
            store.set(key, bytes(buf.raw[:128]))
        uid = store.get(key)
        comm = VP()
        _check(lib.rph_nccl_init(uid, world, rank, C.byref(comm)), "rph_nccl_init")
        self.comm = comm.value
        self.rank, self.world = rank, world

    def allreduce_(self, t: torch.Tensor, stream=None):
        fn = {torch.float32: _lib.rph_nccl_allreduce_f32, torch.float64: _lib.rph_nccl_allreduce_f64,
              torch.int32: _lib.rph_nccl_allreduce_u32}[t.dtype]
        _check(fn(self.comm, ptr(t), t.numel(), stream_handle(stream)), "rph_nccl_allreduce")

    def close(self):
        if self.comm is not None:
            _lib.rph_nccl_destroy(self.comm)
            self.comm = None


DP_SLOTS = 4


class IpcMailbox:
    """Peer-mapped mailboxes for the fused xGMI gradient all-reduce.

    Every rank allocates ``[DP_SLOTS][W][R]`` 8-byte entries (a float + flag
    pair per entry for the ticket path; a data-tagged {value, seq} granule for
    the lagged path) + ``[DP_SLOTS][W]`` flags,
    exports an IPC handle through the torch.distributed store and opens every
    peer's handle.  The step kernel's last-arriving workgroup then writes its
    packet straight into each peer's HBM over xGMI (no RCCL launch, no extra
    kernel per step)."""

    def __init__(self, rank: int, world: int, R: int, store, device, tag: str = "rph_mbox"):
        lib = load(required=True)
        if world > 8:
            raise ValueError("fused xGMI all-reduce supports up to 8 ranks (one node)")
        self.rank, self.world, self.R = rank, world, R
        data_bytes = DP_SLOTS * world * R * 8
        self.flag_off = (data_bytes + 255) // 256 * 256
        nbytes = self.flag_off + DP_SLOTS * world * 4 + 256
        hs = lib.rph_ipc_handle_size()
        buf = C.create_string_buffer(hs)
        p = VP()
        _check(lib.rph_ipc_alloc(nbytes, C.byref(p), buf), "rph_ipc_alloc")
        self.own = p.value
        self.finegrained = lib.rph_ipc_is_finegrained() == 1  # coherent-by-memory-type mailbox
        store.set(f"{tag}_{rank}", bytes(buf.raw[:hs]))
        self.ptrs, self.opened = [], []
        for q in range(world):
            if q == rank:
                self.ptrs.append(self.own)
                continue
            h = store.get(f"{tag}_{q}")
            pq = VP()
            _check(lib.rph_ipc_open(h, C.byref(pq)), "rph_ipc_open")
            self.ptrs.append(pq.value)
            self.opened.append(pq.value)
        self.counter = torch.zeros(4, dtype=torch.int32, device=device)
        self.error = torch.zeros(4, dtype=torch.int32, device=device)

    def fill(self, d: TrainDesc):
        d.dp_world, d.dp_rank = self.world, self.rank
        for q in range(self.world):
            d.dp_mbox[q] = self.ptrs[q]
            d.dp_flags[q] = self.ptrs[q] + self.flag_off
        d.dp_counter = self.counter.data_ptr()
        d.dp_error = self.error.data_ptr()

    def lm_desc(self) -> "LmDpDesc":
        """Descriptor of this mailbox for the LM block exchange (k_lm_dp_exchange,
        and the exchange fused into k_lm_reduce; allocated with R >= LM_DP_PITCH
        entries per row)."""
        x = LmDpDesc()
        for q in range(self.world):
            x.mbox[q] = self.ptrs[q]
        x.counter, x.error = self.counter.data_ptr(), self.error.data_ptr()
        x.world, x.rank, x.pitch = self.world, self.rank, self.R
        return x

    def check(self):
        if int(self.error[0].item()) != 0:
            raise RuntimeError("fused xGMI all-reduce: a peer rank did not arrive (timeout)")

    def close(self):
        for p in self.opened:
            _lib.rph_ipc_close(p)
        self.opened = []
        if self.own is not None:
            _lib.rph_free(self.own)
            self.own = None
