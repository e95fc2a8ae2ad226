"""Data parallelism over Monte-Carlo paths.

One process per GPU.  The global path set ``[0, 2^m)`` is split into
contiguous shards ``[r*n/W, (r+1)*n/W)``; Sobol points are index-addressable so
every rank generates its own shard with no communication.  Per optimizer step
the 512-byte gradient packet (grads + loss/metric partials) is summed over
ranks INSIDE the step kernel (default ``RPH_DP=xgmi``): IPC-mapped peer
mailboxes, system-scope stores over xGMI, bounded in-kernel polls, identical
fixed-order sums on every rank (csrc/hedge_lag.h, csrc/hedge_core.h).
:func:`select_transport` probes that path once and falls back to ONE RCCL
all-reduce of the packet per step on the compute stream (graph-captured with
the step kernels, ``RPH_DP=rccl``).  Statistics, quantile histograms and the
bias-init P(OTM) use ``torch.distributed`` collectives (nccl = RCCL on ROCm;
gloo on CPU and for ranks sharing one GPU).

Sizing for xGMI: the per-step packet is latency-bound (one-shot), so the design
levers are one exchange per step with no extra launch, and large per-rank
batches (fewer steps); bucketing is moot at 512 B.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")
    comm: object = None          # native RCCL communicator (HIP path)
    initialized_here: bool = False
    dp_mode: str = "xgmi"        # xgmi: fused IPC all-reduce in the step kernel; rccl: RCCL + update kernel
    lm_dp_mode: str = "xgmi"     # LM reduced block: xgmi (k_lm_dp_exchange over IPC mailboxes) or rccl
    lm_comm: object = None       # RCCL communicator of the LM block when only its probe failed
    shared_device: bool = False  # several local ranks on ONE GPU (single-GPU rehearsal of the DP path)
    probe: dict | None = None    # select_transport's probe result (per-rank ok flags, chosen transport)

    @property
    def is_main(self) -> bool:
        return self.rank == 0


_INFO: DistInfo | None = None


def env_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def init(backend: str | None = None, device: str | None = None, native_comm: bool = True,
         timeout_s: float = 600.0) -> DistInfo:
    """Initialise (or reuse) the process group from torchrun env vars.

    ``backend``: 'nccl' (RCCL) on GPU, 'gloo' on CPU.  With ``native_comm`` on a
    GPU a native RCCL communicator is created for the training hot path.
    """
    global _INFO
    if _INFO is not None:
        return _INFO
    import datetime

    import torch.distributed as dist

    # the host driver supports dmabuf IPC only: the mailboxes' and RCCL's
    # cross-process mappings need the non-legacy IPC mode, set before the HIP
    # runtime initialises (external torchrun launches included)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    world = env_world()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = torch.cuda.is_available() and (device is None or str(device).startswith("cuda"))
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count())) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(dev)
    # the IPC-mapped xGMI mailboxes only reach peers on this node: the in-kernel
    # exchange is the default only when every rank is local (one node, <= 8 GPUs)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    one_node = local_world == world
    mode = os.environ.get("RPH_DP", "xgmi" if (world <= 8 and one_node) else "rccl")
    info = DistInfo(rank=rank, world=world, local_rank=local, device=dev, dp_mode=mode, lm_dp_mode=mode)
    if use_gpu:
        info.shared_device = int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) > torch.cuda.device_count()
    if world > 1:
        # RCCL refuses two ranks on one GPU ("duplicate GPU"): ranks sharing a
        # card (single-GPU rehearsal of the DP path) bootstrap over gloo; the
        # gradient exchange itself still runs in-kernel through IPC mailboxes
        be = backend or os.environ.get("RPH_DIST_BACKEND") or (
            "nccl" if use_gpu and not info.shared_device else "gloo")
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = {}
            if be == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(be, timeout=datetime.timedelta(seconds=timeout_s), **kw)
            info.initialized_here = True
        info.backend = be
        if use_gpu and native_comm and info.dp_mode == "rccl":
            from ..ops.native import NcclComm

            store = _store()
            info.comm = NcclComm(rank, world, store)
    _INFO = info
    return info


def _store():
    import torch.distributed as dist

    # the default group's store (c10d); prefixed keys avoid collisions
    from torch.distributed import distributed_c10d as c10d

    return c10d._get_default_store() if hasattr(c10d, "_get_default_store") else dist.distributed_c10d._get_default_store()


_MBOX_GEN = [0]  # mailboxes created by this process (every rank creates them in the same order)


def make_mailbox(info: DistInfo, R: int, tag: str = "rph_mbox", mode: str | None = None):
    """IPC mailbox for the fused xGMI all-reduce (None on 1 rank / CPU / rccl mode).

    Collective: every rank calls it in the same order.  The store key carries
    a per-process generation counter, so a second run in the same process (a
    sweep, repeated API calls) never picks up a peer's handle from an earlier
    run; the barrier after the exchange means no rank closes (frees) an old
    mailbox a peer might still be opening."""
    if info.world <= 1 or info.device.type != "cuda" or (mode or info.dp_mode) != "xgmi":
        return None
    from ..ops.native import IpcMailbox

    _MBOX_GEN[0] += 1
    err = None
    try:
        mb = IpcMailbox(info.rank, info.world, R, _store(), info.device, tag=f"{tag}_g{_MBOX_GEN[0]}")
    except Exception as e:  # still join the barrier: the peers must not pair it with a later collective
        mb, err = None, e
    barrier()
    if err is not None:
        raise err
    # ranks sharing one GPU cannot use schedules whose EVERY workgroup waits for
    # the peers (a peer's kernel may find no free CU): engine picks "ticket"
    mb.shared_device = info.shared_device
    return mb


def close_mailbox(mb):
    """Collective teardown of a mailbox: every rank's kernels are done with
    every peer buffer before any rank frees its own."""
    if mb is None:
        return
    if mb.own is not None and torch.cuda.is_available():
        torch.cuda.synchronize()
    barrier()
    mb.close()


class TorchComm:
    """All-reduce through the torch.distributed process group with the
    ``NcclComm.allreduce_(t, stream)`` interface: the stream is drained, the
    tensor summed (through the host under gloo) and written back before the
    next launch.  Eager only (not graph-capturable).  Two uses: the
    INDEPENDENT reference transport of the LM transport probe, and the LM
    fallback of ranks that share one GPU (RCCL refuses two ranks per card)."""

    def __init__(self, device):
        self.device = device

    def allreduce_(self, t: torch.Tensor, stream=None):
        if t.is_cuda:
            torch.cuda.synchronize(t.device)
        all_reduce_(t, "sum")
        if t.is_cuda:
            torch.cuda.synchronize(t.device)

    def close(self):
        pass


# the LM transport probe: a 1-8-8-2 net, 2^12 paths per rank, 2048-path global
# Gram subsample, output-layer Newton step (the output-Gram exchange rows too)
_PROBE_LOCAL_LOG2 = 12
_PROBE_GRAM = 2048
_PROBE_PASSES = 4
PROBE_RTOL = 1e-5  # fused fit vs the independent all-reduce fit (fp64 sums in another order)


def _probe_data(info: DistInfo, world_data: bool):
    """The probe's global problem, identical on every rank (fixed generator):
    this rank's shard and the simulated global Gram subsample."""
    from ..engine import DateData, gram_subsample
    from ..ops.paths import path_indices
    import numpy as np

    n = 1 << _PROBE_LOCAL_LOG2
    W = info.world
    g = torch.Generator().manual_seed(100)
    xa = torch.rand(n * W, generator=g) * 0.6 + 0.7
    ya = torch.relu(xa * 1.01 - 1.0) + 0.02 * torch.sin(9.0 * xa)
    x = xa[info.rank * n:(info.rank + 1) * n].to(info.device)
    y = ya[info.rank * n:(info.rank + 1) * n].to(info.device)
    ns, blk, stride = gram_subsample(n * W, _PROBE_GRAM)
    idx = torch.as_tensor(path_indices(ns, 0, (blk, stride)).astype(np.int64))
    gf = xa[idx].contiguous().to(info.device)
    kw = dict(gram_feats=[gf], gram_prices_next=[gf * 1.01]) if world_data else {}
    return DateData(feats=[x], prices_next=[x * 1.01], bond_next=1.0, target=y, prices_now=[x], **kw)


def _probe_lm_fit(info: DistInfo, mb, lmb=None, lm_comm=None, fault: int = 0):
    """One LM probe fit over the production exchange (``lmb``: the gradient
    region summed inside k_lm_reduce, LmDesc.dp_fused) or over ``lm_comm``
    (the split launches + an independent all-reduce).  Returns (weights,
    fused flag, clean flag)."""
    from ..engine import FitConfig, HipBackend, TrainConfig
    from ..models.hedge_mlp import NetSpec, init_weights

    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    n = 1 << _PROBE_LOCAL_LOG2
    be = HipBackend(spec, n, TrainConfig(batch_size=n * info.world, chunk_log2=6, lm_gram_paths=_PROBE_GRAM,
                                         lm_out_fix=True),
                    device=info.device, world=info.world, rank=info.rank, mailbox=mb, lm_mailbox=lmb,
                    lm_comm=lm_comm)
    if lmb is not None and fault:
        be._cache.get(("lm_dp",), lmb.lm_desc).fault = int(fault)
    data = _probe_data(info, world_data=True)
    w, o, f = be.new_weights(init_weights(spec, [0.5, 0.0])), be.new_opt(), be.new_fit()
    be.fit(w, o, f, data, FitConfig(epochs=_PROBE_PASSES, optimizer="lm", early_stopping=False), seed=5)
    torch.cuda.synchronize(info.device)
    clean = lmb is None or int(lmb.error[0].item()) == 0
    return w[: spec.nparams].double().clone(), bool(be.lm_last_fused), clean


def _probe_xgmi_local(info: DistInfo, mb, lmb, lm: bool) -> tuple[bool, torch.Tensor | None, dict]:
    """This rank's half of one probe: a tiny data-parallel fit over one of the
    in-kernel exchanges the runs use.

    packet: Keras-Adam steps over the fused packet exchange (``mb``, the
    lagged schedule).  lm: Levenberg-Marquardt passes over EXACTLY the
    production LM exchange - the global Gram subsample is given, so every
    rank builds the same Gram and the gradient region (+ the output-Gram rows)
    is summed inside k_lm_reduce (``lm_dp_sum_wave``) - and, as a reference,
    the same fit through the split launches with an independent
    torch.distributed all-reduce of the same region.  The probe passes only
    if the fused fit ran fused, is clean and matches the reference to
    PROBE_RTOL: a wrong sum that is identical on every rank fails too.
    Returns (ok, fitted weights, record)."""
    from ..engine import DateData, FitConfig, HipBackend, TrainConfig
    from ..models.hedge_mlp import NetSpec, init_weights

    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    rec: dict = {}
    if mb is None or (lm and lmb is None):
        return False, None, rec
    # fault injection (tests): RPH_PROBE_FAIL = packet | lm | both fails that
    # probe on every rank, or only on RPH_PROBE_FAIL_RANK; RPH_PROBE_FAULT=lm_drop
    # corrupts the fused LM sum itself (rank W-1 dropped on every rank)
    inj = os.environ.get("RPH_PROBE_FAIL", "")
    inj_rank = os.environ.get("RPH_PROBE_FAIL_RANK")
    injected = bool(inj and (inj == "both" or inj == ("lm" if lm else "packet")) and (
        inj_rank is None or int(inj_rank) == info.rank))
    if injected and not (lm and inj_rank is not None):
        return False, None, rec
    if lm:
        # the fused fit, then - on EVERY rank, whatever the fused fit did (a
        # raising rank must not skip the reference fit's collectives) - the
        # reference fit over the process group
        fault = 1 if os.environ.get("RPH_PROBE_FAULT", "") == "lm_drop" else 0
        wv = wr = None
        fused = clean = False
        if not injected:  # (a one-rank injection still joins the reference fit's collectives)
            try:
                wv, fused, clean = _probe_lm_fit(info, mb, lmb=lmb, fault=fault)
            except Exception as e:
                rec["exception"] = f"{type(e).__name__}: {e}"[:200]
        try:
            wr, _, _ = _probe_lm_fit(info, mb, lm_comm=TorchComm(info.device))
        except Exception as e:
            rec["exception_reference"] = f"{type(e).__name__}: {e}"[:200]
        if wv is None or wr is None:
            return False, wv, rec
        dev = float((wv - wr).abs().max().item() / max(float(wr.abs().max().item()), 1e-30))
        rec.update({"fused": fused, "clean": clean, "max_rel_dev_vs_allreduce": dev, "rtol": PROBE_RTOL,
                    "fault_injected": bool(fault)})
        ok = fused and clean and bool(torch.isfinite(wv).all()) and dev <= PROBE_RTOL
        return ok, wv, rec
    try:
        n = 1 << 12
        g = torch.Generator().manual_seed(100 + info.rank)          # different data per rank
        x = (torch.rand(n, generator=g) * 0.6 + 0.7).to(info.device)
        be = HipBackend(spec, n, TrainConfig(batch_size=n * info.world, chunk_log2=6, lm_gram_paths=2048),
                        device=info.device, world=info.world, rank=info.rank, mailbox=mb)
        data = DateData(feats=[x], prices_next=[x * 1.01], bond_next=1.0, target=torch.relu(x - 1.0),
                        prices_now=[x])
        w, o, f = be.new_weights(init_weights(spec, [0.5, 0.0])), be.new_opt(), be.new_fit()
        be.fit(w, o, f, data, FitConfig(epochs=4, patience=10 ** 6, early_stopping=False), seed=5)
        torch.cuda.synchronize(info.device)
        wv = w[: spec.nparams].double()
        clean = int(mb.error[0].item()) == 0
        return clean and bool(torch.isfinite(wv).all()), wv, {"clean": clean}
    except Exception as e:
        return False, None, {"exception": f"{type(e).__name__}: {e}"[:200]}


def select_transport(info: DistInfo) -> str:
    """Probe-then-choose, like a collective library's transport selection,
    separately for the two in-kernel exchanges: the Keras-Adam gradient packet
    (``info.dp_mode``) and the LM reduced block (``info.lm_dp_mode``).  Each
    keeps its xGMI mailbox exchange when a tiny DP fit over it is clean on
    every rank, the replicas agree bit for bit and (LM) the fit matches the
    same fit over an independent all-reduce; otherwise that exchange falls
    back to an RCCL all-reduce (ranks sharing one GPU: the torch.distributed
    group, RCCL refuses two ranks per card).  Runs once, outside any timed
    region; all ranks agree.

    Every rank issues the SAME collective sequence whatever its local outcome
    (per probe: min of the ok flags, max/min of the weights, min of the
    equality flag), so a failure seen by only some ranks cannot pair
    mismatched collectives (the LM reference fit's all-reduces run on every
    rank whose fused fit ran; a rank whose fit raised skips both, and the
    process group's timeout then surfaces it)."""
    if info.world <= 1 or info.device.type != "cuda" or info.dp_mode != "xgmi":
        return info.dp_mode
    from ..models.hedge_mlp import NetSpec
    from ..ops import layout as L

    def try_mailbox(R, tag):  # make_mailbox joins its barrier on every rank even when it raises
        try:
            return make_mailbox(info, R, tag=tag)
        except Exception:
            return None

    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    mb = try_mailbox(spec.red_width, "rph_probe")
    lmb = try_mailbox(L.LM_DP_PITCH, "rph_probe_lm")
    probe = {}
    for name, lm in (("packet", False), ("lm", True)):
        ok_l, wv, rec = _probe_xgmi_local(info, mb, lmb, lm)
        ok = torch.tensor([1.0 if ok_l else 0.0], dtype=torch.float64, device=info.device)
        all_reduce_(ok, "min")
        w = wv if (wv is not None and wv.numel() == spec.nparams) else \
            torch.zeros(spec.nparams, dtype=torch.float64, device=info.device)
        mx, mn = w.clone(), w.clone()
        all_reduce_(mx, "max")
        all_reduce_(mn, "min")
        same = torch.tensor([1.0 if bool(torch.equal(mx, mn)) else 0.0], dtype=torch.float64, device=info.device)
        all_reduce_(same, "min")
        all_ok = float(ok.item()) >= 1.0 and float(same.item()) >= 1.0
        probe[name] = {"local_ok": bool(ok_l), "all_ok": bool(float(ok.item()) >= 1.0),
                       "bitwise_equal_weights": bool(float(same.item()) >= 1.0),
                       "chosen": "xgmi" if all_ok else "rccl", **rec}
    # collective teardown with ONE unconditional barrier (a rank whose mailbox
    # creation failed holds None and must still join it)
    torch.cuda.synchronize(info.device)
    barrier()
    for m in (mb, lmb):
        if m is not None:
            try:
                m.close()
            except Exception:
                pass
    info.probe = probe
    info.lm_dp_mode = probe["lm"]["chosen"]
    from ..ops.native import NcclComm

    # fallback communicators are created here, collectively and outside any
    # graph capture (never lazily inside a captured fit); ranks sharing one
    # GPU fall back to the process group (RCCL refuses a duplicate GPU)
    def fallback(tag):
        return TorchComm(info.device) if info.shared_device else NcclComm(info.rank, info.world, _store(), tag=tag)

    if probe["packet"]["chosen"] != "xgmi":
        info.dp_mode = "rccl"
        info.comm = fallback("rph_fallback")
    elif info.lm_dp_mode != "xgmi":
        info.lm_comm = fallback("rph_lm_fallback")
    for k in ("packet", "lm"):
        if probe[k]["chosen"] != "xgmi":
            probe[k]["fallback_comm"] = "torch.distributed" if info.shared_device else "rccl"
    return info.dp_mode


def dist_world() -> int:
    """World size of the initialised process group (1 without one)."""
    import torch.distributed as dist

    return dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1


def shard(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """(offset, count) of the contiguous shard of ``rank``."""
    if n_total % world:
        raise ValueError(f"{n_total} paths not divisible by world size {world}")
    per = n_total // world
    return rank * per, per


def barrier():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def all_reduce_(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    """In-place all-reduce; device tensors go through the host when the
    process group is gloo (single-GPU multi-rank rehearsals)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        o = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        if t.is_cuda and dist.get_backend() == "gloo":
            h = t.detach().cpu()
            dist.all_reduce(h, op=o)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=o)
    return t


def all_reduce_scalar(x: float, op: str = "sum", device=None) -> float:
    dev = device or (_INFO.device if _INFO is not None else torch.device("cpu"))
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    return float(all_reduce_(t, op).item())


def shutdown():
    global _INFO
    import torch.distributed as dist

    for c in ((_INFO.comm, _INFO.lm_comm) if _INFO is not None else ()):
        if c is not None:
            try:
                c.close()
            except Exception:
                pass
    if _INFO is not None and _INFO.initialized_here and dist.is_initialized():
        dist.destroy_process_group()
    _INFO = None
