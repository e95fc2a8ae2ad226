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
    shared_device: bool = False  # several local ranks on ONE GPU (single-GPU rehearsal of the DP path)

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

    world = env_world()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = torch.cuda.is_available() and (device is None or str(device).startswith("cuda"))
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count())) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(dev)
    info = DistInfo(rank=rank, world=world, local_rank=local, device=dev,
                    dp_mode=os.environ.get("RPH_DP", "xgmi" if world <= 8 else "rccl"))
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


def make_mailbox(info: DistInfo, R: int, tag: str = "rph_mbox"):
    """IPC mailbox for the fused xGMI all-reduce (None on 1 rank / CPU / rccl mode)."""
    if info.world <= 1 or info.device.type != "cuda" or info.dp_mode != "xgmi":
        return None
    from ..ops.native import IpcMailbox

    mb = IpcMailbox(info.rank, info.world, R, _store(), info.device, tag=tag)
    # ranks sharing one GPU cannot use schedules whose EVERY workgroup waits for
    # the peers (a peer's kernel may find no free CU): engine picks "ticket"
    mb.shared_device = info.shared_device
    return mb


def _probe_xgmi(info: DistInfo) -> bool:
    """Tiny data-parallel fit over the fused xGMI exchange (the default lagged
    schedule): no peer timeout, and bitwise-identical weights on every rank."""
    from ..engine import DateData, FitConfig, HipBackend, TrainConfig
    from ..models.hedge_mlp import NetSpec, init_weights

    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    mb = make_mailbox(info, spec.red_width, tag="rph_probe")
    try:
        n = 1 << 12
        g = torch.Generator().manual_seed(100 + info.rank)          # different data per rank
        x = (torch.rand(n, generator=g) * 0.6 + 0.7).to(info.device)
        be = HipBackend(spec, n, TrainConfig(batch_size=n * info.world, chunk_log2=6), device=info.device,
                        world=info.world, rank=info.rank, mailbox=mb)
        data = DateData(feats=[x], prices_next=[x * 1.01], bond_next=1.0, target=torch.relu(x - 1.0),
                        prices_now=[x])
        w, o, f = be.new_weights(init_weights(spec, [0.5, 0.0])), be.new_opt(), be.new_fit()
        be.fit(w, o, f, data, FitConfig(epochs=4, patience=10 ** 6, early_stopping=False), seed=5)
        torch.cuda.synchronize(info.device)
        if int(mb.error[0].item()) != 0:
            return False
        wv = w[: spec.nparams].double()
        mx, mn = wv.clone(), wv.clone()
        all_reduce_(mx, "max")
        all_reduce_(mn, "min")
        return bool(torch.equal(mx, mn)) and bool(torch.isfinite(wv).all())
    except Exception:
        return False
    finally:
        mb.close()


def select_transport(info: DistInfo) -> str:
    """Probe-then-choose, like a collective library's transport selection: keep
    the in-kernel xGMI exchange when a tiny DP fit over it is clean on every
    rank, otherwise fall back to an RCCL all-reduce of the packet (+ update
    kernel).  Runs once, outside any timed region; all ranks agree."""
    if info.world <= 1 or info.device.type != "cuda" or info.dp_mode != "xgmi":
        return info.dp_mode
    ok = torch.tensor([1.0 if _probe_xgmi(info) else 0.0], dtype=torch.float64, device=info.device)
    all_reduce_(ok, "min")
    if float(ok.item()) < 1.0:
        from ..ops.native import NcclComm

        info.dp_mode = "rccl"
        info.comm = NcclComm(info.rank, info.world, _store(), tag="rph_fallback")
    return info.dp_mode


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

    if _INFO is not None and _INFO.comm is not None:
        try:
            _INFO.comm.close()
        except Exception:
            pass
    if _INFO is not None and _INFO.initialized_here and dist.is_initialized():
        dist.destroy_process_group()
    _INFO = None
