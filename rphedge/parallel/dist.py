"""Data parallelism over Monte-Carlo paths.

One process per GPU.  The global path set ``[0, 2^m)`` is split into
contiguous shards ``[r*n/W, (r+1)*n/W)``; Sobol points are index-addressable so
every rank generates its own shard with no communication.  Per optimizer step
the 512-byte gradient packet (grads + loss/metric partials) is summed with ONE
RCCL all-reduce issued by the native runtime on the compute stream (captured
into the same hipGraph as the step kernels); statistics and histograms use
``torch.distributed`` collectives (nccl = RCCL on ROCm, gloo on CPU).

Sizing for xGMI: the per-step packet is latency-bound (one-shot/LL protocol),
so the design lever is FEWER steps (large per-rank batches) rather than
bandwidth; bucketing is moot at 512 B.
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
    if world > 1:
        be = backend or os.environ.get("RPH_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
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

    return IpcMailbox(info.rank, info.world, R, _store(), info.device, tag=tag)


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
