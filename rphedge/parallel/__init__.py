"""Data parallelism over Monte-Carlo paths (RCCL over xGMI)."""
from .dist import DistInfo, all_reduce_, barrier, init, shard, shutdown  # noqa: F401
