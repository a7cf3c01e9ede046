"""Collectives — the MI355X counterpart of deephall/constants.py:29-41.

The reference runs one process over all local devices with ``jax.pmap`` and
averages with ``lax.pmean`` over axis ``qmc_pmap_axis``.  Here each GPU is its own
process (torch.distributed, backend "nccl" = RCCL over xGMI on ROCm, "gloo" on
CPU for tests) and ``pmean`` is an all-reduce SUM divided by the world size.
The hot path issues exactly one packed ``pmean`` per VMC iteration
(see loss.py / train.py).
"""

from __future__ import annotations

import torch
import torch.distributed as dist

PMAP_AXIS_NAME = "qmc_pmap_axis"


def world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def pmean(x: torch.Tensor) -> torch.Tensor:
    """Mean over all ranks (lax.pmean).  Single process: identity."""
    n = world_size()
    if n == 1:
        return x
    y = x.clone()
    dist.all_reduce(y, op=dist.ReduceOp.SUM)
    return y / n


def pmean_(x: torch.Tensor) -> torch.Tensor:
    """In-place mean over ranks (one all-reduce; identity on one process)."""
    n = world_size()
    if n > 1:
        dist.all_reduce(x, op=dist.ReduceOp.SUM)
        x.div_(n)
    return x


def pmap(func, *args, **kwargs):
    """The per-device function already runs on this rank's shard: identity wrapper."""
    return func
