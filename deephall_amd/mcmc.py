"""Metropolis-Hastings walker update on MI355X — mirror of deephall/mcmc.py.

``make_mcmc_step(batch_network, batch_per_device, steps)`` (mcmc.py:105-150)
returns ``mcmc_step(params, data, key, width) -> (data, pmove)``.  The whole
call — the initial log-probability (mcmc.py:142), ``steps`` all-electron
proposals (sph_sampling, mcmc.py:67-102), network evaluations and accept/select
(mh_update, mcmc.py:25-64) — runs in the HIP library (dh_mcmc_step); ``data``
is updated in place (the reference donates it, train.py:75).  ``pmove`` is the
acceptance ratio averaged over ranks (mcmc.py:146-147).

``update_mcmc_width`` (mcmc.py:153-186) is host logic and is kept verbatim in
behaviour.
"""

from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib, constants
from .networks.psiformer import Psiformer, _ptr, _stream
from .random import Key


def native_network(f) -> Psiformer | None:
    """The network of this library behind ``f`` (itself, its bound .apply, or a function
    carrying ``.network``), or None for any other callable."""
    if isinstance(f, Psiformer):
        return f
    owner = getattr(f, "__self__", None)
    if isinstance(owner, Psiformer):
        return owner
    net = getattr(f, "network", None)
    if isinstance(net, Psiformer):
        return net
    return None


def resolve_network(f) -> Psiformer:
    """The network itself, for the paths that need its parameters (loss, training)."""
    net = native_network(f)
    if net is None:
        raise TypeError("this path needs a deephall_amd network (Psiformer / Laughlin or its bound .apply)")
    return net


def make_mcmc_step(batch_network, batch_per_device: int, steps: int = 10):
    """Native networks run the whole call in dh_mcmc_step; any other batched callable
    ``batch_network(params, data[B, N, 2]) -> complex[B]`` goes through generic.py (its log
    psi evaluated by the caller's code, proposal and accept in HIP on the same streams)."""
    net = native_network(batch_network)
    if net is None:
        if not callable(batch_network):
            raise TypeError("batch_network must be callable")
        from . import generic

        return generic.make_mcmc_step(batch_network, batch_per_device, steps)

    def mcmc_step(params, data: torch.Tensor, key: Key, width, *, noise=None, walker_offset=None, reduce=True):
        """Run ``steps`` MH moves in place.  Returns (data, pmove) with pmove a 0-d tensor.

        noise: optional injected randoms [steps, B, 2N+1] (normals, phi uniforms, accept uniform).
        walker_offset: global index of walker 0 (defaults to rank * batch_per_device).
        reduce: pmean the acceptance over ranks (reference behaviour); the VMC driver
                passes False and folds pmove into its single packed all-reduce.
        """
        h = net.prepare(params, data.device)
        if data.dtype != torch.float32 or not data.is_contiguous():
            raise ValueError("walkers must be contiguous float32 [B, N, 2] (updated in place)")
        B = data.shape[0]
        if B != batch_per_device:
            raise ValueError(f"expected {batch_per_device} walkers per device, got {B}")
        N = net.spec.nelec
        if noise is not None:
            noise = noise.to(device=data.device, dtype=torch.float32).contiguous()
            if tuple(noise.shape) != (steps, B, 2 * N + 1):
                raise ValueError(f"noise must be [{steps}, {B}, {2 * N + 1}]")
        woff = constants.rank() * batch_per_device if walker_offset is None else int(walker_offset)
        lp = torch.empty(B, dtype=torch.float32, device=data.device)
        nacc = torch.empty(B, dtype=torch.int32, device=data.device)
        nbytes = h.lib.dh_workspace_bytes(h.h, B, 0)
        ws = h.workspace(nbytes)
        _lib.check(
            h.lib.dh_mcmc_step(
                h.h,
                _ptr(data),
                _ptr(lp),
                _ptr(nacc),
                B,
                int(steps),
                C.c_float(float(width)),
                C.c_uint64(int(key.seed)),
                C.c_uint64(int(key.counter)),
                C.c_int64(woff),
                _ptr(noise),
                _ptr(ws),
                ws.numel(),
                _stream(data.device),
            )
        )
        mcmc_step.last_lp = lp
        mcmc_step.last_n_accept = nacc
        pmove = nacc.sum(dtype=torch.float32) / float(max(steps, 1) * batch_per_device)
        if reduce:
            pmove = constants.pmean(pmove)
        return data, pmove

    mcmc_step.steps = steps
    return mcmc_step


def update_mcmc_width(t, width, adapt_frequency, pmove, pmoves, pmove_max=0.55, pmove_min=0.5):
    """mcmc.py:153-186."""
    t_since = t % adapt_frequency
    pmoves[t_since] = float(pmove.item() if isinstance(pmove, torch.Tensor) else pmove)
    if t > 0 and t_since == 0:
        if np.mean(pmoves) > pmove_max:
            width *= 1.1
        elif np.mean(pmoves) < pmove_min:
            width /= 1.1
    return width, pmoves
