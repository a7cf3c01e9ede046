"""NetObs's Observable / Estimator interface and a minimal evaluation loop.

The estimators mirror deephall/netobs_bridge/observables/*.py method for method:
``empty_val_state(steps) -> (values, state)``, ``evaluate(i, params, key, data, system,
state, aux_data) -> (values_i, state)``, ``digest(all_values, state) -> results``.
``evaluate`` below is a stand-in for NetObs's driver (absent here, so its exact
bookkeeping is unpinned): walker means of each step's values are stored at index i of the
arrays ``empty_val_state`` allocated.
"""

from __future__ import annotations

import logging
from typing import Any

import torch

from ..random import Key

logger = logging.getLogger("deephall_amd")
_MASK = 0xFFFFFFFFFFFFFFFF


class Observable:
    def __init__(self, system, options: dict | None = None):
        self.options = dict(options or {})
        self.shape = tuple(self.shapeof(system))

    def shapeof(self, system) -> tuple[int, ...]:
        return ()


class Estimator:
    observable_type = Observable

    def __init__(self, adaptor, system, estimator_options: dict | None, observable_options: dict | None):
        self.adaptor = adaptor
        self.system = system
        self.options = dict(estimator_options or {})
        self.observable = self.observable_type(system, observable_options)

    def empty_val_state(self, steps: int) -> tuple[dict[str, torch.Tensor], dict[str, Any]]:
        raise NotImplementedError

    def evaluate(self, i, params, key, data, system, state, aux_data):
        raise NotImplementedError

    def digest(self, all_values, state) -> dict[str, torch.Tensor]:
        return {}


def _batch_mean(v: torch.Tensor) -> torch.Tensor:
    v = torch.as_tensor(v)
    if v.ndim == 0:
        return v
    if v.is_complex():
        ok = ~(torch.isnan(v.real) | torch.isnan(v.imag))
        ok = ok.reshape(ok.shape[0], -1).all(dim=-1)
        return v[ok].mean(dim=0)
    return torch.nanmean(v, dim=0)


def evaluate(adaptor, estimator_cls, ckpt_file, steps: int, *, burn_in: int = 100, walk_steps: int = 10,
             seed: int = 0, estimator_options: dict | None = None, observable_options: dict | None = None,
             device=None):
    """Restore a checkpoint, burn in, then ``steps`` x (walk, evaluate); returns the digest and state."""
    params, data, system, aux = adaptor.restore(ckpt_file, device=device)
    est = estimator_cls(adaptor, system, estimator_options, observable_options)
    walk = adaptor.make_walking_step(None, walk_steps, system)
    key = Key(int(seed) & _MASK)  # walk key: every Metropolis step consumes one counter value
    for _ in range(burn_in):
        data, aux = walk(key, params, data, aux)
        key = key.advance(walk_steps)
    values, state = est.empty_val_state(steps)
    for i in range(steps):
        data, aux = walk(key, params, data, aux)
        key = key.advance(walk_steps)
        ekey = Key((int(seed) * 0x9E3779B97F4A7C15 + i + 1) & _MASK)  # estimator draws (one_rdm's r')
        vals, state = est.evaluate(i, params, ekey, data, system, state, aux)
        for name, v in vals.items():
            values[name][i] = _batch_mean(v).to(values[name].dtype)
    out = dict(est.digest(values, state))
    out.update({k: v for k, v in state.items() if k not in out})
    return out, values
