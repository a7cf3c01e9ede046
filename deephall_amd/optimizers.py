"""Optimizer steps — mirror of deephall/optimizers/ (__init__.py:25-35, adam.py:24-43,
none.py:22-35).

``make_optimizer_step(cfg, network) -> (init, step)`` with
``step(state, key) -> (state, stats)`` over a ``CheckpointState``.  The gradient is
the loss of ``make_loss_fn(..., ENERGY_GRAD)`` (reverse mode in the HIP library,
averaged over ranks by the second all-reduce of the iteration — the reference's Adam
path omits that average, SURVEY.md finding 9); the Adam update is one HIP kernel over
the flat parameter buffer (``dh_adam_update``, optax.adam semantics).  KFAC
(optimizers/kfac.py, kfac_jax) is not built on MI355X: asking for it raises.
"""

from __future__ import annotations

import torch

from . import _lib
from .config import Config, LearningRate, OptimizerName
from .loss import LossMode, make_loss_fn
from .networks.psiformer import ParamTree, _ptr, _stream
from .types import CheckpointState


def lr_schedule(lr: LearningRate, t: int) -> float:
    """rate * (1 / (1 + t / delay)) ** decay (config.py:125-137)."""
    return float(lr.rate * (1.0 / (1.0 + (t / lr.delay))) ** lr.decay)


class AdamState:
    """optax ScaleByAdamState (count, mu, nu) + the schedule's count, on the device."""

    def __init__(self, params: ParamTree):
        self.mu = torch.zeros_like(params.flat)
        self.nu = torch.zeros_like(params.flat)
        self.count = 0

    def state_dict(self):
        return {"mu": self.mu, "nu": self.nu, "count": self.count}

    def load_state_dict(self, d):
        self.mu.copy_(torch.as_tensor(d["mu"]))
        self.nu.copy_(torch.as_tensor(d["nu"]))
        self.count = int(d["count"])


def adam_update(params: ParamTree, grads: ParamTree, state: AdamState, lr: float, b1=0.9, b2=0.999, eps=1e-8):
    """One optax.adam step in place on ``params.flat`` (dh_adam_update)."""
    p = params.flat
    if not (p.is_cuda and grads.flat.shape == p.shape):
        raise ValueError("params and grads must be matching flat device buffers")
    _lib.check(
        _lib.load().dh_adam_update(_ptr(p), _ptr(grads.flat), _ptr(state.mu), _ptr(state.nu), p.numel(), float(lr),
                                   float(b1), float(b2), float(eps), int(state.count), _stream(p.device))
    )
    state.count += 1


def make_adam_training_step(cfg: Config, network):
    loss_grad_fn = make_loss_fn(network, cfg.system, LossMode.ENERGY_GRAD)
    net = loss_grad_fn.network

    def init(params, key=None, data=None):
        del key, data
        return AdamState(params)

    def step(state: CheckpointState, key=None):
        params, data, opt_state, width = state
        stats, grads = loss_grad_fn(params, data)
        adam_update(params, grads, opt_state, lr_schedule(cfg.optim.adam.lr, opt_state.count))
        net.invalidate()  # the kernel wrote the flat buffer behind torch's version counter
        return CheckpointState(params, data, opt_state, width), stats

    return init, step


def make_inference_step(cfg: Config, network):
    loss_fn = make_loss_fn(network, cfg.system, LossMode.ENERGY_DIFF)

    def init(params, key=None, data=None):
        return None

    def step(state: CheckpointState, key=None):
        stats, _ = loss_fn(state.params, state.data)
        return state, stats

    return init, step


def make_optimizer_step(cfg: Config, network):
    """optimizers/__init__.py:25-35."""
    name = cfg.optim.optimizer
    name = OptimizerName(getattr(name, "value", name)) if name is not None else OptimizerName.none
    if name == OptimizerName.adam:
        return make_adam_training_step(cfg, network)
    if name == OptimizerName.none:
        return make_inference_step(cfg, network)
    if name == OptimizerName.kfac:
        raise NotImplementedError(
            "KFAC (optimizers/kfac.py, kfac_jax) is not implemented on MI355X yet: use optim.optimizer=adam or none"
        )
    raise ValueError(f"Optimizer {name} is not implemented!")
