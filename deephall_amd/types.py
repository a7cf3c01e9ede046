"""Boundary types — deephall/types.py:22-82 with torch tensors in place of jax arrays."""

from __future__ import annotations

from typing import Any, NamedTuple, Protocol, TypedDict

import torch


class AngularMomenta(TypedDict):
    angular_momentum_z: torch.Tensor
    angular_momentum_z_square: torch.Tensor
    angular_momentum_square: torch.Tensor


class OtherObservables(AngularMomenta):
    kinetic: torch.Tensor
    potential: torch.Tensor


class LossStats(OtherObservables):
    energy: torch.Tensor
    variance: torch.Tensor


class CheckpointState(NamedTuple):
    params: Any
    data: torch.Tensor
    opt_state: Any
    mcmc_width: float


class LocalEnergy(Protocol):
    def __call__(self, params: Any, data: torch.Tensor) -> tuple[torch.Tensor, OtherObservables]:
        """Batched local energy: data [B, N, 2] -> (E_L complex [B], observables [B])."""


class LogPsiNetwork(Protocol):
    def __call__(self, params: Any, data: torch.Tensor) -> torch.Tensor:
        """Batched log psi: data [B, N, 2] -> complex [B]."""
