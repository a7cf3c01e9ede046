"""DeepHallAdaptor (netobs_bridge/adaptor.py:36-115) on the native path.

``restore`` reads ``config.yml`` beside the checkpoint (our LogManager's format: a
``git_commit`` line, then the Config), builds the network, and restores parameters,
this rank's walkers and the MCMC width (log.py restore_checkpoint).  The walking step is
``dh_mcmc_step``; the energies are ``dh_local_energy`` (kinetic) and ``dh_potential``.
"""

from __future__ import annotations

import math
from pathlib import Path
from typing import Any, TypedDict

import torch

from ..config import Config
from ..hamiltonian import make_local_kinetic_energy, make_potential
from ..log import LogManager
from ..mcmc import make_mcmc_step
from ..networks import make_network
from .hall_system import HallSystem


class DeepHallAuxData(TypedDict):
    mcmc_width: float


class DeepHallAdaptor:
    def __init__(self, config: Any = None, args: list[str] | None = None) -> None:
        self.config, self.args = config, list(args or [])
        self.cfg = None
        self.model = None

    def restore(self, ckpt_file: str | None = None, device=None):
        """adaptor.py:43-66: (params, walkers, HallSystem, {"mcmc_width": w})."""
        if ckpt_file is None:
            raise ValueError("Must specify a checkpoint")
        import yaml

        ckpt_path = Path(ckpt_file)
        raw = yaml.safe_load((ckpt_path.parent / "config.yml").read_text())
        raw.pop("git_commit", None)
        self.cfg = cfg = Config.from_dict(raw)
        self.model = model = make_network(cfg.system, cfg.network)
        device = torch.device(device or "cuda")
        self.batch_per_device = None
        Q = cfg.system.flux / 2
        radius = float(cfg.system.radius or math.sqrt(Q))
        self.kinetic_energy = make_local_kinetic_energy(model, Q, radius)
        self.potential_energy = make_potential(cfg.system.interaction_type, Q, radius)
        _, state = LogManager.restore_checkpoint(ckpt_path, model, device)
        self.batch_per_device = state.data.shape[0]
        system = HallSystem(spins=list(cfg.system.nspins), ndim=2, flux=cfg.system.flux)
        return state.params, state.data, system, DeepHallAuxData(mcmc_width=float(state.mcmc_width))

    def call_network(self, params, electrons: torch.Tensor, system=None) -> torch.Tensor:
        """Batched complex log psi [B] of walkers [B, N, 2] (the reference vmaps one walker)."""
        return self.model.apply(params, electrons)

    def call_signed_network(self, params, electrons: torch.Tensor, system=None):
        """adaptor.py:68-72: (sign 1, log psi) — the phase lives in the complex log."""
        return torch.ones((), device=electrons.device), self.call_network(params, electrons, system)

    def make_walking_step(self, batch_log_psi, steps: int, system=None):
        """adaptor.py:74-93: walk(key, params, electrons, aux) -> (electrons, aux)."""
        if batch_log_psi is not None and getattr(batch_log_psi, "__self__", None) is not self.model:
            raise TypeError("the MI355X walk runs the native network of this adaptor (pass None)")
        mcmc_step = make_mcmc_step(self.model, batch_per_device=self.batch_per_device, steps=steps)

        def walk(key, params, electrons, aux_data):
            new_data, _ = mcmc_step(params, electrons, key, aux_data["mcmc_width"])
            return new_data, aux_data

        return walk

    def call_local_kinetic_energy(self, params, key, electrons, system=None):
        del key, system
        return self.kinetic_energy(params, electrons)[0]

    def call_local_potential_energy(self, params, key, electrons, system=None):
        del params, key, system
        return self.potential_energy(electrons) * self.cfg.system.interaction_strength


DEFAULT = DeepHallAdaptor
