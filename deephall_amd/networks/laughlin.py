"""Laughlin wavefunction on MI355X — mirror of deephall/networks/laughlin.py:19-100.

``Laughlin(nspins, flux, cf_flux=1, excitation_lz=0)`` (the reference module's fields;
networks/__init__.py:25-27 passes ``System.lz_center`` as ``excitation_lz``): the
ground state (N = 2 Q1 + 1) and the quasihole state (N = 2 Q1), Q1 = flux/2 - p (N - 1).
It has no parameters: ``init`` returns an empty tree.  ``apply`` is batched log psi
(dh_logpsi); the MCMC step and the local energy run the HIP kernels of laughlin.hip
through the same entry points as the Psiformer (make_mcmc_step, local_energy,
make_local_kinetic_energy), with the full analytic Hessian in double precision.
The quasiparticle state (laughlin.py:82-100) is rejected with a clear error.
"""

from __future__ import annotations

import torch

from .. import _lib
from .psiformer import NetworkSpec, ParamTree, Psiformer, _ptr, _stream, get_handle


class Laughlin(Psiformer):
    """Parameter-free analytic wavefunction sharing the Psiformer's native plumbing."""

    def __init__(self, nspins, flux, cf_flux: int = 1, excitation_lz: float = 0.0, system=None):
        self.nspins = tuple(int(n) for n in nspins)
        self.flux = int(flux)
        self.cf_flux = int(cf_flux)
        self.excitation_lz = float(excitation_lz)
        self.Q = self.flux / 2
        radius = getattr(system, "radius", None) if system is not None else None
        lam = getattr(system, "interaction_strength", 1.0) if system is not None else 1.0
        itype = getattr(system, "interaction_type", "coulomb") if system is not None else "coulomb"
        self.spec = NetworkSpec(
            nspins=self.nspins, flux=self.flux, ndets=1, num_heads=1, heads_dim=4, num_layers=0,
            radius=radius, interaction_strength=float(lam), interaction_type=str(getattr(itype, "value", itype)),
            network_type="laughlin", excitation_lz=self.excitation_lz, cf_flux=self.cf_flux,
        )
        self._flat_cache = {}
        self._epoch = 0

    def init(self, key=None, data=None, device=None) -> ParamTree:
        if device is None:
            device = data.device if isinstance(data, torch.Tensor) else ("cuda" if torch.cuda.is_available() else "cpu")
        return ParamTree.zeros(self.spec, device)

    def prepare(self, params, device):
        return get_handle(self.spec, device)  # nothing to upload

    def vjp(self, *args, **kwargs):
        raise TypeError("the Laughlin wavefunction has no parameters to differentiate")


__all__ = ["Laughlin", "_lib", "_ptr", "_stream"]
