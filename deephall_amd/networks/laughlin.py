"""Laughlin wavefunction on MI355X — mirror of deephall/networks/laughlin.py:19-100.

``Laughlin(nspins, flux, cf_flux=1, excitation_lz=0)`` (the reference module's fields;
networks/__init__.py:25-27 passes ``System.lz_center`` as ``excitation_lz``): the
ground state (N = 2 Q1 + 1), the quasihole state (N = 2 Q1) and the quasiparticle state
(N = 2 Q1 + 2, laughlin.py:82-100), Q1 = flux/2 - p (N - 1).
It has no parameters: ``init`` returns an empty tree.  ``apply`` is batched log psi
(dh_logpsi); the MCMC step and the local energy run the HIP kernels of laughlin.hip
through the same entry points as the Psiformer (make_mcmc_step, local_energy,
make_local_kinetic_energy), with the full analytic Hessian in double precision.  The
quasiparticle's LLL-projected excited orbital depends on every electron through the
Jastrow derivatives; laughlin.hip carries that column's dense derivatives through the
determinant algebra (see the kernel's header).
`LaughlinQuasiparticle` is the same state as a plain log-psi callable (the reference's own
slogdet form, evaluated through the library's callable boundary, deephall_amd.generic:
torch.func derivatives): a second, independent route the tests compare the kernel with.
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


def laughlin_q1(nspins, flux, cf_flux: int = 1) -> float:
    """Composite-fermion monopole strength Q1 = flux/2 - p (N - 1) (laughlin.py:34)."""
    return float(flux) / 2 - int(cf_flux) * (sum(nspins) - 1)


class LaughlinQuasiparticle:
    """laughlin.py:19-100 for N = 2 Q1 + 2: log psi of walkers x [N, 2] (per walker, the
    reference's f convention) or data [B, N, 2] (batched), complex128.  No parameters."""

    def __init__(self, nspins, flux, cf_flux: int = 1, excitation_lz: float = 0.0, system=None):
        self.nspins = tuple(int(n) for n in nspins)
        self.flux = int(flux)
        self.cf_flux = int(cf_flux)
        self.excitation_lz = float(excitation_lz)
        self.system = system
        N = sum(self.nspins)
        self.Q1 = laughlin_q1(self.nspins, self.flux, self.cf_flux)
        if N != 2 * self.Q1 + 2:
            raise ValueError(f"not a quasiparticle filling: N = {N}, Q1 = {self.Q1}")
        diff = self.excitation_lz - self.Q1  # laughlin.py:49-52
        if int(diff) != diff or not (-abs(self.Q1) - 1 <= self.excitation_lz <= abs(self.Q1) + 1):
            raise ValueError(f"impossible Lz = {self.excitation_lz} for the quasiparticle (Q1 = {self.Q1})")

    def init(self, key=None, data=None, device=None) -> dict:
        return {}

    def _logpsi(self, x: torch.Tensor) -> torch.Tensor:
        x = x.to(torch.float64)
        N, Q, m1 = x.shape[0], self.Q1, self.excitation_lz
        theta, phi = x[:, 0], x[:, 1]
        u = (torch.cos(theta / 2) * torch.exp(0.5j * phi))[:, None]  # laughlin.py:61-62
        v = (torch.sin(theta / 2) * torch.exp(-0.5j * phi))[:, None]
        k = torch.arange(0, int(round(2 * Q)) + 1, device=x.device, dtype=torch.float64)  # Q + m, m = -Q .. Q
        orbitals = u**k * v ** (2 * Q - k)
        eye = torch.eye(N, dtype=u.dtype, device=x.device)
        element = u * v[:, 0] - u[:, 0] * v + eye  # laughlin.py:91
        jastrow = torch.prod(element, dim=-1, keepdim=True)
        # LLL projection (u* -> d/du, v* -> d/dv), laughlin.py:93-95
        jastrow_dv = jastrow * (torch.sum(-u[:, 0] / element, dim=-1, keepdim=True) + u)
        jastrow_du = jastrow * (torch.sum(v[:, 0] / element, dim=-1, keepdim=True) - v)
        excited = (u ** (Q + m1) * v ** (Q - m1)) * ((Q + 1 + m1) * v * jastrow_dv - (Q + 1 - m1) * u * jastrow_du)
        orb = torch.cat([orbitals * jastrow, excited], dim=-1)
        sign, logdet = torch.linalg.slogdet(orb)  # one determinant: log-sum-exp reduces to this
        return logdet + torch.log(sign)

    def __call__(self, params, data: torch.Tensor) -> torch.Tensor:
        if data.dim() == 2:
            return self._logpsi(data)
        return torch.vmap(self._logpsi)(data)

    apply = __call__


__all__ = ["Laughlin", "LaughlinQuasiparticle", "laughlin_q1", "_lib", "_ptr", "_stream"]
