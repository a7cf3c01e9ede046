"""Arbitrary log-psi callables — the reference's callable boundary.

The reference's ``make_local_kinetic_energy(f, Q, r)`` (hamiltonian.py:83-172) and
``make_mcmc_step(batch_network, ...)`` (mcmc.py:105-150) accept ANY log psi: its
tests pass analytic Slater determinants (tests/hamiltonian_test.py:29-76), NetObs
passes the network (netobs_bridge/adaptor.py:56,77).  A callable that is not a
network of this library is the caller's own code, so it is evaluated — and, for the
kinetic energy, differentiated with ``torch.func.grad`` / ``hessian``, the
counterpart of the reference's ``jax.grad`` / ``jax.hessian`` at hamiltonian.py:105-113
— wherever its tensors live.  Everything the framework computes runs in HIP:

* the proposal and the Metropolis accept, on the same Philox streams as
  ``dh_mcmc_step`` (``dh_mh_propose`` / ``dh_mh_accept``), so a callable that returns
  a native network's log psi walks exactly as the native MCMC does;
* the kinetic energy, Lz, Lz^2 and L^2 from the derivatives
  (``dh_kinetic_from_derivatives``, kinetic.hip, double precision);
* the potential (``dh_potential``).

Conventions follow the reference: ``f(params, x[N, 2]) -> complex`` is per walker
(the returned functions take batched ``data[B, N, 2]`` and vmap it), while
``batch_network(params, data[B, N, 2]) -> complex[B]`` is batched.  Tensors must be on
the GPU: there is no CPU path.
"""

from __future__ import annotations

import torch
from torch.func import grad, hessian, vmap

from . import _lib, constants
from .networks.psiformer import _ptr, _stream


def _cuda(data: torch.Tensor, what: str):
    if not isinstance(data, torch.Tensor) or data.device.type != "cuda":
        raise RuntimeError(f"{what}: deephall_amd runs on the GPU only (no CPU fallback): pass CUDA/HIP tensors")
    if data.dim() != 3 or data.shape[-1] != 2:
        raise ValueError(f"{what}: walkers must be [B, N, 2], got {tuple(data.shape)}")


def derivatives(f, params, data: torch.Tensor, chunk_size: int | None = None):
    """First derivatives g[B, N, 2] and Hessian H[B, N, 2, N, 2] (complex) of a per-walker
    ``f(params, x[N, 2])``, real and imaginary parts separately as hamiltonian.py:105-113."""

    def fr(p, x):
        return f(p, x).real

    def fi(p, x):
        return f(p, x).imag

    def dv(fn):
        return vmap(fn, in_dims=(None, 0), chunk_size=chunk_size)(params, data)

    g = torch.complex(dv(grad(fr, argnums=1)), dv(grad(fi, argnums=1)))
    H = torch.complex(dv(hessian(fr, argnums=1)), dv(hessian(fi, argnums=1)))
    return g, H


def kinetic_from_derivatives(data: torch.Tensor, g: torch.Tensor, H: torch.Tensor, Q: float, r: float):
    """KE complex64 [B] and AngularMomenta from x, g and H (dh_kinetic_from_derivatives)."""
    _cuda(data, "kinetic_from_derivatives")
    B, N, _ = data.shape
    if tuple(g.shape) != (B, N, 2) or tuple(H.shape) != (B, N, 2, N, 2):
        raise ValueError(f"derivatives of shape {tuple(g.shape)} / {tuple(H.shape)} do not match walkers {(B, N)}")
    x = data.to(torch.float64).contiguous()
    gr = torch.view_as_real(g.to(torch.complex128)).contiguous()
    Hr = torch.view_as_real(H.to(torch.complex128)).contiguous()
    ke = torch.empty(B, 2, dtype=torch.float32, device=data.device)
    mom = torch.empty(B, 3, dtype=torch.float32, device=data.device)
    lib = _lib.load()
    _lib.check(
        lib.dh_kinetic_from_derivatives(
            _ptr(x), _ptr(gr), _ptr(Hr), B, N, float(Q), float(r), _ptr(ke), _ptr(mom), _stream(data.device)
        )
    )
    return torch.complex(ke[:, 0], ke[:, 1]), {
        "angular_momentum_z": mom[:, 0],
        "angular_momentum_z_square": mom[:, 1],
        "angular_momentum_square": mom[:, 2],
    }


def make_local_kinetic_energy(f, Q: float, r, chunk_size: int | None = None):
    """hamiltonian.py:83-172 for any per-walker ``f``: ``ke(params, data[B, N, 2])``."""
    r = float(r)

    def ke(params, data: torch.Tensor):
        _cuda(data, "make_local_kinetic_energy")
        g, H = derivatives(f, params, data, chunk_size)
        return kinetic_from_derivatives(data, g, H, Q, r)

    return ke


def local_energy(f, system, chunk_size: int | None = None):
    """hamiltonian.py:175-212 for any per-walker ``f``: ``_e_l(params, data[B, N, 2])``."""
    from .hamiltonian import make_potential

    Q = system.flux / 2
    r = float(system.radius) if system.radius is not None else Q**0.5
    ke = make_local_kinetic_energy(f, Q, r, chunk_size)
    pe = make_potential(system.interaction_type, Q, r)
    strength = float(system.interaction_strength)

    def _e_l(params, data: torch.Tensor):
        potential = pe(data) * strength
        kinetic, moms = ke(params, data)
        return kinetic + potential, dict(moms, potential=potential, kinetic=kinetic)

    return _e_l


def _logpsi_pairs(v: torch.Tensor, B: int) -> torch.Tensor:
    """log psi [B] (complex, or real = log|psi|) -> float32 [B, 2] (re, im)."""
    if v.shape != (B,):
        raise ValueError(f"batch_network must return log psi of shape [{B}], got {tuple(v.shape)}")
    if v.is_complex():
        return torch.view_as_real(v.to(torch.complex64)).contiguous()
    return torch.stack([v.to(torch.float32), torch.zeros_like(v, dtype=torch.float32)], -1)


def make_mcmc_step(batch_network, batch_per_device: int, steps: int = 10):
    """mcmc.py:105-150 for any batched ``batch_network``; same signature and walker update
    as the native ``mcmc.make_mcmc_step`` (``data`` updated in place)."""

    def mcmc_step(params, data: torch.Tensor, key, width, *, noise=None, walker_offset=None, reduce=True):
        _cuda(data, "mcmc_step")
        if data.dtype != torch.float32 or not data.is_contiguous():
            raise ValueError("walkers must be contiguous float32 [B, N, 2] (updated in place)")
        B, N, _ = data.shape
        if B != batch_per_device:
            raise ValueError(f"expected {batch_per_device} walkers per device, got {B}")
        if noise is not None:
            noise = noise.to(device=data.device, dtype=torch.float32).contiguous()
            if tuple(noise.shape) != (steps, B, 2 * N + 1):
                raise ValueError(f"noise must be [{steps}, {B}, {2 * N + 1}]")
        woff = constants.rank() * batch_per_device if walker_offset is None else int(walker_offset)
        lib, s = _lib.load(), _stream(data.device)
        lp = torch.empty(B, dtype=torch.float32, device=data.device)
        nacc = torch.empty(B, dtype=torch.int32, device=data.device)
        _lib.check(lib.dh_mh_init(_ptr(_logpsi_pairs(batch_network(params, data), B)), _ptr(lp), _ptr(nacc), B, s))
        x2 = torch.empty_like(data)
        seed = int(key.seed)
        for st in range(int(steps)):
            step = int(key.counter) + st
            nz = noise[st] if noise is not None else None
            _lib.check(lib.dh_mh_propose(_ptr(data), _ptr(x2), B, N, float(width), seed, step, woff, _ptr(nz), s))
            lp2 = _logpsi_pairs(batch_network(params, x2), B)
            _lib.check(
                lib.dh_mh_accept(_ptr(data), _ptr(x2), _ptr(lp), _ptr(lp2), _ptr(nacc), B, N, seed, step, woff,
                                 _ptr(nz), s)
            )
        mcmc_step.last_lp = lp
        mcmc_step.last_n_accept = nacc
        pmove = nacc.sum(dtype=torch.float32) / float(max(steps, 1) * batch_per_device)
        if reduce:
            pmove = constants.pmean(pmove)
        return data, pmove

    mcmc_step.steps = steps
    return mcmc_step


__all__ = ["derivatives", "kinetic_from_derivatives", "make_local_kinetic_energy", "local_energy", "make_mcmc_step"]
