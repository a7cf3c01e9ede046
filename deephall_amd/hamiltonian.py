"""Local energy on MI355X — mirror of deephall/hamiltonian.py.

``local_energy(f, system)`` (hamiltonian.py:175-212) returns a batched
``_e_l(params, data[B,N,2]) -> (E_L complex64 [B], OtherObservables)``.  The
reference differentiates ``f`` with ``jax.grad`` and two full ``jax.hessian``
calls (hamiltonian.py:105-113); here the kernels propagate 2N+5 forward-mode
channels through the network and assemble KE, Lz, Lz^2, L^2 and
the potential in one native call (dh_local_energy).  Any other callable ``f`` (the
reference's tests pass analytic Slater determinants) goes through generic.py:
torch.func derivatives of the caller's function, HIP assembly of KE / L^2.
"""

from __future__ import annotations

import math

import torch

from . import _lib
from .config import InteractionType, System
from .mcmc import native_network
from .networks.psiformer import NetworkSpec, Psiformer, _ptr, _stream, get_handle

DEFAULT_WORKSPACE_BYTES = 24 << 30


def _run_local_energy(net: Psiformer, params, data: torch.Tensor, ws_budget: int = DEFAULT_WORKSPACE_BYTES):
    h = net.prepare(params, data.device)
    x = net._check_walkers(data)
    B = x.shape[0]
    e_l = torch.empty(B, 2, dtype=torch.float32, device=x.device)
    obs = torch.empty(B, 8, dtype=torch.float32, device=x.device)
    need = h.lib.dh_workspace_bytes(h.h, B, 1)
    one = h.lib.dh_workspace_bytes(h.h, 1, 1)
    nbytes = max(min(need, ws_budget), one)
    ws = h.workspace(nbytes)
    _lib.check(h.lib.dh_local_energy(h.h, _ptr(x), B, _ptr(e_l), _ptr(obs), _ptr(ws), ws.numel(), _stream(x.device)))
    return e_l, obs


def _observables(e_l, obs):
    kinetic = torch.complex(obs[:, 0], obs[:, 1])
    out = {
        "angular_momentum_z": obs[:, 3],
        "angular_momentum_z_square": obs[:, 4],
        "angular_momentum_square": obs[:, 5],
        "potential": obs[:, 2],
        "kinetic": kinetic,
    }
    return torch.complex(e_l[:, 0], e_l[:, 1]), out


def local_energy(f, system: System):
    net = native_network(f)
    if net is None:
        from . import generic

        return generic.local_energy(f, system)
    _check_system(net, system)

    def _e_l(params, data: torch.Tensor):
        e_l, obs = _run_local_energy(net, params, data)
        return _observables(e_l, obs)

    _e_l.network = net
    _e_l.raw = lambda params, data: _run_local_energy(net, params, data)  # (e_l [B,2], obs [B,8]) f32
    return _e_l


make_local_energy = local_energy


def make_local_kinetic_energy(f, Q: float, r):
    """hamiltonian.py:83-172: returns ``ke(params, data) -> (KE complex [B], AngularMomenta)``."""
    net = native_network(f)
    if net is None:
        from . import generic

        return generic.make_local_kinetic_energy(f, Q, r)
    if abs(2 * Q - net.spec.flux) > 1e-6:
        raise ValueError(f"Q={Q} does not match the network's flux {net.spec.flux}")
    r = float(r)
    spec = net.spec
    if spec.radius is None and abs(r - math.sqrt(Q)) < 1e-7 * max(1.0, r):
        knet = net
    else:
        knet = net.with_system(radius=r, interaction_strength=0.0)

    def ke(params, data):
        e_l, obs = _run_local_energy(knet, params, data)
        _, o = _observables(e_l, obs)
        return o["kinetic"], {
            k: o[k] for k in ("angular_momentum_z", "angular_momentum_z_square", "angular_momentum_square")
        }

    return ke


def make_potential(interaction_type, Q: float, r):
    """hamiltonian.py:63-80: returns ``potential(data[B,N,2]) -> PE [B]`` (not times the strength)."""
    itype = str(getattr(interaction_type, "value", interaction_type))

    def potential(data: torch.Tensor):
        N = data.shape[1]
        spec = NetworkSpec(
            nspins=(N, 0), flux=int(round(2 * Q)), ndets=1, num_heads=1, heads_dim=4, num_layers=0,
            radius=float(r), interaction_type=itype,
        )
        h = get_handle(spec, data.device)
        x = data.to(torch.float32).contiguous()
        pe = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
        _lib.check(h.lib.dh_potential(h.h, _ptr(x), x.shape[0], _ptr(pe), _stream(x.device)))
        return pe

    return potential


def _check_system(net: Psiformer, system: System):
    s = net.spec
    if tuple(system.nspins) != s.nspins or int(system.flux) != s.flux:
        raise ValueError("system does not match the network it was built with")
    want = (
        system.radius,
        float(system.interaction_strength),
        str(getattr(system.interaction_type, "value", system.interaction_type)),
    )
    have = (s.radius, s.interaction_strength, s.interaction_type)
    if want != have:
        raise ValueError(f"system {want} differs from the network's {have}; build the network with make_network(system, ...)")


__all__ = ["local_energy", "make_local_energy", "make_local_kinetic_energy", "make_potential", "InteractionType"]
