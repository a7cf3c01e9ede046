"""make_network (deephall/networks/__init__.py:22-37)."""

from __future__ import annotations

from ..config import Network, NetworkType, System
from .laughlin import Laughlin, LaughlinQuasiparticle
from .psiformer import Psiformer


def make_network(system: System, network: Network) -> Psiformer:
    Q = system.flux / 2
    ntype = str(getattr(network.type, "value", network.type))
    if ntype == NetworkType.laughlin.value:  # networks/__init__.py:24-27 (ground state, quasihole and
        # quasiparticle fillings all run on laughlin.hip)
        return Laughlin(flux=system.flux, nspins=system.nspins, excitation_lz=system.lz_center, system=system)
    if ntype == NetworkType.psiformer.value:
        return Psiformer(
            Q=Q,
            nspins=system.nspins,
            ndets=network.psiformer.determinants,
            num_heads=network.psiformer.num_heads,
            num_layers=network.psiformer.num_layers,
            heads_dim=network.psiformer.heads_dim,
            orbital_type=network.orbital,
            system=system,
        )
    raise ValueError(f"unknown network type {network.type}")


__all__ = ["make_network", "Psiformer", "Laughlin", "LaughlinQuasiparticle"]
