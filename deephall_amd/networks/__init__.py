"""make_network (deephall/networks/__init__.py:22-37)."""

from __future__ import annotations

from ..config import Network, NetworkType, System
from .psiformer import Psiformer


def make_network(system: System, network: Network) -> Psiformer:
    Q = system.flux / 2
    ntype = str(getattr(network.type, "value", network.type))
    if ntype == NetworkType.laughlin.value:
        raise NotImplementedError("the Laughlin network (networks/laughlin.py) is outside the MI355X hot path")
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


__all__ = ["make_network", "Psiformer"]
