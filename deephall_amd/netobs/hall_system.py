"""hall_system.py:17-19: NetObs's electron-gas system description plus the flux."""

from __future__ import annotations


class HallSystem(dict):
    """``{"spins": [n_up, n_dn], "ndim": 2, "flux": 2Q}`` (a TypedDict in the reference)."""

    def __init__(self, spins, ndim: int = 2, flux: int = 0):
        super().__init__(spins=list(spins), ndim=int(ndim), flux=int(flux))
