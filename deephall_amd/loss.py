"""Energy statistics of one VMC iteration — the stats part of deephall/loss.py:47-92.

``make_loss_fn(network, system)`` returns ``loss_and_grad(params, data)`` that
evaluates E_L on this rank's walkers (dh_local_energy), reduces them on the
device (dh_energy_stats: nanmean, IQR-clipped nanmean with LOCAL quantiles as in
loss.py:30-38, observable means) and averages over ranks with ONE packed
all-reduce (the reference issues one ``pmean`` per statistic, loss.py:68-91).
Returns (LossStats, None): the parameter-gradient half (loss.py:53-64, 93-108)
is the next row of the build plan, not this hot path.
"""

from __future__ import annotations

import enum

import torch

from . import _lib, constants
from .hamiltonian import _run_local_energy
from .mcmc import resolve_network
from .networks.psiformer import _ptr, _stream, get_handle

# packed all-reduce layout (first 12 entries of dh_energy_stats + count)
_PACK = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11]


class LossMode(enum.Enum):
    ENERGY_GRAD = enum.auto()
    ENERGY_DIFF = enum.auto()
    SR_F_VECTOR = enum.auto()


def device_stats(net, e_l, obs, n_accept=None, steps=1):
    """dh_energy_stats on this rank: float32 [16] device tensor (DH_STAT_* layout)."""
    h = get_handle(net.spec, e_l.device)
    out = torch.empty(_lib.DH_NSTATS, dtype=torch.float32, device=e_l.device)
    _lib.check(
        h.lib.dh_energy_stats(
            h.h, _ptr(e_l), _ptr(obs), _ptr(n_accept), e_l.shape[0], int(steps), _ptr(out), None, 0, _stream(e_l.device)
        )
    )
    return out


def reduce_stats(local: torch.Tensor) -> dict:
    """One all-reduce of the packed device-local stats -> LossStats dict (0-d tensors)."""
    g = constants.pmean(local[: len(_PACK)])
    energy = torch.complex(g[0], g[1])
    return {
        "energy": energy,
        "clipped_energy": torch.complex(g[2], g[3]),
        "variance": g[4] - g[0] * g[0],  # pmean(nanmean(Re E^2)) - Re(energy)^2 (loss.py:91)
        "kinetic": torch.complex(g[5], g[6]),
        "potential": g[7],
        "angular_momentum_z": g[8],
        "angular_momentum_z_square": g[9],
        "angular_momentum_square": g[10],
        "pmove": g[11],
    }


def make_loss_fn(network, system, mode: LossMode = LossMode.ENERGY_DIFF):
    if mode != LossMode.ENERGY_DIFF:
        raise NotImplementedError("parameter gradients (loss.py:53-64) are not on the MI355X hot path yet")
    net = resolve_network(network)

    def loss_and_grad(params, data, n_accept=None, steps=1):
        e_l, obs = _run_local_energy(net, params, data)
        local = device_stats(net, e_l, obs, n_accept, steps)
        stats = reduce_stats(local)
        loss_and_grad.last = (e_l, obs)
        return stats, None

    return loss_and_grad
