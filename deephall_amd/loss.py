"""Energy statistics of one VMC iteration — the stats part of deephall/loss.py:47-92.

``make_loss_fn(network, system)`` returns ``loss_and_grad(params, data)`` that
evaluates E_L on this rank's walkers (dh_local_energy), reduces them on the
device (dh_energy_stats: nanmean, IQR-clipped nanmean with LOCAL quantiles as in
loss.py:30-38, observable means) and averages over ranks with ONE packed
all-reduce (the reference issues one ``pmean`` per statistic, loss.py:68-91).
The parameter-gradient half (loss.py:53-64, 93-108) runs as reverse mode in the HIP
library (dh_loss_diff -> dh_grad_cotangent -> dh_logpsi_vjp) and a second all-reduce.
"""

from __future__ import annotations

import enum

import torch

from . import _lib, constants
from .hamiltonian import _run_local_energy
from .mcmc import native_network, resolve_network
from .networks.psiformer import ParamTree, _ptr, _stream, get_handle

# packed all-reduce: every DH_STAT_* entry (16 floats; the clipped Lz^2 / Lz / L^2 means
# are 0 unless the penalties are on)
_NPACK = _lib.DH_NSTATS


class LossMode(enum.Enum):
    ENERGY_GRAD = enum.auto()
    ENERGY_DIFF = enum.auto()
    SR_F_VECTOR = enum.auto()


def _handle(net, device):
    """The library handle of a native network, or NULL for a caller's log-psi callable."""
    spec = getattr(net, "spec", None) if net is not None else None
    return get_handle(spec, device).h if spec is not None else None


def device_stats(net, e_l, obs, n_accept=None, steps=1, penalties=False):
    """dh_energy_stats on this rank: float32 [16] device tensor (DH_STAT_* layout)."""
    out = torch.empty(_lib.DH_NSTATS, dtype=torch.float32, device=e_l.device)
    _lib.check(
        _lib.load().dh_energy_stats(
            _handle(net, e_l.device), _ptr(e_l), _ptr(obs), _ptr(n_accept), e_l.shape[0], int(steps),
            int(bool(penalties)), _ptr(out), _stream(e_l.device),
        )
    )
    return out


def reduce_stats(local: torch.Tensor, raw: bool = False, flags=None):
    """One all-reduce of the packed device-local stats -> LossStats dict (0-d tensors).
    ``raw=True`` also returns the reduced packed vector (device, DH_STAT_* layout).
    ``flags``: host floats appended to the packed vector and averaged with it (the driver's
    checkpoint / signal decisions, so every rank acts on the same value); returned as
    ``out["flags"]`` (device tensor, the mean over ranks)."""
    local = local[:_NPACK]
    if flags:
        local = torch.cat([local, torch.tensor([float(f) for f in flags], dtype=local.dtype).to(local.device)])
    g = constants.pmean(local)
    energy = torch.complex(g[0], g[1])
    out = {
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
    if flags:
        out["flags"] = g[_NPACK:]
    return (out, g) if raw else out


def loss_diff(net, e_l, obs, gstats, lz_penalty=0.0, lz_center=0.0, l2_penalty=0.0):
    """dh_loss_diff: diff = iqr_clip(E_L - <E_L>_clip + penalties) (loss.py:75-89) with the
    reduced clipped means ``gstats`` (device, DH_STAT_* layout).  Returns (diff [B,2] f32,
    nvalid [1] f32 = walkers with a non-NaN diff)."""
    B = e_l.shape[0]
    diff = torch.empty(B, 2, dtype=torch.float32, device=e_l.device)
    nvalid = torch.empty(1, dtype=torch.float32, device=e_l.device)
    _lib.check(
        _lib.load().dh_loss_diff(
            _handle(net, e_l.device), _ptr(e_l), _ptr(obs), B, _ptr(gstats), float(lz_penalty), float(lz_center), float(l2_penalty),
            _ptr(diff), _ptr(nvalid), _stream(e_l.device),
        )
    )
    return diff, nvalid


def grad_cotangent(diff, nvalid, part=0):
    """dh_grad_cotangent: per-walker weights of 2 nanmean(conj(d log psi) diff) (loss.py:59-64);
    part 0 = its real part (ENERGY_GRAD), part 1 = its imaginary part."""
    B = diff.shape[0]
    ct = torch.empty(B, 2, dtype=torch.float32, device=diff.device)
    _lib.check(_lib.load().dh_grad_cotangent(_ptr(diff), _ptr(nvalid), B, int(part), _ptr(ct), _stream(diff.device)))
    return ct


def _kfac_buffer(net, device):
    """[gradient (dh_ref_layout) | curvature statistics] float32, cached per network and
    device; returns (buffer, number of gradient floats)."""
    cache = net.__dict__.setdefault("_kfac_buffers", {})
    if device not in cache:
        nref = get_handle(net.spec, device).nref
        cache[device] = (torch.empty(nref + net.kfac_layout(device)["nstats"], dtype=torch.float32, device=device), nref)
    return cache[device]


def make_loss_fn(network, system, mode: LossMode = LossMode.ENERGY_GRAD, curvature: bool = False):
    """loss.py:47-110.  ``loss_and_grad(params, data) -> (LossStats, aux)`` where aux is
    diff [B] complex (ENERGY_DIFF), the real parameter gradient (ENERGY_GRAD, a ParamTree)
    or the complex one ({name: complex tensor}, SR_F_VECTOR).  Every statistic and the
    gradient are averaged over ranks: one packed all-reduce of the statistics, one of the
    gradient (the reference's Adam path skips the latter, SURVEY.md finding 9).

    ``curvature=True`` (ENERGY_GRAD, the KFAC optimizer): the same forward pass also yields
    the Fisher curvature statistics of the batch — the reference registers
    ``register_normal_predictive_distribution(Re log psi)`` inside this function (loss.py:98)
    for kfac_jax to trace — averaged over ranks in the SAME all-reduce as the gradient and
    left in ``loss_and_grad.curvature`` (float32 [nstats], dh_kfac_layout)."""
    pen = (float(system.lz_penalty), float(system.lz_center), float(system.l2_penalty))
    penalties = pen[0] != 0.0 or pen[2] != 0.0
    if native_network(network) is None:
        return _make_callable_loss_fn(network, system, mode, pen, penalties)
    net = resolve_network(network)

    def loss_and_grad(params, data, n_accept=None, steps=1, flags=None):
        """``n_accept`` [B] int (mcmc_step(..., reduce=False).last_n_accept) puts pmove into
        the packed statistics; ``flags`` rides in the same all-reduce (reduce_stats)."""
        e_l, obs = _run_local_energy(net, params, data)
        local = device_stats(net, e_l, obs, n_accept, steps, penalties=penalties)
        stats, g = reduce_stats(local, raw=True, flags=flags)
        loss_and_grad.last = (e_l, obs)
        diff, nvalid = loss_diff(net, e_l, obs, g, *pen)
        if mode == LossMode.ENERGY_DIFF:
            return stats, torch.complex(diff[:, 0], diff[:, 1])
        if curvature:
            if mode != LossMode.ENERGY_GRAD:
                raise ValueError("curvature statistics go with LossMode.ENERGY_GRAD")
            buf, nref = _kfac_buffer(net, data.device)
            grad = ParamTree.view_of(net.spec, buf[:nref])
            curv = buf[nref:]
            net.kfac_vjp(params, data, grad_cotangent(diff, nvalid, 0), grad, curv)
            constants.pmean_(buf)  # gradient and curvature statistics: one all-reduce
            loss_and_grad.curvature = curv
            return stats, grad
        grad = net.vjp(params, data, grad_cotangent(diff, nvalid, 0))
        constants.pmean_(grad.flat)
        if mode == LossMode.ENERGY_GRAD:
            return stats, grad
        gim = net.vjp(params, data, grad_cotangent(diff, nvalid, 1))
        constants.pmean_(gim.flat)
        return stats, {k: torch.complex(grad[k], gim[k]) for k in grad}

    loss_and_grad.network = net
    return loss_and_grad


def _make_callable_loss_fn(f, system, mode, pen, penalties):
    """make_loss_fn for a log-psi callable that is not a network of this library (e.g. the
    Laughlin quasiparticle): E_L through deephall_amd.generic, then the same device statistics,
    packed all-reduce and clipped difference.  Such a callable has no parameters here, so
    only ENERGY_DIFF (optimizer none) is served."""
    from . import generic

    if mode != LossMode.ENERGY_DIFF:
        raise TypeError("parameter gradients need a network of this library (Psiformer)")
    e_fn = generic.local_energy(f, system)

    def loss_and_grad(params, data, n_accept=None, steps=1, flags=None):
        e, o = e_fn(params, data)
        B = e.shape[0]
        e_l = torch.view_as_real(e.to(torch.complex64)).contiguous()
        obs = torch.zeros(B, 8, dtype=torch.float32, device=e.device)  # KE re, im, PE, Lz, Lz^2, L^2
        obs[:, 0] = o["kinetic"].real.float()
        obs[:, 1] = o["kinetic"].imag.float()
        obs[:, 2] = o["potential"].float()
        obs[:, 3] = o["angular_momentum_z"].float()
        obs[:, 4] = o["angular_momentum_z_square"].float()
        obs[:, 5] = o["angular_momentum_square"].float()
        local = device_stats(None, e_l, obs, n_accept, steps, penalties=penalties)
        stats, g = reduce_stats(local, raw=True, flags=flags)
        loss_and_grad.last = (e_l, obs)
        diff, _ = loss_diff(None, e_l, obs, g, *pen)
        return stats, torch.complex(diff[:, 0], diff[:, 1])

    loss_and_grad.network = None
    return loss_and_grad
