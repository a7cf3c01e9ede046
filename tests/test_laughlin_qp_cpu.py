"""Laughlin quasiparticle (networks/laughlin.py:82-100) on the host, float64: the state
carries Lz = excitation_lz (a rotation about z by a multiplies psi by exp(i Lz a)), its
filling and Lz are validated as laughlin.py:34-52 does — by the callable form and by the
native dh_create (laughlin.hip serves make_network's model for N = 2 Q1 + 2).  The GPU pins (KE = N/2, L^2 = L (L + 1)) are in test_gpu_laughlin.py."""

from __future__ import annotations

import math

import pytest
import torch

from deephall_amd import config, make_network
from deephall_amd.networks import Laughlin, LaughlinQuasiparticle


def _walkers(N, seed):
    g = torch.Generator().manual_seed(seed)
    th = torch.arccos(torch.rand(N, generator=g, dtype=torch.float64) * 2 - 1)
    ph = (torch.rand(N, generator=g, dtype=torch.float64) * 2 - 1) * math.pi
    return torch.stack([th, ph], -1)


@pytest.mark.parametrize("N,lz", [(4, 0.0), (4, 1.0), (4, 2.0), (6, -1.0)])
def test_quasiparticle_lz_phase(N, lz):
    m = LaughlinQuasiparticle((N, 0), 3 * (N - 1) - 1, excitation_lz=lz)
    for seed in range(4):
        x = _walkers(N, seed)
        a = 0.37
        xr = x.clone()
        xr[:, 1] += a
        d = (m(None, xr) - m(None, x))
        assert abs(d.real.item()) < 1e-10
        assert abs(math.remainder(d.imag.item() - lz * a, 2 * math.pi)) < 1e-10


def test_quasiparticle_permutation_antisymmetry():
    m = LaughlinQuasiparticle((4, 0), 8, excitation_lz=1.0)
    x = _walkers(4, 11)
    xs = x[[1, 0, 2, 3]]
    d = m(None, xs) - m(None, x)
    assert abs(d.real.item()) < 1e-10 and abs(math.remainder(d.imag.item() - math.pi, 2 * math.pi)) < 1e-10


def test_quasiparticle_selection_and_checks():
    net = config.Network()
    net.type = config.NetworkType.laughlin
    assert isinstance(make_network(config.System(nspins=(4, 0), flux=8), net), Laughlin)  # native kernel
    assert isinstance(make_network(config.System(nspins=(4, 0), flux=10), net), Laughlin)  # quasihole
    with pytest.raises(ValueError):
        LaughlinQuasiparticle((4, 0), 8, excitation_lz=0.5)  # Lz - Q1 not an integer
    with pytest.raises(ValueError):
        LaughlinQuasiparticle((4, 0), 8, excitation_lz=3.0)  # |Lz| > Q1 + 1
    with pytest.raises(ValueError):
        LaughlinQuasiparticle((4, 0), 10)  # not the quasiparticle filling


def test_native_quasiparticle_validation():
    """dh_create (network_type laughlin) accepts the quasiparticle filling N = 2 Q1 + 2 with
    Lz - Q1 integer and |Lz| <= Q1 + 1 (laughlin.py:44-52) and rejects the rest."""
    import ctypes as C

    from deephall_amd import _lib
    from deephall_amd.networks.psiformer import NetworkSpec

    lib = _lib.load()

    def create(nspins, flux, lz):
        spec = NetworkSpec(nspins=nspins, flux=flux, ndets=1, num_heads=1, heads_dim=4, num_layers=0,
                           network_type="laughlin", excitation_lz=lz)
        h = C.c_void_p()
        rc = lib.dh_create(C.byref(spec.to_c()), C.byref(h))
        if rc == 0:
            lib.dh_destroy(h)
        return rc

    for lz in (-2.0, -1.0, 0.0, 1.0, 2.0):
        assert create((4, 0), 8, lz) == 0, lz  # Q1 = 1
    assert create((3, 2), 11, 0.5) == 0  # Q1 = 3/2
    for lz in (0.5, 3.0, -3.0):
        assert create((4, 0), 8, lz) != 0, lz
        assert b"quasiparticle" in lib.dh_last_error()
    assert create((4, 0), 11, 0.0) != 0  # 2 Q1 = 5: no supported filling
