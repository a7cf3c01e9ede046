"""Laughlin quasiparticle (networks/laughlin.py:82-100) on the host, float64: the state
carries Lz = excitation_lz (a rotation about z by a multiplies psi by exp(i Lz a)), its
filling and Lz are validated as laughlin.py:34-52 does, and make_network picks it for
N = 2 Q1 + 2.  The GPU pins (KE = N/2, L^2 = L (L + 1)) are in test_gpu_laughlin.py."""

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
    assert isinstance(make_network(config.System(nspins=(4, 0), flux=8), net), LaughlinQuasiparticle)
    assert isinstance(make_network(config.System(nspins=(4, 0), flux=10), net), Laughlin)  # quasihole
    with pytest.raises(ValueError):
        LaughlinQuasiparticle((4, 0), 8, excitation_lz=0.5)  # Lz - Q1 not an integer
    with pytest.raises(ValueError):
        LaughlinQuasiparticle((4, 0), 8, excitation_lz=3.0)  # |Lz| > Q1 + 1
    with pytest.raises(ValueError):
        LaughlinQuasiparticle((4, 0), 10)  # not the quasiparticle filling
