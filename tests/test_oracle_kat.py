"""Pin the float64 oracle to the reference's own known answers (CPU).

* tests/hamiltonian_test.py:42-62 (free electrons, Q=0, r=1): KE = 3, L^2 = 0
* tests/hamiltonian_test.py:65-76 (LLL Slater determinants u^m v^(2Q-m), r=sqrt Q):
  KE = N/2, L^2 in {2, 0, 0} for (N, Q) = (1,1), (3,1), (9,4); atol 1e-3
* engineered Psiformer: orbital kernels 0, real bias delta(p, j), Jastrow 0 ->
  Phi = LLL determinant u^j v^(2Q-j), j < N, so KE = N/2 and L^2 = L(L+1) with
  L = |Lz| = |sum_j (j - Q)| for EVERY walker, through the real network code.
* the forward-mode channel restatement agrees with the full-Hessian one.
"""

from __future__ import annotations

import math

import numpy as np
import pytest
import torch

from helpers import make_params, make_walkers, oracle_config
from oracle import channels as CH
from oracle import reference as R


def sample(B, N, seed=1898):
    g = np.random.default_rng(seed)
    return torch.tensor(R.init_guess_from_uniforms(g.random((B, N)), g.random((B, N))))


def lll(N, Q):
    def f(p, x):
        th, ph = x[..., 0], x[..., 1]
        u = torch.cos(th / 2) * torch.exp(0.5j * ph.to(torch.complex128))
        v = torch.sin(th / 2) * torch.exp(-0.5j * ph.to(torch.complex128))
        orb = torch.stack([u**m * v ** (2 * Q - m) for m in range(N)], -1)
        s, ld = torch.linalg.slogdet(orb)
        return ld + torch.log(s)

    return f


def test_free_electron():
    def f(p, x):
        th, ph = x[..., 0], x[..., 1]
        orb = torch.stack([torch.sin(th) * torch.cos(ph), torch.cos(th), torch.sin(th) * torch.sin(ph)], -1)
        s, ld = torch.linalg.slogdet(orb.to(torch.complex128))
        return ld + torch.log(s)

    x = sample(2, 3)
    ke = R.make_local_kinetic_energy(f, 0, 1.0)
    for b in range(2):
        k, o = ke(None, x[b])
        assert abs(k - 3) < 1e-3
        assert abs(o["angular_momentum_square"]) < 1e-3


@pytest.mark.parametrize("nelec,Q,L_square", [(1, 1, 2), (3, 1, 0), (9, 4, 0)])
def test_kinetic_and_angular_momentum(nelec, Q, L_square):
    x = sample(2, nelec)
    ke = R.make_local_kinetic_energy(lll(nelec, Q), Q, math.sqrt(Q))
    for b in range(2):
        k, o = ke(None, x[b])
        assert abs(k - nelec / 2) < 1e-3
        assert abs(o["angular_momentum_square"] - L_square) < 1e-3


def engineered_params(cfg, seed=5):
    """Psiformer whose determinant is the LLL droplet u^j v^(2Q-j), j = 0..N-1."""
    p = R.init_params(cfg, seed=seed)
    M, N = int(cfg.flux) + 1, cfg.nelec
    ob = "Orbitals_0/featured_orbitals/"
    for k in list(p):
        if k.startswith(ob):
            p[k] = torch.zeros_like(p[k])
    b = torch.zeros(M, N, 1, dtype=torch.float64)
    for j in range(N):
        b[j, j, 0] = 1.0
    p[ob + "DenseGeneral_0/bias"] = b
    p["Jastrow_0/ee_par"][:] = 0.0
    p["Jastrow_0/ee_anti"][:] = 0.0
    return p


def droplet_L2(N, flux):
    Lz = sum(j - flux / 2 for j in range(N))
    return abs(Lz) * (abs(Lz) + 1), Lz


@pytest.mark.parametrize("name", ["C1", "C2"])
def test_engineered_psiformer_known_answer(name):
    cfg = oracle_config(name, interaction_strength=0.0)
    p = engineered_params(cfg)
    x = torch.tensor(make_walkers(3, cfg.nelec), dtype=torch.float64)
    L2, Lz = droplet_L2(cfg.nelec, cfg.flux)
    e, o = R.local_energy(p, cfg, x[:2])
    assert np.allclose(o["kinetic"].numpy(), cfg.nelec / 2, atol=1e-8)
    assert np.allclose(o["angular_momentum_square"].numpy(), L2, atol=1e-6)
    assert np.allclose(o["angular_momentum_z"].numpy(), Lz, atol=1e-8)
    _, ke, o2, _ = CH.local_energy(p, cfg, x)
    assert np.allclose(ke.numpy(), cfg.nelec / 2, atol=1e-8)
    assert np.allclose(o2["angular_momentum_square"].numpy(), L2, atol=1e-6)
    assert np.allclose(o2["angular_momentum_z_square"].numpy(), Lz * Lz, atol=1e-6)


@pytest.mark.parametrize("name", ["C1", "MIX"])
def test_channels_match_full_hessian(name):
    cfg = oracle_config(name)
    p = make_params(cfg)
    x = torch.tensor(make_walkers(3, cfg.nelec), dtype=torch.float64)
    e, o = R.local_energy(p, cfg, x)
    lp = R.batch_logpsi(p, cfg, x)
    lp2, ke, o2, _ = CH.local_energy(p, cfg, x)
    assert torch.allclose(lp, lp2, atol=1e-10)
    assert torch.allclose(o["kinetic"], ke, atol=1e-9)
    for k in o2:
        assert torch.allclose(o[k], o2[k], atol=1e-8), k


def test_gradient_finite_difference():
    cfg = oracle_config("C1")
    p = make_params(cfg)
    x = torch.tensor(make_walkers(1, cfg.nelec), dtype=torch.float64)[0]
    f = lambda y: R.logpsi(p, cfg, y).real  # noqa: E731
    g = torch.func.grad(f)(x)
    eps = 1e-6
    for i in range(cfg.nelec):
        for a in range(2):
            d = torch.zeros_like(x)
            d[i, a] = eps
            fd = (f(x + d) - f(x - d)) / (2 * eps)
            assert abs(fd - g[i, a]) < 1e-6
