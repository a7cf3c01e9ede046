"""The arbitrary-callable boundary (generic.py) on the GPU.

* tests/hamiltonian_test.py:42-76 of the reference, verbatim in substance: analytic
  Slater determinants (l = 1 spherical harmonics at Q = 0; filled lowest Landau levels)
  through make_local_kinetic_energy give KE = 3 / nelec / 2 and L^2 = 0 / 2 (the
  reference asserts atol 1e-3 in float32; here float64 derivatives and a float32
  result: KE atol 1e-5, L^2 atol 1e-4 — L^2 cancels terms of size ~N^2 Q^2).
* dh_kinetic_from_derivatives against oracle.reference.kinetic_from_derivatives
  (hamiltonian.py:115-169 restated) on random complex derivatives, near-pole walkers
  included: within 2e-7 relative (double inside, the float32 rounding of the output).
* The generic MCMC around a callable that evaluates the native network reproduces the
  golden injected-noise fixtures (tests/golden/mcmc_*.npz) and the native dh_mcmc_step
  walkers bit for bit, with the device RNG as well.
"""

from __future__ import annotations

import json
import math
from pathlib import Path

import numpy as np
import pytest
import torch

from deephall_amd import config, generic, hamiltonian
from deephall_amd.mcmc import make_mcmc_step
from deephall_amd.random import Key
from helpers import make_params, make_walkers, oracle_config, to_device_params
from oracle import reference as R
from test_gpu_parity import build, cart_err

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"


def sample(batch, nelec, seed=1898, device="cuda"):
    """hamiltonian_test.py:22-26: theta = arccos U(-1, 1), phi = U(-pi, pi)."""
    g = torch.Generator().manual_seed(seed)
    theta = torch.arccos(torch.rand(batch, nelec, generator=g, dtype=torch.float64) * 2 - 1)
    phi = (torch.rand(batch, nelec, generator=g, dtype=torch.float64) * 2 - 1) * math.pi
    return torch.stack([theta, phi], -1).to(device)


def make_lll(nelec: int, Q: int):
    """hamiltonian_test.py:29-39: the filled lowest Landau levels as one determinant."""

    def log_psi(params, data):
        theta, phi = data[..., 0], data[..., 1]
        u = torch.cos(theta / 2) * torch.exp(1j * phi / 2)
        v = torch.sin(theta / 2) * torch.exp(-1j * phi / 2)
        orb = torch.stack([u**m * v ** (2 * Q - m) for m in range(nelec)], -1)
        sign, logdet = torch.linalg.slogdet(orb)
        return logdet + torch.log(sign)

    return log_psi


def free_electron(params, data):
    """hamiltonian_test.py:43-55: l = 1 spherical harmonics."""
    theta, phi = data[..., 0], data[..., 1]
    orb = torch.stack([torch.sin(theta) * torch.cos(phi), torch.cos(theta), torch.sin(theta) * torch.sin(phi)], -1)
    sign, logdet = torch.linalg.slogdet(orb.to(torch.complex128))
    return logdet + torch.log(sign)


def test_free_electron(cuda):
    data = sample(2, 3)
    ke, obs = hamiltonian.make_local_kinetic_energy(free_electron, Q=0, r=1)(None, data)
    assert torch.allclose(ke.real.double(), torch.full_like(ke.real.double(), 3.0), atol=1e-6)
    assert torch.allclose(obs["angular_momentum_square"].double(), torch.zeros(2, dtype=torch.float64, device=cuda), atol=1e-5)


@pytest.mark.parametrize("nelec,Q,L_square", [(1, 1, 2), (3, 1, 0), (9, 4, 0)])
def test_kinetic_and_angular_momentum(cuda, nelec, Q, L_square):
    data = sample(2, nelec)
    ke, obs = hamiltonian.make_local_kinetic_energy(make_lll(nelec, Q), Q, math.sqrt(Q))(None, data)
    assert torch.allclose(ke.real.double(), torch.full((2,), nelec / 2, dtype=torch.float64, device=cuda), atol=1e-5)
    assert torch.allclose(
        obs["angular_momentum_square"].double(), torch.full((2,), float(L_square), dtype=torch.float64, device=cuda),
        atol=1e-4,
    )
    # orbitals m = 0 .. nelec-1 of u^m v^(2Q-m) carry Lz = m - Q each (a filled shell sums to 0)
    lz = sum(m - Q for m in range(nelec))
    assert (obs["angular_momentum_z"].double() - lz).abs().max().item() < 1e-5
    assert (obs["angular_momentum_z_square"].double() - lz * lz).abs().max().item() < 1e-4


@pytest.mark.parametrize("N,Q,r", [(1, 1.5, 1.3), (3, 0.0, 1.0), (6, 7.5, math.sqrt(7.5)), (20, 28.5, 2.0)])
def test_assembly_matches_oracle(cuda, N, Q, r):
    rng = np.random.default_rng(N)
    B = 33
    x = make_walkers(B, N, seed=N).astype(np.float64)
    x[0, 0, 0] = 1e-3  # near the pole: the cot / 1/sin^2 terms dominate
    x[1, -1, 0] = math.pi - 2e-3
    g = rng.standard_normal((B, N, 2)) + 1j * rng.standard_normal((B, N, 2))
    H = rng.standard_normal((B, N, 2, N, 2)) + 1j * rng.standard_normal((B, N, 2, N, 2))
    H = (H + H.transpose(0, 3, 4, 1, 2)) / 2  # a Hessian is symmetric
    xd = torch.tensor(x, device=cuda)
    ke, obs = generic.kinetic_from_derivatives(xd, torch.tensor(g, device=cuda), torch.tensor(H, device=cuda), Q, r)
    for b in range(B):
        xt = torch.tensor(x[b])
        kref, oref = R.kinetic_from_derivatives(
            torch.tensor(g[b, :, 0]), torch.tensor(g[b, :, 1]), torch.tensor(H[b]), xt[:, 0], xt[:, 1], Q, r
        )
        # outputs are float32 (dh_local_energy's layout): compare at f32 rounding of the value
        def close(a, ref):
            ref = float(ref)
            assert abs(float(a) - ref) <= 2e-7 * max(1.0, abs(ref)), (b, float(a), ref)

        close(ke[b].real, kref.real)
        close(ke[b].imag, kref.imag)
        for k in ("angular_momentum_z", "angular_momentum_z_square", "angular_momentum_square"):
            close(obs[k][b], oref[k])


def test_generic_local_energy(cuda):
    """local_energy(f, system) for a callable (filled shell N = 3, Q = 1, Coulomb, r = 1):
    E_L = KE + strength * PE with KE = N / 2 and PE = sum_{i<j} 1 / |r_i - r_j| / r."""
    system = config.System(nspins=(3, 0), flux=2, interaction_strength=0.7)
    data = sample(5, 3, seed=3)
    e, obs = hamiltonian.local_energy(make_lll(3, 1), system)(None, data)
    xs = data.cpu()
    pe_ref = []
    for b in range(5):
        th, ph = xs[b, :, 0], xs[b, :, 1]
        xyz = torch.stack([torch.sin(th) * torch.cos(ph), torch.sin(th) * torch.sin(ph), torch.cos(th)], -1)
        pe_ref.append(R.coulomb_potential(xyz @ xyz.T, 1.0))
    pe_ref = torch.stack(pe_ref)
    assert torch.allclose(obs["potential"].double().cpu(), 0.7 * pe_ref, rtol=1e-5)
    assert torch.allclose(e.real.double().cpu(), 1.5 + 0.7 * pe_ref, rtol=1e-5)
    assert torch.allclose(e, obs["kinetic"] + obs["potential"].to(e.dtype))


@pytest.mark.parametrize("name", ["C1", "C2"])
def test_generic_mcmc_golden(cuda, name):
    """A callable wrapping the native network walks the golden injected-noise chain."""
    g = np.load(GOLDEN / f"mcmc_{name}.npz")
    ocfg = R.OracleConfig(**json.loads(str(g["config"])))
    ocfg.nspins = tuple(ocfg.nspins)
    _, model = build(ocfg)
    params = to_device_params(make_params(ocfg))
    noise = torch.tensor(g["noise"], device=cuda)
    steps, B = noise.shape[:2]

    def batch_network(p, data):  # an opaque callable: not resolvable to the network
        return model.apply(p, data)

    step = make_mcmc_step(batch_network, batch_per_device=B, steps=steps)
    assert step.__module__ == generic.__name__
    x = torch.tensor(g["x0"], device=cuda)
    x, pmove = step(params, x, Key(0), float(g["width"]), noise=noise)
    assert np.array_equal(step.last_n_accept.cpu().numpy(), g["n_acc"])
    assert cart_err(x.cpu().numpy(), g["x"]) < 2e-6
    assert float(pmove) == pytest.approx(g["n_acc"].sum() / (steps * B))


def test_generic_mcmc_matches_native(cuda):
    """Same walkers, acceptances and lp as dh_mcmc_step with the device RNG."""
    ocfg = oracle_config("C2")
    _, model = build(ocfg)
    params = to_device_params(make_params(ocfg))
    B, N = 256, ocfg.nelec
    x0 = torch.tensor(make_walkers(B, N, seed=4), device=cuda)
    native = make_mcmc_step(model, batch_per_device=B, steps=6)
    xa, pa = native(params, x0.clone(), Key(21, 40), 0.15, walker_offset=5)
    gen = make_mcmc_step(lambda p, d: model.apply(p, d), batch_per_device=B, steps=6)
    xb, pb = gen(params, x0.clone(), Key(21, 40), 0.15, walker_offset=5)
    assert torch.equal(native.last_n_accept, gen.last_n_accept)
    assert torch.equal(xa, xb)
    assert torch.equal(native.last_lp, gen.last_lp)
    assert float(pa) == float(pb)


def test_generic_mcmc_analytic_callable(cuda):
    """A pure-torch log psi (filled LLL, N = 3, Q = 1): walkers move, lp = 2 Re log psi(x)."""
    f = make_lll(3, 1)

    def batch_network(p, data):
        return torch.stack([f(p, data[b].double()) for b in range(data.shape[0])])

    B = 64
    x = sample(B, 3, seed=5).float().contiguous()
    x0 = x.clone()
    step = make_mcmc_step(batch_network, batch_per_device=B, steps=4)
    x, pmove = step(None, x, Key(3), 0.3)
    assert 0.05 < float(pmove) <= 1.0
    moved = (x != x0).any(-1).any(-1)
    assert torch.equal(moved, step.last_n_accept > 0)
    assert torch.allclose(step.last_lp.double(), 2 * batch_network(None, x).real, atol=1e-5)
