"""Laughlin wavefunction (networks/laughlin.py:19-100) on MI355X.

* log psi and the local energy (KE, Lz, Lz^2, L^2, PE) against the float64 restatement
  (oracle.reference.laughlin_*: the reference module restated in torch, autograd full
  Hessian through hamiltonian.py's formulas); the kernels work in double, so 1e-5.
* Analytic pins on every walker of a full batch: the Laughlin ground state lies in the
  lowest Landau level with L = 0 (KE = N/2, L^2 = Lz = 0); the quasihole has L = Q1
  (L^2 = Q1 (Q1 + 1), Lz = excitation_lz); the quasiparticle (laughlin.py:82-100) has
  L = Q1 + 1 = N/2 — on the native kernel and, as an independent route, on the reference's
  slogdet form through the callable boundary (torch.func derivatives).
* The reference's CLI test restated (tests/cli_test.py:24-42): Laughlin N=3, 2Q=6,
  Coulomb, optimizer none, 100 iterations, seed 42, batch 3360 -> the energy log shows
  2.58 and L_square=0.0000.
"""

from __future__ import annotations

import csv
import logging

import numpy as np
import pytest
import torch

from deephall_amd import Config, config, hamiltonian, make_network, train
from helpers import make_walkers
from oracle import reference as R

pytestmark = pytest.mark.gpu
CASES = [dict(nspins=(3, 0), flux=6), dict(nspins=(5, 0), flux=12), dict(nspins=(4, 0), flux=10, excitation_lz=0.0),
         dict(nspins=(4, 0), flux=10, excitation_lz=1.0), dict(nspins=(2, 1), flux=6, interaction_type="harmonic"),
         dict(nspins=(3, 0), flux=6, radius=2.0),
         # quasiparticle fillings N = 2 Q1 + 2 (laughlin.py:82-100): lz = -2 / 2 are the edge
         # orbitals whose u^(Q1+m1) / v^(Q1-m1) exponent is -1 (its weight Q1 + 1 -+ m1 is 0)
         dict(nspins=(4, 0), flux=8, excitation_lz=1.0), dict(nspins=(4, 0), flux=8, excitation_lz=-2.0),
         dict(nspins=(4, 0), flux=8, excitation_lz=2.0), dict(nspins=(6, 0), flux=14, excitation_lz=0.0),
         dict(nspins=(3, 2), flux=11, excitation_lz=0.5, interaction_type="harmonic")]


def build(case):
    lz = case.get("excitation_lz", 0.0)
    system = config.System(nspins=case["nspins"], flux=case["flux"], lz_center=lz, radius=case.get("radius"),
                           interaction_type=config.InteractionType(case.get("interaction_type", "coulomb")))
    net = config.Network()
    net.type = config.NetworkType.laughlin
    ocfg = R.LaughlinConfig(nspins=case["nspins"], flux=case["flux"], excitation_lz=lz, radius=case.get("radius"),
                            interaction_type=case.get("interaction_type", "coulomb"))
    return system, make_network(system, net), ocfg


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_laughlin_vs_oracle(cuda, case):
    system, model, ocfg = build(case)
    params = model.init(0, device=cuda)
    x = make_walkers(8, ocfg.nelec, seed=7, margin=0.05)
    xt = torch.tensor(x, dtype=torch.float64)
    lp = model.apply(params, torch.tensor(x, device=cuda)).cpu().numpy()
    lp_ref = np.array([complex(R.laughlin_logpsi(ocfg, xt[b]).item()) for b in range(len(x))])
    assert np.max(np.abs(lp.real - lp_ref.real) / np.maximum(1, np.abs(lp_ref.real))) < 1e-6
    assert np.max(np.abs(np.angle(np.exp(1j * (lp.imag - lp_ref.imag))))) < 1e-5
    e, o = hamiltonian.local_energy(model, system)(params, torch.tensor(x, device=cuda))
    e_ref, o_ref = R.laughlin_local_energy(ocfg, xt)
    scale = lambda v: np.maximum(1.0, np.abs(v))  # noqa: E731
    assert np.max(np.abs(e.cpu().numpy() - e_ref.numpy()) / scale(e_ref.numpy())) < 1e-5
    for k in ("kinetic", "potential", "angular_momentum_z", "angular_momentum_z_square", "angular_momentum_square"):
        ref = o_ref[k].detach().numpy()
        assert np.max(np.abs(o[k].cpu().numpy() - ref) / scale(ref)) < 1e-5, k


@pytest.mark.parametrize("case,L2", [(dict(nspins=(3, 0), flux=6), 0.0), (dict(nspins=(6, 0), flux=15), 0.0),
                                     (dict(nspins=(4, 0), flux=10, excitation_lz=1.0), 6.0)])
def test_laughlin_analytic_pins(cuda, case, L2):
    system, model, ocfg = build(case)
    params = model.init(0, device=cuda)
    x = torch.tensor(make_walkers(4096, ocfg.nelec, seed=3, margin=0.05), device=cuda)
    e, o = hamiltonian.local_energy(model, system)(params, x)
    N = ocfg.nelec
    lz = case.get("excitation_lz", 0.0)
    st = torch.sin(x[..., 0].double().cpu())
    geo = (ocfg.Q**2 * (1 / st).sum(-1) ** 2).numpy()  # size of the cancelling magnetic terms
    for k, want in (("kinetic", N / 2), ("angular_momentum_square", L2), ("angular_momentum_z", lz),
                    ("angular_momentum_z_square", lz * lz)):
        err = np.abs(o[k].real.cpu().numpy() - want) / np.maximum(1.0, geo)
        assert np.max(err) < 1e-6, (k, np.max(err))


@pytest.mark.parametrize("N,lz,B", [(4, 0.0, 4096), (4, 1.0, 4096), (4, -2.0, 4096), (4, 2.0, 4096), (6, 1.0, 4096),
                                    (8, -1.0, 1024), (10, 0.0, 512)])
def test_quasiparticle_analytic_pins(cuda, N, lz, B):
    """laughlin.py:82-100 (N = 2 Q1 + 2, 2Q = 3 (N - 1) - 1): the LLL-projected quasiparticle
    is a lowest-Landau-level state (KE = N/2 on every walker) with L = Q1 + 1 = N/2 and
    Lz = excitation_lz — on every walker of a batch, through the native kernel (laughlin.hip,
    make_network's model), and on the first 128 walkers also through the callable boundary
    (torch.func derivatives of the reference's slogdet form, `LaughlinQuasiparticle`): the
    two routes agree to 1e-6 relative on log psi and to 1e-5 (relative to the size of the
    cancelling magnetic terms, as the pins) on every observable."""
    from deephall_amd.networks import Laughlin, LaughlinQuasiparticle

    flux = 3 * (N - 1) - 1
    system = config.System(nspins=(N, 0), flux=flux, lz_center=lz)
    net = config.Network()
    net.type = config.NetworkType.laughlin
    model = make_network(system, net)
    assert isinstance(model, Laughlin)
    x = torch.tensor(make_walkers(B, N, seed=5, margin=0.05), device=cuda)
    params = model.init(0, device=cuda)
    e, o = hamiltonian.local_energy(model, system)(params, x)
    L = N / 2
    st = torch.sin(x[..., 0].double().cpu())
    geo = ((flux / 2) ** 2 * (1 / st).sum(-1) ** 2).numpy()  # size of the cancelling magnetic terms
    for k, want in (("kinetic", N / 2), ("angular_momentum_square", L * (L + 1)), ("angular_momentum_z", lz),
                    ("angular_momentum_z_square", lz * lz)):
        err = np.abs(o[k].real.cpu().numpy() - want) / np.maximum(1.0, geo)
        assert np.max(err) < 1e-5, (k, np.max(err))
    assert np.max(np.abs(o["kinetic"].imag.cpu().numpy()) / np.maximum(1.0, geo)) < 1e-5
    # the callable route on the same walkers
    qp = LaughlinQuasiparticle(flux=flux, nspins=(N, 0), excitation_lz=lz, system=system)
    assert qp.Q1 == (N - 2) / 2
    xs = x[:128].contiguous()
    lp_native = model.apply(params, xs).cpu().numpy()
    lp_callable = qp(None, xs).cpu().numpy()
    assert np.max(np.abs(lp_native.real - lp_callable.real) / np.maximum(1, np.abs(lp_callable.real))) < 1e-6
    assert np.max(np.abs(np.angle(np.exp(1j * (lp_native.imag - lp_callable.imag))))) < 1e-5
    e2, o2 = hamiltonian.local_energy(qp, system)(qp.init(), xs)
    for k in ("kinetic", "potential", "angular_momentum_z", "angular_momentum_z_square", "angular_momentum_square"):
        a, r = o[k][:128].cpu().numpy(), o2[k].cpu().numpy()
        err = np.abs(a - r) / np.maximum(np.maximum(1.0, np.abs(r)), geo[:128])
        print(f"N={N} lz={lz} {k}: native vs callable {np.max(err):.1e}")
        assert np.max(err) < 1e-5, (k, np.max(err))


def test_quasiparticle_mcmc(cuda):
    """make_mcmc_step on the quasiparticle callable (the generic path: HIP proposal / accept on
    the dh_mcmc_step random streams): walkers stay on the sphere, the acceptance is sane, and
    log psi of the moved walkers equals the callable's."""
    from deephall_amd.mcmc import make_mcmc_step
    from deephall_amd.random import PRNGKey

    system = config.System(nspins=(4, 0), flux=8, lz_center=1.0)
    net = config.Network()
    net.type = config.NetworkType.laughlin
    model = make_network(system, net)
    x = torch.tensor(make_walkers(512, 4, seed=9, margin=0.05), device=cuda).contiguous()
    step = make_mcmc_step(model, batch_per_device=512, steps=5)
    x, pmove = step(model.init(), x, PRNGKey(2), 0.3)
    pm = float(pmove)
    assert 0.05 < pm <= 1.0, pm
    assert torch.isfinite(x).all()
    assert (x[..., 0] >= 0).all() and (x[..., 0] <= np.pi).all()
    lp = model.apply(model.init(0, device=cuda), x)
    assert torch.isfinite(lp.real).all()


def test_cli_laughlin_energy(cuda, tmp_path):
    """tests/cli_test.py:24-42 restated: the MC energy of the N=3, 2Q=6 Laughlin state."""
    cfg = Config.from_dict({
        "seed": 42,
        "system": {"nspins": (3, 0), "flux": 6},
        "network": {"type": "laughlin"},
        "optim": {"iterations": 100, "optimizer": "none"},
        "log": {"save_path": str(tmp_path)},
    })
    lines = []

    class Capture(logging.Handler):
        def emit(self, record):
            lines.append(record.getMessage())

    h = Capture()
    logging.getLogger("deephall_amd").addHandler(h)
    try:
        train(cfg)
    finally:
        logging.getLogger("deephall_amd").removeHandler(h)
    with open(tmp_path / "train_stats.csv") as f:
        rows = list(csv.DictReader(f))
    e = np.array([float(r["energy"]) for r in rows])
    print("Laughlin N=3 2Q=6 energy: mean", e.mean(), "min", e.min(), "max", e.max())
    assert abs(e.mean() - 2.58) < 0.01
    text = "\n".join(lines)
    assert "energy=2.58" in text
    assert all(r["L_square"] in ("0.0000", "-0.0000") for r in rows)


def test_quasiparticle_train_inference(cuda, tmp_path):
    """The deephall CLI flow (train.py:80-167, optimizer none) on the quasiparticle: MCMC and
    statistics through the callable boundary; the logged L_square is L (L + 1) = 6 and Lz the
    excitation_lz on every iteration (exact eigenstate), the kinetic energy N/2 = 2."""
    cfg = Config.from_dict({
        "seed": 7,
        "batch_size": 256,
        "system": {"nspins": (4, 0), "flux": 8, "lz_center": 1.0},
        "network": {"type": "laughlin"},
        "mcmc": {"burn_in": 5},
        "optim": {"iterations": 4, "optimizer": "none"},
        "log": {"save_path": str(tmp_path)},
    })
    train(cfg)
    with open(tmp_path / "train_stats.csv") as f:
        rows = list(csv.DictReader(f))
    assert len(rows) == 4
    for r in rows:
        assert abs(float(r["L_square"]) - 6.0) < 1e-3, r
        assert abs(float(r["Lz"]) - 1.0) < 1e-3, r
        assert np.isfinite(float(r["energy"]))
