"""NetObs estimators on MI355X (deephall/netobs_bridge/observables/*.py).

* kernels vs the float64 restatement (oracle/netobs.py): theta / pair-angle histograms on
  random walkers, the LLL monopole harmonics at flux 2..57, the one-body density matrix
  estimator of a random Psiformer with the oracle's float64 log-amplitudes;
* analytic pins: the filled lowest Landau level (the engineered Psiformer droplet, N = 3,
  2Q = 2, sampled by the native MCMC) has 1-RDM = identity (diagonal 1, trace N); the
  Laughlin state's overlap with itself is 1;
* the driver: a short training run's checkpoint restored by DeepHallAdaptor and evaluated
  with every estimator (counts, normalisation, shapes).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from deephall_amd import Config, config, make_mcmc_step, make_network, train
from deephall_amd.netobs import DeepHallAdaptor, HallSystem, evaluate
from deephall_amd.netobs._native import histograms, monopole_orbitals
from deephall_amd.netobs.observables import density, one_rdm, overlap, pair_corr
from deephall_amd.random import Key
from deephall_amd.train import init_guess
from helpers import make_params, make_walkers, oracle_config, to_device_params
from oracle import netobs as O
from oracle import reference as R
from test_gpu_parity import build
from test_oracle_kat import engineered_params

pytestmark = pytest.mark.gpu


def uniform(B, N, seed):
    rng = np.random.default_rng(seed)
    return np.stack([np.arccos(rng.uniform(-1, 1, (B, N))), rng.uniform(-np.pi, np.pi, (B, N))], -1).astype(np.float32)


def test_histograms_match_oracle(cuda):
    x = uniform(3000, 6, 1)
    d, p = histograms(torch.tensor(x, device=cuda), density_bins=50, pair_bins=200)
    d_ref = O.density_hist(x, 50)
    p_ref = O.pair_corr(x, 200) * 3000 * 36 * np.pi / (4 * 200)  # unnormalised weighted counts
    assert np.abs(d.cpu().numpy() - d_ref).max() <= 1.0  # a value on a bin edge may fall either side
    assert d.sum().item() == 3000 * 6
    assert np.allclose(p.cpu().numpy(), p_ref, rtol=2e-4, atol=1e-3)


@pytest.mark.parametrize("flux", [2, 6, 15, 23, 57])
def test_monopole_orbitals_match_oracle(cuda, flux):
    pts = uniform(256, 1, flux)[:, 0]
    pts[:4, 0] = [0.0, 1e-3, np.pi - 1e-3, np.pi]  # the clipped poles
    y = monopole_orbitals(torch.tensor(pts, device=cuda), flux).cpu().numpy()
    y_ref = O.lll_orbitals(pts.astype(np.float64), flux)
    assert np.max(np.abs(y - y_ref)) < 2e-6 * max(1.0, np.max(np.abs(y_ref)))


class _Adaptor:
    """The adaptor surface the estimators use: cfg, model, call_network."""

    def __init__(self, model, cfg=None):
        self.model, self.cfg = model, cfg

    def call_network(self, params, x, system=None):
        return self.model.apply(params, x)


def test_one_rdm_product_matches_oracle(cuda):
    ocfg = oracle_config("C2")
    system, model = build(ocfg)
    p64 = make_params(ocfg, seed=11)
    params = to_device_params(p64)
    x = make_walkers(8, ocfg.nelec, seed=4)
    rp = uniform(8, 1, 9)[:, 0]
    est = one_rdm.OneRDMEstimator(_Adaptor(model), HallSystem([6, 0], flux=15), {}, {})
    got = est.product(params, torch.tensor(x, device=cuda), torch.tensor(rp, device=cuda)).cpu().numpy()
    xt = torch.tensor(x, dtype=torch.float64)
    lp = R.batch_logpsi(p64, ocfg, xt).numpy()
    xp = np.repeat(x[:, None], 6, 1).astype(np.float64)
    for a in range(6):
        xp[:, a, a] = rp
    lpp = R.batch_logpsi(p64, ocfg, torch.tensor(xp.reshape(-1, 6, 2))).numpy().reshape(8, 6)
    ref = O.one_rdm_product(x.astype(np.float64), rp.astype(np.float64), lp, lpp, 15)
    assert np.max(np.abs(got - ref)) < 2e-4 * np.max(np.abs(ref))


def test_filled_lll_one_rdm_is_identity(cuda):
    """N = 2Q + 1 = 3: the droplet fills the LLL, so rho = 1 in the Y_{Q,Q,m} basis."""
    ocfg = oracle_config("C1", interaction_strength=0.0)
    system, model = build(ocfg)
    params = to_device_params(engineered_params(ocfg))
    B = 4096
    x = init_guess(Key(3), B, 3, cuda, network=model)
    step = make_mcmc_step(model, batch_per_device=B, steps=10)
    key = Key(5)
    for _ in range(30):
        x, _ = step(params, x, key, 0.3)
        key = key.advance(10)
    est = one_rdm.OneRDMEstimator(_Adaptor(model), HallSystem([3, 0], flux=2), {}, {})
    acc = torch.zeros(3, 3, dtype=torch.complex64)
    nsteps = 20
    for i in range(nsteps):
        x, _ = step(params, x, key, 0.3)
        key = key.advance(10)
        r = init_guess(Key(1000 + i), B, 1, cuda, network=model)[:, 0]
        acc += est.product(params, x, r).mean(0).cpu()
    rho = (acc / nsteps).numpy()
    print("filled LLL 1-RDM:\n", np.round(rho, 3))
    assert np.allclose(np.diag(rho).real, 1.0, atol=0.05)
    assert abs(np.trace(rho).real - 3.0) < 0.05
    assert np.max(np.abs(rho - np.diag(np.diag(rho)))) < 0.05


def test_overlap_of_laughlin_with_itself(cuda):
    sys_cfg = config.System(nspins=(3, 0), flux=6)
    net_cfg = config.Network()
    net_cfg.type = config.NetworkType.laughlin
    lau = make_network(sys_cfg, net_cfg)
    cfg = Config.from_dict({"system": {"nspins": (3, 0), "flux": 6}, "network": {"type": "laughlin"}})
    est = overlap.OverlapEstimator(_Adaptor(lau, cfg), HallSystem([3, 0], flux=6), {}, {})
    values, state = est.empty_val_state(3)
    x = torch.tensor(make_walkers(512, 3, seed=2), device=cuda)
    for i in range(3):
        v, state = est.evaluate(i, {}, None, x, None, state, None)
        values["ratio"][i] = v["ratio"].mean()
        values["ratio_square"][i] = v["ratio_square"].mean()
    ov = est.digest(values, state)["overlap"].item()
    assert abs(ov - 1.0) < 1e-5
    r, r2 = O.overlap_ratio(np.zeros(4), np.ones(4) * 0.3)
    assert abs(O.overlap_digest(r, r2) - 1.0) < 1e-12


def test_driver_on_a_checkpoint(cuda, tmp_path):
    cfg = Config.from_dict({
        "batch_size": 64, "seed": 3,
        "system": {"nspins": (3, 0), "flux": 6, "interaction_strength": 0.0},  # 2Q = 6: Laughlin 1/3 exists
        "network": {"psiformer": {"num_layers": 1, "num_heads": 1, "heads_dim": 4}},
        "mcmc": {"burn_in": 5},
        "optim": {"iterations": 3, "optimizer": "adam"},
        "log": {"save_path": str(tmp_path)},
    })
    train(cfg)
    ckpt = sorted(tmp_path.glob("ckpt_*.npz"))[-1]
    steps = 4
    out, _ = evaluate(DeepHallAdaptor(), density.DEFAULT, ckpt, steps, burn_in=3)
    assert out["map"].shape == (50,) and out["map"].sum().item() == steps * 64 * 3
    out, _ = evaluate(DeepHallAdaptor(), pair_corr.DEFAULT, ckpt, steps, burn_in=3, estimator_options={"bins": 40})
    assert out["pair_corr"].shape == (40,) and torch.isfinite(out["pair_corr"]).all()
    out, vals = evaluate(DeepHallAdaptor(), one_rdm.DEFAULT, ckpt, steps, burn_in=3)
    assert vals["one_rdm"].shape == (steps, 7, 7) and out["diagonal"].shape == (7,)
    # trace = N x the state's weight in the lowest Landau level (<= N; the Jastrow factor of
    # a 3-iteration network moves some weight out); a 4-step, 64-walker estimate is noisy
    assert torch.isfinite(out["trace"]).all() and 0.3 < out["trace"].real.item() < 4.0
    out, vals = evaluate(DeepHallAdaptor(), overlap.DEFAULT, ckpt, steps, burn_in=3)
    assert 0.0 <= out["overlap"].item() <= 1.0 + 1e-6
