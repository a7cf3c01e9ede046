"""CPU checks of the KFAC restatement (oracle/kfac.py; parity unpinned: kfac_jax is not
importable here).  The layer taps must see exactly the network's dense
layers: for every block, sum over rows of x~^T dy equals sqrt(2) times the autograd
gradient of sum_b Re log psi_b with respect to [kernel; bias]; the factors are symmetric
positive semi-definite; the damped inverses invert the pi-adjusted factors; averaging
device shards equals the full-batch statistics for the dense factors."""

from __future__ import annotations

import math

import numpy as np
import torch

from helpers import make_params, make_walkers, oracle_config
from oracle import kfac as KF
from oracle import reference as R


def _cfg():
    return oracle_config("MIX", num_layers=1)


def test_taps_reproduce_parameter_gradient():
    cfg = _cfg()
    p = make_params(cfg)
    xs = torch.tensor(make_walkers(4, cfg.nelec, seed=2), dtype=torch.float64)
    bl, generic = KF.blocks(cfg)
    ct = torch.zeros(4, 2, dtype=torch.float64)
    ct[:, 0] = 1.0
    grad = R.logpsi_param_grad(p, cfg, xs, ct)
    # rebuild x~^T dy per block from the taps
    sums = {}
    for b in range(4):
        pr = {k: v.clone() for k, v in p.items()}
        taps = {}

        def tap(name, x_in, y):
            eps = torch.zeros_like(y, requires_grad=True)
            taps[name] = (x_in.detach(), eps)
            return y + eps

        lp = R.logpsi(pr, cfg, xs[b], tap)
        gs = torch.autograd.grad(lp.real, [taps[n][1] for n in taps])
        for n, gy in zip(taps, gs):
            x = taps[n][0].reshape(taps[n][0].shape[0], -1)
            x = torch.cat([x, torch.ones(x.shape[0], 1, dtype=x.dtype)], 1)
            sums[n] = sums.get(n, 0.0) + x.T @ gy.reshape(gy.shape[0], -1)
    assert set(sums) == {blk.name for blk in bl}
    for blk in bl:
        s = sums[blk.name]
        gk = grad[blk.kernel].reshape(blk.din, blk.dout)
        assert torch.allclose(s[: blk.din], gk, atol=1e-10 * max(1.0, gk.abs().max().item()))
        if blk.bias:
            assert torch.allclose(s[blk.din], grad[blk.bias].reshape(-1), atol=1e-10)


def test_statistics_symmetric_psd_and_shards():
    cfg = _cfg()
    p = make_params(cfg)
    xs = torch.tensor(make_walkers(4, cfg.nelec, seed=3), dtype=torch.float64)
    full, diag = KF.batch_statistics(p, cfg, xs)
    halves, diag2 = KF.batch_statistics(p, cfg, xs, shards=2)
    for name, (A, G) in full.items():
        for F in (A, G):
            assert torch.allclose(F, F.T)
            assert torch.linalg.eigvalsh(F).min() > -1e-10 * max(1.0, F.abs().max().item())
        # dense factors are means over equal row counts: shard average == full batch
        assert torch.allclose(halves[name][0], A, atol=1e-12)
        assert torch.allclose(halves[name][1], G, atol=1e-12)
    assert set(diag) == set(diag2)
    # with a bias the last diagonal entry of A is the mean of 1
    for blk in KF.blocks(cfg)[0]:
        if blk.bias:
            assert abs(full[blk.name][0][-1, -1].item() - 1.0) < 1e-12


def test_damped_inverse_and_step():
    cfg = _cfg()
    p = make_params(cfg)
    xs = torch.tensor(make_walkers(4, cfg.nelec, seed=4), dtype=torch.float64)
    stats, diag = KF.batch_statistics(p, cfg, xs)
    A, G = next(iter(stats.values()))
    Ai, Gi, pi = KF.damped_inverses(A, G, 3.0)
    As = math.sqrt(3.0) * A
    assert torch.allclose(Ai @ (As + pi * math.sqrt(KF.DAMPING) * torch.eye(A.shape[0], dtype=A.dtype)),
                          torch.eye(A.shape[0], dtype=A.dtype), atol=1e-8)
    ct = torch.zeros(4, 2, dtype=torch.float64)
    ct[:, 0] = 0.3
    grads = R.logpsi_param_grad(p, cfg, xs, ct)
    st = KF.KfacState()
    new, st, info = KF.kfac_step(p, cfg, grads, st, stats, diag)
    assert st.weight == 1.0 and st.step == 1
    assert 0.0 < info["coef"] <= 1.0 and info["sq"] > 0
    # the norm constraint bounds the update: lr^2 c^2 <Pg, g> <= norm_constraint
    assert info["lr"] ** 2 * info["coef"] ** 2 * info["sq"] <= KF.NORM_CONSTRAINT * (1 + 1e-12)
    step = {k: (new[k] - p[k]) for k in info["pg"]}
    assert all(torch.isfinite(v).all() for v in step.values())
    # a second step with the same statistics: the EMA value is unchanged (weighted mean)
    st2 = KF.update_curvature(st, stats, diag)
    name = next(iter(stats))
    assert torch.allclose(st2.raw_A[name] / st2.weight, stats[name][0])
    assert np.isclose(st2.weight, 1.95)


def test_sparse_orbital_blocks():
    """"sparse" orbitals (blocks.py:52-62): the featured DenseGeneral blocks (8 N K outputs)
    and the complex lll_weight block (kfac.py:127-133, 175-181).  The taps see the layers the
    autograd gradient sees: featured blocks as in test_taps_reproduce_parameter_gradient; for
    lll_weight, sum over (walker, i, j, k) of Re x^T Re dy + Im x^T Im dy (the natural
    grouping: the 8-axis is the input) equals sqrt(2)^0 x the autograd gradient of the real
    kernel.  Its KFAC statistics use kfac_jax's literal regrouping (8 x 8 and M x M factors,
    scale 8 N^2); the lll bias is generic."""
    cfg = oracle_config("C1", orbital="sparse", num_layers=1)
    p = make_params(cfg)
    B = 3
    xs = torch.tensor(make_walkers(B, cfg.nelec, seed=4), dtype=torch.float64)
    bl, generic = KF.blocks(cfg)
    lll = [b for b in bl if b.lll]
    assert len(lll) == 1 and lll[0].din == 8 and lll[0].dout == int(round(cfg.flux)) + 1
    assert lll[0].scale == 8 * cfg.nelec**2 and "Orbitals_0/lll_weight/bias" in generic
    ct = torch.zeros(B, 2, dtype=torch.float64)
    ct[:, 0] = 1.0
    grad = R.logpsi_param_grad(p, cfg, xs, ct)
    sums = {}
    for b in range(B):
        taps = {}

        def tap(name, x_in, y):
            eps = torch.zeros_like(y, requires_grad=True)
            taps[name] = (x_in.detach(), eps)
            return y + eps

        lp = R.logpsi({k: v.clone() for k, v in p.items()}, cfg, xs[b], tap)
        gs = torch.autograd.grad(lp.real, [taps[n][1] for n in taps])
        for n, gy in zip(taps, gs):
            x = taps[n][0]
            if n.endswith("lll_weight"):
                xn = x.permute(0, 2, 3, 1).reshape(-1, 8)
                gn = gy.permute(0, 2, 3, 1).reshape(-1, gy.shape[1])
                s = xn.real.T @ gn.real + xn.imag.T @ gn.imag
            else:
                xx = torch.cat([x.reshape(x.shape[0], -1), torch.ones(x.shape[0], 1, dtype=x.dtype)], 1)
                s = xx.T @ gy.reshape(gy.shape[0], -1)
            sums[n] = sums.get(n, 0.0) + s
    assert set(sums) == {blk.name for blk in bl}
    for blk in bl:
        gk = grad[blk.kernel].reshape(blk.din, blk.dout)
        assert torch.allclose(sums[blk.name][: blk.din], gk, atol=1e-10 * max(1.0, gk.abs().max().item())), blk.name
        if blk.bias:
            assert torch.allclose(sums[blk.name][blk.din], grad[blk.bias].reshape(-1), atol=1e-10)
    stats, diag = KF.batch_statistics(p, cfg, xs)
    A, G = stats["Orbitals_0/lll_weight"]
    assert A.shape == (8, 8) and G.shape == (lll[0].dout, lll[0].dout)
    for F in (A, G):
        assert torch.allclose(F, F.T) and torch.linalg.eigvalsh(F).min() > -1e-12 * F.abs().max().item()
    assert diag["Orbitals_0/lll_weight/bias"].shape == (lll[0].dout,)
    # one step through the restated update: every parameter moves, finitely
    state = KF.KfacState()
    new, state, info = KF.kfac_step(p, cfg, grad, state, stats, diag)
    assert all(torch.isfinite(new[k]).all() for k in new) and 0 < info["coef"] <= 1.0
