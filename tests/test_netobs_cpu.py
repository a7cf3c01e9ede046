"""NetObs estimator oracle pinned by analytic properties — CPU only.

* the kernel's collapsed LLL harmonic (l = q: only the s = 0 term, c_m = (-1)^(Q-m) 2^-Q
  sqrt((2Q+1)/4pi) sqrt(binom(2Q, Q-m))) equals one_rdm.py's general sum;
* the LLL harmonics are orthonormal on the sphere (the 1-RDM basis, one_rdm.py:27-29);
* independent uniform points give a flat pair correlation (N - 1) / N per bin
  (pair_corr.py:57's normalisation);
* the estimator modules load without a GPU and expose the reference's option defaults.
"""

from __future__ import annotations

import math

import numpy as np
import pytest
from scipy import special as ss

from oracle import netobs as O


def collapsed(pts, flux):
    Q = flux / 2
    th, ph = pts[..., 0], pts[..., 1]
    x = np.clip(np.cos(th), -1 + 1e-4, 1 - 1e-4)
    out = []
    for k in range(flux + 1):
        m = -Q + k
        c = (-1.0) ** (flux - k) * 2.0**-Q * math.sqrt((2 * Q + 1) / (4 * math.pi)) * math.sqrt(ss.comb(flux, flux - k))
        out.append(c * (1 - x) ** ((Q - m) / 2) * (1 + x) ** ((Q + m) / 2) * np.exp(1j * m * ph))
    return np.stack(out, -1)


@pytest.mark.parametrize("flux", [2, 5, 15, 23])
def test_collapsed_harmonic_equals_general_sum(flux):
    rng = np.random.default_rng(flux)
    pts = np.stack([np.arccos(rng.uniform(-1, 1, 64)), rng.uniform(-np.pi, np.pi, 64)], -1)
    a, b = O.lll_orbitals(pts, flux), collapsed(pts, flux)
    assert np.max(np.abs(a - b)) < 1e-10 * max(1.0, np.max(np.abs(a)))


@pytest.mark.parametrize("flux", [2, 6, 15])
def test_lll_harmonics_orthonormal(flux):
    # Gauss-Legendre in cos theta x uniform phi: exact for these polynomials in u, v
    n = flux + 8
    xg, wg = np.polynomial.legendre.leggauss(n)
    nph = 2 * flux + 4
    ph = np.linspace(-np.pi, np.pi, nph, endpoint=False)
    T, P = np.meshgrid(np.arccos(xg), ph, indexing="ij")
    W = np.repeat(wg[:, None], nph, 1) * (2 * np.pi / nph)
    Y = O.lll_orbitals(np.stack([T, P], -1), flux)  # [n, nph, norb]
    G = np.einsum("tp,tpi,tpj->ij", W, np.conj(Y), Y)
    # the clip of cos theta to +-(1 - 1e-4) perturbs the pole values slightly
    assert np.max(np.abs(G - np.eye(flux + 1))) < 5e-3


def test_uniform_points_flat_pair_correlation():
    rng = np.random.default_rng(0)
    B, N, bins = 20000, 6, 20
    x = np.stack([np.arccos(rng.uniform(-1, 1, (B, N))), rng.uniform(-np.pi, np.pi, (B, N))], -1)
    g = O.pair_corr(x, bins)
    # the 1/sin weight makes the end bins heavy-tailed: the interior and the mean are tight
    assert np.allclose(g[2:-2], (N - 1) / N, rtol=0.04) and abs(g.mean() / ((N - 1) / N) - 1) < 0.02
    d = O.density_hist(x, bins)
    want = B * N * (np.cos(np.linspace(0, np.pi, bins + 1)[:-1]) - np.cos(np.linspace(0, np.pi, bins + 1)[1:])) / 2
    assert np.allclose(d, want, rtol=0.05)


def test_estimator_defaults_without_gpu():
    from deephall_amd.netobs import ESTIMATORS, HallSystem
    from deephall_amd.netobs.observables import density, one_rdm, pair_corr

    sys_ = HallSystem(spins=[3, 0], flux=2)
    assert one_rdm.OneRDM(sys_).shape == (3, 3)
    assert density.DensityEstimator(None, sys_, {}, {}).hist_bins == 50
    assert pair_corr.PairCorrelationEstimator(None, sys_, {}, {}).bins == 200
    assert set(ESTIMATORS) == {"density", "pair_corr", "overlap", "one_rdm"}
