"""TEST INFRASTRUCTURE ONLY — float64 numpy restatement of the NetObs estimators.

Follows deephall/netobs_bridge/observables/*.py in behaviour (not in code):

* density    density.py:38-44   histogram of theta, range (0, pi), numpy's bin rule
* pair_corr  pair_corr.py:43-58 pair angles over i < j, weight 1 / sin, times
                                4 bins / (B N^2 pi)
* orbitals   one_rdm.py:31-54   Y_{q,l,m} with the general sum over s (the kernel uses the
                                l = q collapse), cos theta clipped to +-(1 - 1e-4)
* one_rdm    one_rdm.py:81-99   4 pi sum_a psi(R_a') / psi(R) Y_i(r_a) conj(Y_j(r')),
                                one r' per walker
* overlap    overlap.py:55-70   ratio = exp(log phi - log psi - mean), |mean|^2 / mean |.|^2

Only tests/ may import this module.
"""

from __future__ import annotations

import numpy as np
from scipy import special as ss


def density_hist(x: np.ndarray, bins: int = 50) -> np.ndarray:
    theta = np.asarray(x, dtype=np.float64)[..., 0].reshape(-1)
    return np.histogram(theta, bins, (0.0, np.pi))[0].astype(np.float64)


def pair_angles(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.float64)
    th, ph = x[..., 0], x[..., 1]
    xyz = np.stack([np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)], -1)
    cos12 = np.einsum("bid,bjd->bij", xyz, xyz)
    iu = np.triu_indices(x.shape[1], 1)
    return np.arccos(cos12[:, iu[0], iu[1]].reshape(-1))


def pair_corr(x: np.ndarray, bins: int = 200) -> np.ndarray:
    B, N, _ = x.shape
    t = pair_angles(x)
    h = np.histogram(t, bins, (0.0, np.pi), weights=1.0 / np.sin(t))[0]
    return h * 4 * bins / B / N**2 / np.pi


def monopole_harm(q: float, l: float, m: float, pts: np.ndarray) -> np.ndarray:  # noqa: E741
    """one_rdm.py:31-51 (general q, l, m)."""
    norm = np.sqrt(((2 * l + 1) / (4 * np.pi)) * (ss.factorial(l - m) * ss.factorial(l + m))
                   / (ss.factorial(l - q) * ss.factorial(l + q)))
    s = np.arange(int(round(l - m)) + 1)
    fac = (-1.0) ** (l - m - s) * ss.comb(l - q, s) * ss.comb(l + q, l - m - s)
    th, ph = pts[..., 0], pts[..., 1]
    x = np.clip(np.cos(th), -1 + 1e-4, 1 - 1e-4)
    part = np.sum(fac * (1 - x[..., None]) ** (l - s - (m + q) / 2) * (1 + x[..., None]) ** (s + (m + q) / 2), -1)
    return norm / 2**l * part * np.exp(1j * m * ph)


def lll_orbitals(pts: np.ndarray, flux: int) -> np.ndarray:
    Q = flux / 2
    pts = np.asarray(pts, dtype=np.float64)
    return np.stack([monopole_harm(Q, Q, m, pts) for m in np.arange(-Q, Q + 1)], -1)


def one_rdm_product(x, r_prime, logpsi, logpsi_prime, flux) -> np.ndarray:
    """Per-walker [B, norb, norb] from given log-amplitudes (logpsi [B], logpsi_prime [B, N])."""
    ratio = np.exp(np.asarray(logpsi_prime) - np.asarray(logpsi)[:, None])
    phi = lll_orbitals(x, flux)          # [B, N, norb]
    phip = lll_orbitals(r_prime, flux)   # [B, norb]
    return 4 * np.pi * np.einsum("ba,bai,bj->bij", ratio, phi, np.conj(phip))


def overlap_ratio(logpsi, logphi):
    d = np.asarray(logphi) - np.asarray(logpsi)
    r = np.exp(d - d.mean())
    return r, np.abs(r) ** 2


def overlap_digest(ratio_steps, ratio_square_steps) -> float:
    return float(np.abs(np.nanmean(ratio_steps)) ** 2 / np.nanmean(ratio_square_steps))
