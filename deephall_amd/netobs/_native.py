"""Thin wrappers of the NetObs kernels (csrc/netobs.hip).  No CPU path: the library must load."""

from __future__ import annotations

import torch

from .. import _lib
from ..networks.psiformer import _ptr, _stream


def _check_cuda(t: torch.Tensor) -> torch.Tensor:
    if not t.is_cuda:
        raise RuntimeError("NetObs estimators run on the GPU (HIP kernels); got a CPU tensor")
    return t.contiguous().float()


def histograms(x: torch.Tensor, density_bins: int = 0, pair_bins: int = 0):
    """Unnormalised theta histogram and 1/sin-weighted pair-angle histogram of walkers x[B, N, 2]."""
    x = _check_cuda(x)
    B, N, _ = x.shape
    dens = torch.zeros(max(density_bins, 1), dtype=torch.float32, device=x.device)
    pair = torch.zeros(max(pair_bins, 1), dtype=torch.float32, device=x.device)
    lib = _lib.load()
    _lib.check(lib.dh_histograms(_ptr(x), B, N, density_bins, pair_bins, _ptr(dens), _ptr(pair), _stream(x.device)))
    return dens[:density_bins], pair[:pair_bins]


def monopole_orbitals(points: torch.Tensor, flux: int) -> torch.Tensor:
    """Y_{Q,Q,m}(points), m = -Q..Q: complex64 [..., flux + 1] (one_rdm.py:31-54)."""
    pts = _check_cuda(points)
    shape = pts.shape[:-1]
    flat = pts.reshape(-1, 2)
    out = torch.empty(flat.shape[0], flux + 1, 2, dtype=torch.float32, device=pts.device)
    lib = _lib.load()
    _lib.check(lib.dh_monopole_orbitals(_ptr(flat), flat.shape[0], int(flux), _ptr(out), _stream(pts.device)))
    return torch.view_as_complex(out).reshape(*shape, flux + 1)
