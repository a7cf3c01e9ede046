"""one_rdm.py:25-119: one-body density matrix in the lowest-Landau-level basis Y_{Q,Q,m}.

Per walker R one uniform point r' on the sphere (uniform_sample, one_rdm.py:56-60 — one
point per walker: the [:, :, None, :] of one_rdm.py:110 gives each walker a single r'),
and for every electron a the configuration R_a' with r_a replaced by r':
    rho_ij = 4 pi < sum_a psi(R_a') / psi(R) Y_i(r_a) conj(Y_j(r')) >     (one_rdm.py:90-99)
The N displaced configurations of every walker go through one batched ``dh_logpsi`` call;
Y is the ``dh_monopole_orbitals`` kernel; the walker sum is one (norb x B) (B x norb) product.
"""

from __future__ import annotations

import math

import torch

from ...train import init_guess
from .._native import monopole_orbitals
from ..estimator import Estimator, Observable


class OneRDM(Observable):
    def shapeof(self, system) -> tuple[int, ...]:
        norbs = system["flux"] + 1
        return (norbs, norbs)


class OneRDMEstimator(Estimator):
    observable_type = OneRDM

    def __init__(self, adaptor, system, estimator_options, observable_options):
        super().__init__(adaptor, system, estimator_options, observable_options)
        self.flux = int(system["flux"])

    def empty_val_state(self, steps: int):
        dtype = getattr(torch, self.options.get("dtype", "complex64"))
        return {"one_rdm": torch.zeros((steps, *self.observable.shape), dtype=dtype)}, {}

    def product(self, params, x: torch.Tensor, r_prime: torch.Tensor) -> torch.Tensor:
        """Per-walker estimator [B, norb, norb] (one_rdm.py:81-99), r_prime [B, 2]."""
        B, N, _ = x.shape
        logpsi = self.adaptor.call_network(params, x)                            # [B]
        xp = x.unsqueeze(1).repeat(1, N, 1, 1)                                   # [B, a, N, 2]
        idx = torch.arange(N, device=x.device)
        xp[:, idx, idx, :] = r_prime[:, None, :]
        logpsi_p = self.adaptor.call_network(params, xp.reshape(B * N, N, 2)).reshape(B, N)
        ratio = torch.exp(logpsi_p - logpsi[:, None])                            # [B, a]
        phi = monopole_orbitals(x, self.flux)                                    # [B, a, norb]
        phip = monopole_orbitals(r_prime, self.flux)                             # [B, norb]
        u = (ratio[..., None] * phi).sum(dim=1)                                  # [B, norb]
        return (4 * math.pi) * u[:, :, None] * phip.conj()[:, None, :]

    def evaluate(self, i, params, key, data, system, state, aux_data):
        del i, aux_data, system
        x = data.reshape(-1, *data.shape[-2:])
        r_prime = init_guess(key, x.shape[0], 1, x.device, network=self.adaptor.model)[:, 0, :]
        return {"one_rdm": self.product(params, x, r_prime).cpu()}, state

    def digest(self, all_values, state):
        del state
        one_rdm = all_values["one_rdm"].mean(dim=0)
        return {"diagonal": torch.diagonal(one_rdm), "trace": torch.trace(one_rdm)}


DEFAULT = OneRDMEstimator  # Useful in CLI
