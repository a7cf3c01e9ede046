"""overlap.py:24-70: overlap |<Laughlin|psi>|^2 from the ratio phi_L / psi on psi's walkers.

Both log-amplitudes are native (``dh_logpsi`` of the network and of the Laughlin state of
the same system); ratio = exp(log phi - log psi - shift), shift = the walker mean of
log phi - log psi; digest: |nanmean(ratio)|^2 / nanmean(|ratio|^2) over the steps.
"""

from __future__ import annotations

import dataclasses

import torch

from ...config import NetworkType
from ...networks import make_network
from ..estimator import Estimator, Observable


class Overlap(Observable):
    def shapeof(self, system) -> tuple[int, ...]:
        return ()


class OverlapEstimator(Estimator):
    observable_type = Overlap

    def __init__(self, adaptor, system, estimator_options, observable_options):
        super().__init__(adaptor, system, estimator_options, observable_options)
        cfg = adaptor.cfg
        self.laughlin = make_network(cfg.system, dataclasses.replace(cfg.network, type=NetworkType.laughlin))

    def empty_val_state(self, steps: int):
        return {"ratio": torch.zeros(steps, dtype=torch.complex64), "ratio_square": torch.zeros(steps)}, {}

    def evaluate(self, i, params, key, data, system, state, aux_data):
        del i, aux_data, key, system
        x = data.reshape(-1, *data.shape[-2:])
        logpsi = self.adaptor.call_network(params, x)
        logphi = self.laughlin.apply({}, x)
        d = logphi - logpsi
        shift = d.mean()
        ratio = torch.exp(d - shift)
        return {"ratio": ratio.cpu(), "ratio_square": (ratio.abs() ** 2).cpu()}, state

    def digest(self, all_values, state):
        del state
        ratio = all_values["ratio"]
        ok = ~(torch.isnan(ratio.real) | torch.isnan(ratio.imag))
        overlap = ratio[ok].mean().abs() ** 2 / torch.nanmean(all_values["ratio_square"])
        return {"overlap": overlap}


DEFAULT = OverlapEstimator  # Useful in CLI
