"""density.py:26-51: histogram of every electron's polar angle over [0, pi] (state "map")."""

from __future__ import annotations

import torch

from .._native import histograms
from ..estimator import Estimator, Observable


class Density(Observable):
    def shapeof(self, system) -> tuple[int, ...]:
        return ()


class DensityEstimator(Estimator):
    observable_type = Density

    def __init__(self, adaptor, system, estimator_options, observable_options):
        super().__init__(adaptor, system, estimator_options, observable_options)
        self.hist_bins = self.options.get("bins", 50)

    def empty_val_state(self, steps: int):
        del steps
        return {}, {"map": None}

    def evaluate(self, i, params, key, data, system, state, aux_data):
        del i, params, system, aux_data, key
        x = data.reshape(-1, *data.shape[-2:])
        counts, _ = histograms(x, density_bins=self.hist_bins)
        state["map"] = counts if state["map"] is None else state["map"] + counts
        return {}, state

    def digest(self, all_values, state):
        del all_values, state
        return {}


DEFAULT = DensityEstimator  # Useful in CLI
