"""pair_corr.py:23-67: pair-angle histogram with weight 1 / sin theta_12 (state "pair_corr")."""

from __future__ import annotations

import math

from .._native import histograms
from ..estimator import Estimator, Observable


class PairCorrelation(Observable):
    def shapeof(self, system) -> tuple[int, ...]:
        return ()


class PairCorrelationEstimator(Estimator):
    observable_type = PairCorrelation

    def __init__(self, adaptor, system, estimator_options, observable_options):
        super().__init__(adaptor, system, estimator_options, observable_options)
        self.bins = self.options.get("bins", 200)

    def empty_val_state(self, steps: int):
        del steps
        return {}, {"pair_corr": None}

    def evaluate(self, i, params, key, data, system, state, aux_data):
        del i, params, aux_data, key, system
        x = data.reshape(-1, *data.shape[-2:])
        batch_size, nelec, _ = x.shape
        _, to_add = histograms(x, pair_bins=self.bins)
        # pair_corr.py:55-57: the evaluation-step norm is left to the caller; the 2 of
        # (i != j) -> (i < j) is in the 4
        to_add = to_add * (4 * self.bins / batch_size / nelec**2 / math.pi)
        state["pair_corr"] = to_add if state["pair_corr"] is None else state["pair_corr"] + to_add
        return {}, state

    def digest(self, all_values, state):
        del all_values, state
        return {}


DEFAULT = PairCorrelationEstimator  # Useful in CLI
