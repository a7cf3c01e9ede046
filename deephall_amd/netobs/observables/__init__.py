"""Estimators of netobs_bridge/observables/*.py (the ``deephall@`` names of cli_extend.py)."""

from . import density, one_rdm, overlap, pair_corr

__all__ = ["density", "one_rdm", "overlap", "pair_corr"]
