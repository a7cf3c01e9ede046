"""NetObs bridge (deephall/netobs_bridge/*) on the native kernels.

The reference plugs DeepHall into the third-party NetObs framework (``netobs``, absent
here): an adaptor that restores a checkpoint and exposes the network, the MCMC walk and the
energies (adaptor.py:36-115), a ``HallSystem`` (hall_system.py), and four estimators
(observables/density.py, pair_corr.py, overlap.py, one_rdm.py).  This package mirrors them
with the same names, options, value/state keys and digests:

* histograms (density, pair correlation) and the lowest-Landau-level monopole harmonics of
  the one-body density matrix are HIP kernels (csrc/netobs.hip, ``dh_histograms``,
  ``dh_monopole_orbitals``);
* every wavefunction value goes through ``dh_logpsi`` (Psiformer or the native Laughlin
  state), the walk through ``dh_mcmc_step``;
* ``evaluate`` is a minimal stand-in for NetObs's own evaluation loop (restore, burn-in,
  walk + evaluate per step, digest), which cannot be pinned here (the package is absent):
  per step it stores the walker mean of each value, as the estimators' ``empty_val_state``
  shapes (steps, *observable shape) imply.
"""

from .adaptor import DeepHallAdaptor, DeepHallAuxData
from .estimator import Estimator, Observable, evaluate
from .hall_system import HallSystem
from .observables import density, one_rdm, overlap, pair_corr

ESTIMATORS = {
    "density": density.DEFAULT,
    "pair_corr": pair_corr.DEFAULT,
    "overlap": overlap.DEFAULT,
    "one_rdm": one_rdm.DEFAULT,
}

__all__ = ["DeepHallAdaptor", "DeepHallAuxData", "Estimator", "Observable", "HallSystem", "evaluate", "ESTIMATORS"]
