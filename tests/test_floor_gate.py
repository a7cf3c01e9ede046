"""The f32-floor gate itself (helpers.within_f32_floor, used by the GPU parity suites): its
three ratio criteria, the absolute floor and the near-pole max override."""

from __future__ import annotations

import numpy as np

from helpers import FLOOR_X_MAX, within_f32_floor


def _errs(scale_max):
    f = np.full(32, 1e-5)
    f[-1] = 1e-4  # the float32 run's worst walker
    e = f.copy()
    e[-1] = scale_max * 1e-4
    return e, f


def test_max_criterion_and_override():
    e, f = _errs(0.9 * FLOOR_X_MAX)
    assert within_f32_floor(e, f)
    e, f = _errs(1.1 * FLOOR_X_MAX)
    assert not within_f32_floor(e, f)
    assert within_f32_floor(e, f, 0.0, 1.2 * FLOOR_X_MAX)  # an explicit per-call allowance
    e, f = _errs(1.3 * FLOOR_X_MAX)
    assert not within_f32_floor(e, f, 0.0, 1.2 * FLOOR_X_MAX)


def test_median_and_p90_criteria():
    f = np.full(32, 1e-5)
    assert not within_f32_floor(f * 1.6, f)  # median beyond 1.5x
    e = f.copy()
    e[-4:] = 2.5e-5  # the 90th percentile at 2.5x, the median unchanged
    assert not within_f32_floor(e, f)
    assert within_f32_floor(f * 1.4, f)


def test_absolute_floor_passes_outright():
    f = np.full(32, 1e-9)
    e = np.full(32, 5e-6)  # 5000x the float32 run, but every walker within 1e-5
    assert within_f32_floor(e, f, 1e-5)
    assert not within_f32_floor(e, f)
