"""Philox4x32-10 oracle against Random123 known-answer vectors (CPU)."""

import numpy as np

from oracle import philox


def test_random123_kat():
    kat = [
        ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
        ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
        (
            [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
            [0xA4093822, 0x299F31D0],
            [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1],
        ),
    ]
    for ctr, key, want in kat:
        got = philox.philox4x32_10(np.array(ctr, np.uint32), np.array(key, np.uint32))
        assert [int(v) for v in got] == want


def test_counter_layout_and_streams_independent_of_sharding():
    # the noise of global walker g never depends on which rank draws it
    n_all, u_all, a_all = philox.mcmc_noise(123, 5, np.arange(64), 6)
    n_lo, u_lo, a_lo = philox.mcmc_noise(123, 5, np.arange(32), 6)
    n_hi, u_hi, a_hi = philox.mcmc_noise(123, 5, np.arange(32, 64), 6)
    assert np.array_equal(n_all, np.concatenate([n_lo, n_hi]))
    assert np.array_equal(a_all, np.concatenate([a_lo, a_hi]))
    # different steps / purposes give different streams
    n2, _, _ = philox.mcmc_noise(123, 6, np.arange(64), 6)
    assert not np.allclose(n_all, n2)


def test_distributions():
    n, u, a = philox.mcmc_noise(9, 0, np.arange(20000), 4)
    assert abs(n.mean()) < 0.02 and abs(n.std() - 1) < 0.02
    assert 0.0 <= u.min() and u.max() < 1.0 and abs(u.mean() - 0.5) < 0.01
    assert abs(a.mean() - 0.5) < 0.01
