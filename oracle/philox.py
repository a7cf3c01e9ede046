"""TEST INFRASTRUCTURE ONLY — numpy Philox4x32-10, bit-exact mirror of the device RNG.

Published algorithm: Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy
as 1, 2, 3" (SC'11), Random123 philox4x32 with 10 rounds; known-answer vectors
from Random123's kat_vectors are checked in tests/test_oracle_philox.py.
The counter layout and float transforms are those of
deephall_amd/csrc/device_common.h (dh_random, u01, u01_open0, box_muller).
The reference itself uses jax.random threefry (mcmc.py:53,69-72), which cannot be
reproduced here; MCMC parity is checked with injected noise instead.
"""

from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr, key):
    """ctr: uint32 array [..., 4]; key: uint32 array [..., 2] (broadcastable). Returns uint32 [..., 4]."""
    c = np.array(ctr, dtype=np.uint32)
    k = np.array(key, dtype=np.uint32)
    c0, c1, c2, c3 = (c[..., i].astype(np.uint64) for i in range(4))
    k0 = np.broadcast_to(k[..., 0], c0.shape).astype(np.uint32)
    k1 = np.broadcast_to(k[..., 1], c0.shape).astype(np.uint32)
    with np.errstate(over="ignore"):
        for r in range(10):
            if r:
                k0 = (k0 + W0).astype(np.uint32)
                k1 = (k1 + W1).astype(np.uint32)
            p0 = M0 * c0
            p1 = M1 * c2
            hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
            hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
            c0, c1, c2, c3 = (
                hi1 ^ c1 ^ k0.astype(np.uint64),
                lo1,
                hi0 ^ c3 ^ k1.astype(np.uint64),
                lo0,
            )
    return np.stack([c0, c1, c2, c3], -1).astype(np.uint32)


def dh_random(seed, purpose, lane, walker, step):
    """Counter layout of device_common.h dh_random (arrays broadcast)."""
    lane = np.asarray(lane, dtype=np.uint64)
    walker = np.asarray(walker, dtype=np.uint64)
    step = np.asarray(step, dtype=np.uint64)
    shape = np.broadcast_shapes(lane.shape, walker.shape, step.shape)
    ctr = np.empty(shape + (4,), dtype=np.uint32)
    ctr[..., 0] = (np.broadcast_to(lane, shape) | (np.uint64(purpose) << np.uint64(24))) & MASK
    ctr[..., 1] = np.broadcast_to(walker, shape) & MASK
    ctr[..., 2] = np.broadcast_to(step, shape) & MASK
    ctr[..., 3] = np.broadcast_to(step, shape) >> np.uint64(32)
    seed = int(seed)
    key = np.array([seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF], dtype=np.uint32)
    return philox4x32_10(ctr, key)


def u01(b):
    return (np.asarray(b, dtype=np.uint32) >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def u01_open0(b):
    return ((np.asarray(b, dtype=np.uint32) >> np.uint32(8)) + np.uint32(1)).astype(np.float32) * np.float32(
        1.0 / 16777216.0
    )


def box_muller(b0, b1):
    u1 = u01_open0(b0).astype(np.float64)
    u2 = u01(b1).astype(np.float64)
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def mcmc_noise(seed, step, walkers, N):
    """The noise the device draws for one MH step: (normals [B,N], phi uniforms [B,N], accept [B])."""
    walkers = np.asarray(walkers, dtype=np.uint64)
    lanes = np.arange(N, dtype=np.uint64)
    r = dh_random(seed, 0, lanes[None, :], walkers[:, None], step)
    normals = box_muller(r[..., 0], r[..., 1])
    uph = u01(r[..., 2])
    ra = dh_random(seed, 0, np.uint64(N), walkers, step)
    return normals, uph, u01(ra[..., 0])


def init_uniforms(seed, walkers, N):
    """init_guess draws (purpose 1): (u1, u2) each [B,N] in [0,1)."""
    walkers = np.asarray(walkers, dtype=np.uint64)
    lanes = np.arange(N, dtype=np.uint64)
    r = dh_random(seed, 1, lanes[None, :], walkers[:, None], 0)
    return u01(r[..., 0]), u01(r[..., 1])
