"""Counter-based RNG keys for the MCMC kernels.

The reference threads a ``jax.random`` key through every call and splits it
(mcmc.py:53,69; train.py:102-139), with a different key per device
(train.py:89).  Threefry streams cannot be reproduced here, so the MI355X path
uses Philox4x32-10 with key = seed and counter = (electron, global walker id,
MCMC step) — see deephall_amd/csrc/device_common.h and oracle/philox.py.  A
``Key`` is (seed, counter); every Metropolis step consumes one counter value, so
two calls with the same key draw the same numbers (like reusing a jax key) and
the numbers drawn for a walker do not depend on the number of GPUs.
"""

from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Key:
    seed: int
    counter: int = 0

    def advance(self, n: int) -> "Key":
        return Key(self.seed, self.counter + int(n))


def PRNGKey(seed: int) -> Key:  # noqa: N802 (mirrors jax.random.PRNGKey)
    return Key(int(seed) & 0xFFFFFFFFFFFFFFFF, 0)
