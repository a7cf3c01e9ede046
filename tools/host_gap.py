"""Host time of the pieces between a VMC step's closing host sync and its next launch.

bench.py's loop reads pmove at the end of every step (a device sync); the GPU then idles
until the host has issued the next step's first kernel.  This times each host piece of
that window on an idle GPU (mean of 50 calls, microseconds).  Usage: python tools/host_gap.py
"""

import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from deephall_amd import config  # noqa: E402
from deephall_amd.loss import device_stats, reduce_stats  # noqa: E402
from deephall_amd.mcmc import make_mcmc_step, update_mcmc_width  # noqa: E402
from deephall_amd.networks import make_network  # noqa: E402
from deephall_amd.random import Key, PRNGKey  # noqa: E402
from deephall_amd.train import init_guess, make_vmc_iteration  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = make_network(config.System(nspins=(6, 0), flux=15), config.Network())
    B = 4096
    params = model.init(PRNGKey(42), device=dev)
    data = init_guess(Key(4242), B, 6, dev, network=model)
    it = make_vmc_iteration(model, B, 10, 1)
    key = PRNGKey(7)
    pm = np.zeros(100)
    data, e, o, n = it(params, data, key, 0.1)
    st = reduce_stats(device_stats(model, e, o, n, 10))
    torch.cuda.synchronize()
    res = {}

    def t(name, fn, reps=50):
        out = None
        a = time.perf_counter()
        for _ in range(reps):
            out = fn()
        torch.cuda.synchronize()
        res[name] = (time.perf_counter() - a) / reps * 1e6
        return out

    t("item(pmove) on an idle GPU", lambda: float(st["pmove"].item()))
    t("update_mcmc_width", lambda: update_mcmc_width(1, 0.1, 100, st["pmove"], pm))
    t("key.advance", lambda: key.advance(10))
    t("model.prepare", lambda: model.prepare(params, dev))
    t("torch.empty x2", lambda: (torch.empty(B, device=dev), torch.empty(B, dtype=torch.int32, device=dev)))
    t("torch.cuda.current_stream", lambda: torch.cuda.current_stream(dev))
    step = make_mcmc_step(model, batch_per_device=B, steps=0)  # initial log psi pass only
    t("mcmc_step(steps=0): prepare + checks + 1 value pass launch", lambda: step(params, data, key, 0.1, reduce=False),
      reps=20)
    # one empty launch sequence: sync, then time to the first kernel's completion
    x = torch.zeros(1, device=dev)
    t("tiny torch op + sync (launch latency)", lambda: (x.add_(1), torch.cuda.synchronize()))
    for k, v in res.items():
        print(f"{v:9.1f} us  {k}")


if __name__ == "__main__":
    main()
