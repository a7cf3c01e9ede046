"""Rank process of tests/test_gpu_0_multirank.py (not a test module).

One VMC iteration's device work on this rank's contiguous walker shard — mcmc_step with
its pmove pmean, the local energy, dh_energy_stats and the packed statistics all-reduce —
with every rank on device 0 and the gloo backend (a one-GPU box; the 8-GPU runs use RCCL).
Writes the rank's walkers, accept counts and the reduced statistics to argv[1]_<rank>.npz.
"""

from __future__ import annotations

import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out = sys.argv[1]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(0)
    if world > 1:
        dist.init_process_group("gloo")
    from deephall_amd import config, make_network
    from deephall_amd.hamiltonian import _run_local_energy
    from deephall_amd.loss import device_stats, reduce_stats
    from deephall_amd.mcmc import make_mcmc_step
    from deephall_amd.random import Key
    from helpers import make_params, make_walkers, oracle_config, to_device_params

    ocfg = oracle_config("C2")
    system = config.System(nspins=ocfg.nspins, flux=ocfg.flux)
    model = make_network(system, config.Network())
    params = to_device_params(make_params(ocfg))
    B = 64
    per = B // world
    xs = make_walkers(B, ocfg.nelec, seed=3)[rank * per : (rank + 1) * per]
    x = torch.tensor(xs, device="cuda")
    step = make_mcmc_step(model, batch_per_device=per, steps=4)
    x, pmove = step(params, x, Key(77, 5), 0.15)  # walker_offset = rank * per, pmean of pmove
    nacc = step.last_n_accept
    e_l, obs = _run_local_energy(model, params, x)
    stats = reduce_stats(device_stats(model, e_l, obs, nacc, 4))
    torch.cuda.synchronize()
    np.savez(f"{out}_{rank}.npz", x=x.cpu().numpy(), n_acc=nacc.cpu().numpy(), mcmc_pmove=float(pmove),
             e_l=e_l.cpu().numpy(), **{k: complex(v.item()) for k, v in stats.items()})
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
