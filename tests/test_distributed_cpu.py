"""Multi-rank logic on CPU with gloo (world_size 2): the single packed all-reduce
of the per-device statistics reproduces the reference's per-statistic pmeans
(loss.py:68-91, mcmc.py:147), and walker sharding does not change the random
numbers a walker sees."""

from __future__ import annotations

import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deephall_amd import constants
from deephall_amd.loss import reduce_stats


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        assert constants.world_size() == world and constants.rank() == rank
        local = torch.arange(16, dtype=torch.float32) * (rank + 1)
        st = reduce_stats(local)
        x = constants.pmean(torch.tensor([float(rank)]))
        q.put((rank, {k: complex(v.item()) for k, v in st.items()}, float(x)))
    finally:
        dist.destroy_process_group()


def test_packed_pmean_two_ranks():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    locals_ = [np.arange(16, dtype=np.float64) * (r + 1) for r in range(world)]
    g = np.mean(locals_, 0)
    for rank, st, x in res:
        assert x == 0.5
        assert np.isclose(st["energy"], g[0] + 1j * g[1])
        assert np.isclose(st["clipped_energy"], g[2] + 1j * g[3])
        assert np.isclose(st["variance"].real, g[4] - g[0] ** 2)  # pmean(E[Re^2]) - Re(energy)^2
        assert np.isclose(st["kinetic"], g[5] + 1j * g[6])
        assert np.isclose(st["angular_momentum_square"].real, g[10])
        assert np.isclose(st["pmove"].real, g[11])


def test_single_process_pmean_is_identity():
    t = torch.tensor([1.0, 2.0])
    assert torch.equal(constants.pmean(t), t)
