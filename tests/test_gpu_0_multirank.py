"""Multi-rank path on the GPU box: N fresh rank processes started by a
parent that has not initialised the GPU (this module runs first among the GPU tests and
uses no `cuda` fixture), one contiguous walker shard each.  Walker trajectories and
accept counts are bit-identical to one rank holding every walker (the device RNG is
keyed by global walker index), and the packed statistics all-reduce gives the
single-rank statistics to f32 rounding.  All ranks share device 0 with gloo here; the
driver's 8-GPU runs use RCCL.  Also: ``bench.py --gpus 2`` launches its own ranks.
"""

from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _gpu_or_skip():
    if torch.cuda.device_count() < 1:  # counts devices without initialising HIP
        pytest.skip("no GPU")
    if torch.cuda.is_initialized():
        pytest.skip("this process already initialised the GPU: rank processes must come from a clean parent")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(world, out):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(ROOT / "tests" / "multirank_worker.py"), str(out)], env=env))
    rcs = [p.wait(timeout=240) for p in procs]
    assert rcs == [0] * world
    return [dict(np.load(f"{out}_{r}.npz")) for r in range(world)]


def test_two_ranks_match_one_rank(tmp_path):
    _gpu_or_skip()
    one = _run_ranks(1, tmp_path / "w1")[0]
    two = _run_ranks(2, tmp_path / "w2")
    assert np.array_equal(np.concatenate([t["x"] for t in two]), one["x"])
    assert np.array_equal(np.concatenate([t["n_acc"] for t in two]), one["n_acc"])
    assert np.array_equal(np.concatenate([t["e_l"] for t in two]), one["e_l"])
    for k in ("energy", "kinetic", "potential", "angular_momentum_z", "angular_momentum_square", "pmove"):
        a, b = complex(two[0][k]), complex(one[k])
        assert complex(two[1][k]) == a  # every rank holds the same reduced value
        assert abs(a - b) <= 2e-6 * max(1.0, abs(b)), k
    assert float(two[0]["mcmc_pmove"]) == pytest.approx(float(one["mcmc_pmove"]), abs=1e-7)


def test_bench_launches_its_own_ranks():
    _gpu_or_skip()
    env = dict(os.environ, DH_BENCH_ONE_GPU="1", DH_BENCH_BACKEND="gloo")
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                          "--burn-in", "0", "--batch", "256", "--mcmc-calls", "2", "--no-cpu-baseline",
                          "--no-kernel-events"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 512 and line["value"] > 0
