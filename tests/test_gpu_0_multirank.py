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


def _run_ranks(world, out, *args):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(ROOT / "tests" / "multirank_worker.py"), str(out),
                                       *map(str, args)], env=env))
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


def test_gradient_allreduce_two_ranks(tmp_path):
    """loss.py:66-108 across ranks: the statistics all-reduce, the
    clipped difference with the global clipped mean and the gradient pmean.  64 walkers of
    C2 with random-init parameters, none clipped (IQR x 100), equal shards: the mean of the
    two ranks' gradients equals one rank's gradient over all walkers to f32 rounding, and
    both ranks hold the same averaged gradient bit for bit."""
    _gpu_or_skip()
    one = _run_ranks(1, tmp_path / "g1", "grad")[0]
    two = _run_ranks(2, tmp_path / "g2", "grad")
    assert np.array_equal(two[0]["grad"], two[1]["grad"])
    g1, g2 = one["grad"], two[0]["grad"]
    assert np.all(np.isfinite(g1)) and np.abs(g1).max() > 0
    assert np.abs(g2 - g1).max() <= 2e-5 * np.abs(g1).max(), np.abs(g2 - g1).max() / np.abs(g1).max()
    assert abs(complex(two[0]["energy"]) - complex(one["energy"])) <= 2e-6 * abs(complex(one["energy"]))


def test_train_two_ranks_checkpoint(tmp_path):
    """train() on 2 ranks: 2 Adam iterations with a
    checkpoint at every step (save_time_interval 0, save_step_interval 1), so the
    collective save decision, the walker all_gather and the gradient all-reduce all run.
    Both ranks end with the same parameters; ckpt_000001.npz holds the two shards in rank
    order; a one-rank restore reproduces them; one rank running the same job logs the same
    iteration-0 energy to f32 rounding."""
    _gpu_or_skip()
    run2 = tmp_path / "run2"
    two = _run_ranks(2, tmp_path / "t2", "train", run2)
    assert np.array_equal(two[0]["params"], two[1]["params"])
    for step in (0, 1):
        assert (run2 / f"ckpt_{step:06d}.npz").exists()
    with np.load(run2 / "ckpt_000001.npz", allow_pickle=False) as f:
        assert np.array_equal(f["data"], np.concatenate([two[0]["data"], two[1]["data"]]))
        assert int(f["step"]) == 1 and float(f["mcmc_width"]) == float(two[0]["width"])
    rows = (run2 / "train_stats.csv").read_text().splitlines()
    assert len(rows) == 3 and rows[0].startswith("step,pmove,energy")
    run1 = tmp_path / "run1"
    _run_ranks(1, tmp_path / "t1", "train", run1)
    # (parameters after Adam steps are not compared across world sizes: Adam's first update
    # is ~lr * sign(g), so components whose gradient is at rounding level legitimately differ)
    e1 = [float(r.split(",")[2]) for r in (run1 / "train_stats.csv").read_text().splitlines()[1:]]
    e2 = [float(r.split(",")[2]) for r in rows[1:]]
    assert abs(e1[0] - e2[0]) <= 2e-4  # iteration 0: same walkers, same parameters
    # restore on one rank: the re-sharded walkers are the concatenated shards
    code = (f"import sys; sys.path[:0]={[str(ROOT), str(ROOT / 'tests')]!r}\n"
            "import numpy as np, torch\n"
            "from deephall_amd import config, make_network\n"
            "from deephall_amd.log import LogManager\n"
            "m = make_network(config.System(nspins=(3, 0), flux=2, interaction_strength=0.0),"
            " config.from_dict(config.Network, {'psiformer': {'num_layers': 1, 'num_heads': 1, 'heads_dim': 4}}))\n"
            f"step, st = LogManager.restore_checkpoint({str(run2 / 'ckpt_000001.npz')!r}, m, torch.device('cuda'))\n"
            f"np.savez({str(tmp_path / 'restored.npz')!r}, step=step, data=st.data.cpu().numpy(),"
            " params=st.params.flat.cpu().numpy())\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    res = np.load(tmp_path / "restored.npz")
    assert int(res["step"]) == 2
    assert np.array_equal(res["data"], np.concatenate([two[0]["data"], two[1]["data"]]))
    assert np.array_equal(res["params"], two[0]["params"])


def test_kfac_two_ranks(tmp_path):
    """KFAC across ranks (kfac_jax multi_device, reference
    optimizers/kfac.py:214-215): 2 ranks on equal shards of 64 fixed walkers against one rank
    holding all of them.  The ONE [gradient | curvature statistics] all-reduce gives the
    one-rank gradient, and the statistics kfac_jax's multi-device estimator gives: the mean of
    the two shards' statistics (the one-rank run computes each shard's) — for the dense
    factors that is the full-batch Gram matrix, for the generic (NaiveDiagonal) entries
    (sum_shard g)^2 / B_shard averaged, which is not the full-batch value.  After each of two
    KFAC steps both ranks hold bit-identical parameters; on the dense blocks the first step's
    P g equals the one-rank run's to the f32 rounding carried through the damped inverses and
    the update is parallel to it (the generic entries differ by construction); both steps' P g
    and parameters equal oracle/kfac.py's two-shard restatement (below)."""
    _gpu_or_skip()
    one = _run_ranks(1, tmp_path / "k1", "kfac")[0]
    two = _run_ranks(2, tmp_path / "k2", "kfac")
    for k in ("grad", "curv", "p1", "p2", "pg1", "pg2"):
        assert np.array_equal(two[0][k], two[1][k]), k  # every rank holds the same values
    g1, g2 = one["grad"], two[0]["grad"]
    assert np.all(np.isfinite(g1)) and np.abs(g1).max() > 0
    assert np.abs(g2 - g1).max() <= 2e-5 * np.abs(g1).max()
    c2 = two[0]["curv"]
    ce = 0.5 * (one["curv_h0"] + one["curv_h1"])
    assert np.all(np.isfinite(ce)) and np.abs(ce).max() > 0
    assert np.abs(c2 - ce).max() <= 2e-5 * np.abs(ce).max(), np.abs(c2 - ce).max() / np.abs(ce).max()
    dense = ~one["gmask"]
    pg1, pg2 = one["pg1"][dense], two[0]["pg1"][dense]
    assert np.abs(pg2 - pg1).max() <= 1e-3 * np.abs(pg1).max(), np.abs(pg2 - pg1).max() / np.abs(pg1).max()
    # the update is -lr * c * P g with ONE norm-constraint coefficient c, whose <P g, g> includes
    # the generic entries: on the dense blocks the two updates are parallel
    d1, d2 = (one["p1"] - one["p0"])[dense], (two[0]["p1"] - two[0]["p0"])[dense]
    c = float(d1 @ d2) / float(d1 @ d1)
    assert c > 0 and np.abs(d2 - c * d1).max() <= 1e-3 * np.abs(d2).max()
    # step 2 starts from different parameters than the one-rank run (the generic entries and c
    # differ) and P g with damping 1e-3 amplifies that (41 % in round 4), so its comparator is
    # the oracle with the same two-shard semantics: oracle/kfac.py stepped
    # twice on the inputs the ranks all-reduced (each step's gradient and statistics, float32
    # EMA storage) gives the ranks' P g and parameters at both steps; and the oracle's own
    # two-shard statistics at the step-1 parameters (per-device statistics averaged, kfac_jax
    # multi_device; the generic ones are NOT the full-batch value) equal what the ranks
    # all-reduced at step 2, to the tolerances of tests/test_gpu_kfac.py
    r0 = two[0]
    for s in (1, 2):
        pg, pg_ref = r0[f"pg{s}"], r0[f"oracle_pg{s}"]
        assert np.abs(pg - pg_ref).max() <= 2e-5 * np.abs(pg_ref).max(), (s, np.abs(pg - pg_ref).max() / np.abs(pg_ref).max())
        p, p_ref = r0[f"p{s}"], r0[f"oracle_p{s}"]
        assert np.abs(p - p_ref).max() <= 1e-6 * max(1.0, np.abs(p_ref).max()), (s, np.abs(p - p_ref).max())
    assert float(r0["stat2_err_dense"]) < 1.5e-4, float(r0["stat2_err_dense"])
    assert float(r0["stat2_err_generic"]) < 1e-4, float(r0["stat2_err_generic"])


def test_rccl_process_group():
    """a world-size-1 "nccl" process group (RCCL on ROCm) initialises
    on the box and all-reduces on the GPU; constants.pmean runs through it."""
    _gpu_or_skip()
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        res = _run_ranks(1, Path(d) / "n", "nccl")[0]
    assert str(res["backend"]) == "nccl"
    assert np.array_equal(res["t"], np.arange(16, dtype=np.float32))
    assert np.array_equal(res["m"], np.full(3, 2.5, dtype=np.float32))
