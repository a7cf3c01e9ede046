"""VMC driver — the callers of the hot path in deephall/train.py.

* ``init_guess`` (train.py:40-54) — uniform walkers on the sphere, device RNG
* ``initalize_state`` (train.py:57-65) — walkers sharded contiguously by rank
* ``setup_mcmc`` (train.py:68-77)
* ``train`` (train.py:80-167) — checkpoint restore or fresh state, burn-in, initial
  energy, then per iteration: mcmc_step (128-130), update_mcmc_width (131-137), the
  optimizer step (140: Adam or inference, optimizers.py), the stats row to
  train_stats.csv (141-152), checkpoints by time/step interval, on NaN, at the last
  step and on SIGINT/SIGTERM (154-165), NaN / signal abort (166-167)
* ``vmc`` — the inference loop with the iteration's device work fused into one packed
  statistics all-reduce (the bench's step)

Multi-GPU: one process per GPU (torchrun-style env); each rank owns
batch_size / world_size walkers.
"""

from __future__ import annotations

import logging
import os
import signal
import time

import numpy as np
import torch
import torch.distributed as dist

from . import _lib, constants
from .config import Config
from .loss import device_stats, reduce_stats
from .hamiltonian import _run_local_energy
from .mcmc import make_mcmc_step, update_mcmc_width
from .networks import make_network
from .networks.psiformer import _ptr, _stream, get_handle
from .random import Key, PRNGKey

logger = logging.getLogger("deephall_amd")


def init_distributed(backend: str | None = None):
    """Initialise torch.distributed from torchrun env vars if WORLD_SIZE > 1."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws > 1 and not dist.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return constants.rank(), constants.world_size()


def init_guess(key: Key, batch: int, nelec: int, device=None, walker_offset: int = 0, network=None) -> torch.Tensor:
    """train.py:40-54 on the device: theta = arccos U(-1,1), phi = U(-pi,pi)."""
    device = torch.device(device or "cuda")
    spec = getattr(network, "spec", None)
    if spec is None or sum(spec.nspins) != nelec:
        # the device kernel draws nelec = the handle's electron count per walker: a handle of
        # another size (e.g. one_rdm's single r' per walker) would write past x
        from .networks.psiformer import NetworkSpec

        spec = NetworkSpec(nspins=(nelec, 0), flux=2, ndets=1, num_heads=1, heads_dim=4, num_layers=0)
    h = get_handle(spec, device)
    x = torch.empty(batch, nelec, 2, dtype=torch.float32, device=device)
    _lib.check(h.lib.dh_init_walkers(h.h, _ptr(x), batch, int(key.seed), int(walker_offset), _stream(device)))
    return x


def initalize_state(cfg: Config, model, device=None):
    """train.py:57-65: returns (step, (params, data, opt_state, mcmc_width)) for this rank."""
    r, n = constants.rank(), constants.world_size()
    if cfg.batch_size % n:
        raise ValueError("batch_size must be divisible by the number of GPUs")
    per = cfg.batch_size // n
    device = device or torch.device("cuda", torch.cuda.current_device())
    data = init_guess(Key(cfg.seed * 2 + 1), per, sum(cfg.system.nspins), device, walker_offset=r * per, network=model)
    params = model.init(PRNGKey(cfg.seed), data, device=device)
    return 0, (params, data, None, float(cfg.mcmc.width))


def setup_mcmc(cfg: Config, model):
    """train.py:68-77."""
    per = cfg.batch_size // constants.world_size()
    step = make_mcmc_step(model, batch_per_device=per, steps=cfg.mcmc.steps)
    pmoves = np.zeros(cfg.mcmc.adapt_frequency)
    return step, pmoves


def make_vmc_iteration(model, batch_per_device: int, steps: int, groups: int = 1):
    """The device work of one VMC iteration (train.py:128-140 before the statistics):
    ``mcmc_step`` then the local energy, for this rank's walkers.

    The walkers are independent and the device RNG is keyed by global walker index, so
    the batch is cut into ``groups`` contiguous walker groups, each run start to finish
    (its MCMC moves, then its local energies) on its own HIP stream; the results are
    bit-identical to one group (same walkers, same random numbers, same arithmetic).
    Every side stream waits on the caller's stream ONCE, before any group's work is
    queued, so the groups really run concurrently (DESIGN.md §7.1 has the measurement).
    The default is one group.

    Returns ``iteration(params, data, key, width) -> (data, e_l [B,2], obs [B,8],
    n_accept [B])``; data is updated in place.
    """
    B = batch_per_device
    groups = max(1, min(int(groups), B))
    sizes = [B // groups + (1 if g < B % groups else 0) for g in range(groups)]
    mcmc = [make_mcmc_step(model, n, steps) for n in sizes]
    side: list = []

    def iteration(params, data: torch.Tensor, key, width):
        main = torch.cuda.current_stream(data.device)
        while len(side) < groups - 1:
            side.append(torch.cuda.Stream(data.device))
        base = constants.rank() * B
        model.prepare(params, data.device)  # any parameter upload is queued on `main` first
        for s in side[: groups - 1]:
            s.wait_stream(main)  # inputs ready; nothing of this iteration is queued yet
        outs, off = [], 0
        for g, n in enumerate(sizes):
            s = main if g == 0 else side[g - 1]
            with torch.cuda.stream(s):
                d = data[off : off + n]
                mcmc[g](params, d, key, width, reduce=False, walker_offset=base + off)
                e, o = _run_local_energy(model, params, d)
                outs.append((e, o, mcmc[g].last_n_accept))
            off += n
        for s in side[: groups - 1]:
            main.wait_stream(s)
        for g in range(1, groups):
            for t in outs[g]:
                t.record_stream(main)
        if groups == 1:
            return data, outs[0][0], outs[0][1], outs[0][2]
        return data, torch.cat([o[0] for o in outs]), torch.cat([o[1] for o in outs]), torch.cat([o[2] for o in outs])

    iteration.sizes = sizes
    return iteration


def vmc(cfg: Config, iterations: int | None = None, log=None, burn_in: int | None = None, groups: int = 1):
    """Inference-mode VMC loop (optimizer 'none').  Returns the list of per-iteration stats."""
    init_distributed()
    model = make_network(cfg.system, cfg.network)
    _, (params, data, _, width) = initalize_state(cfg, model)
    mcmc_step, pmoves = setup_mcmc(cfg, model)
    key = PRNGKey(cfg.seed)
    steps = cfg.mcmc.steps
    for _ in range(cfg.mcmc.burn_in if burn_in is None else burn_in):
        data, _ = mcmc_step(params, data, key, width, reduce=False)
        key = key.advance(steps)
    history = []
    iters = cfg.optim.iterations if iterations is None else iterations
    iteration = make_vmc_iteration(model, data.shape[0], steps, groups)
    for t in range(iters):
        data, e_l, obs, n_accept = iteration(params, data, key, width)
        key = key.advance(steps)
        local = device_stats(model, e_l, obs, n_accept, steps)
        stats = reduce_stats(local)  # the single all-reduce of this iteration
        width, pmoves = update_mcmc_width(t, width, cfg.mcmc.adapt_frequency, stats["pmove"], pmoves)
        row = {k: (complex(v.item()) if v.is_complex() else float(v.item())) for k, v in stats.items()}
        history.append(row)
        if log is not None and constants.rank() == 0:
            log(
                f"step={t} pmove={row['pmove']:.2f} energy={row['energy'].real:.4f} "
                f"energy_imag={row['energy'].imag:+.4f} variance={row['variance']:.4f} "
                f"Lz={row['angular_momentum_z']:+.4f} L_square={row['angular_momentum_square']:.4f}"
            )
        if np.isnan(row["energy"].real):
            raise SystemExit("=" * 30 + " ABORT " + "=" * 30)
    return history


class GracefulKiller:
    """train.py:170-187: SIGINT / SIGTERM set a flag; the loop checkpoints and exits.

    As the reference does, the first signal restores the original handlers (a second
    Ctrl-C then stops a stuck run); ``restore()`` puts them back when train() returns."""

    kill_now = False

    def __init__(self):
        self.original = {}
        try:
            for sig in (signal.SIGINT, signal.SIGTERM):
                self.original[sig] = signal.signal(sig, self.exit_gracefully)
        except ValueError:  # not the main thread
            self.original = {}

    def exit_gracefully(self, *args):
        self.kill_now = True
        self.restore()

    def restore(self):
        for sig, handler in self.original.items():
            signal.signal(sig, handler)
        self.original = {}


def train(cfg: Config):
    """train.py:80-167 on MI355X.  Returns the final CheckpointState."""
    from . import optimizers
    from .config import OptimizerName
    from .log import LogManager, init_logging
    from .loss import LossMode, make_loss_fn
    from .types import CheckpointState

    init_logging()
    init_distributed()
    log_manager = LogManager(cfg)
    model = make_network(cfg.system, cfg.network)
    mcmc_step, pmoves = setup_mcmc(cfg, model)
    opt_init, training_step = optimizers.make_optimizer_step(cfg, model)
    key = PRNGKey(cfg.seed)
    steps = cfg.mcmc.steps
    device = torch.device("cuda", torch.cuda.current_device())
    restored = log_manager.try_restore_checkpoint(model, device, opt_init)
    if restored is not None:
        initial_step, (params, data, opt_state, width) = restored
        key = key.advance(steps * (cfg.mcmc.burn_in + initial_step))  # fresh draws after a restore
    else:
        initial_step, (params, data, opt_state, width) = initalize_state(cfg, model, device)
    name = cfg.optim.optimizer
    if (
        name is not None and OptimizerName(getattr(name, "value", name)) == OptimizerName.none
        and cfg.log.restore_path is not None and cfg.log.restore_path != cfg.log.save_path
    ):  # inference after a training run starts its own step count (train.py:94-99)
        initial_step = 0
    if opt_state is None:
        opt_state = opt_init(params, None, data)
    logger.info("Start VMC with %s GPU process(es)", constants.world_size())
    if initial_step == 0:
        for _ in range(cfg.mcmc.burn_in):
            data, _ = mcmc_step(params, data, key, width)
            key = key.advance(steps)
        logger.info("Burn in MCMC complete")
        if cfg.log.initial_energy:
            initial_stats, _ = make_loss_fn(model, cfg.system, LossMode.ENERGY_DIFF)(params, data)
            logger.info("Initial energy: %s", float(initial_stats["energy"].real))
    state = CheckpointState(params, data, opt_state, width)
    last_save_time = time.time()
    killer = GracefulKiller()
    try:
        with log_manager.create_writer() as writer:
            writer.hide("kinetic", "potential", "Lz_square")
            for step in range(initial_step, cfg.optim.iterations):
                # mcmc.py:146-147's pmove pmean is folded into the iteration's packed statistics
                # all-reduce, together with this rank's checkpoint / signal flags: one statistics
                # all-reduce (+ the gradient's) per iteration, and every rank takes the same
                # checkpoint decision (save_checkpoint is a collective)
                new_data, _ = mcmc_step(state.params, state.data, key, state.mcmc_width, reduce=False)
                n_accept = mcmc_step.last_n_accept
                key = key.advance(steps)
                state = state._replace(data=new_data)
                flags = (time.time() - last_save_time > cfg.log.save_time_interval, killer.kill_now)
                state, stats = training_step(state, None, n_accept=n_accept, steps=steps, flags=flags)
                pmove = float(stats["pmove"])
                time_due, kill_now = (bool(v > 0) for v in stats["flags"].tolist())
                new_width, pmoves = update_mcmc_width(step - initial_step, state.mcmc_width,
                                                      cfg.mcmc.adapt_frequency, pmove, pmoves)
                state = state._replace(mcmc_width=new_width)
                energy = complex(stats["energy"].item())
                writer.log(
                    step=str(step),
                    pmove=f"{pmove:.2f}",
                    energy=f"{energy.real:.4f}",
                    energy_imag=f"{energy.imag:+.4f}",
                    potential=f"{float(stats['potential']):.4f}",
                    kinetic=f"{complex(stats['kinetic'].item()).real:.4f}",
                    variance=f"{float(stats['variance']):.4f}",
                    Lz=f"{float(stats['angular_momentum_z']):+.4f}",
                    Lz_square=f"{float(stats['angular_momentum_z_square']):.4f}",
                    L_square=f"{float(stats['angular_momentum_square']):.4f}",
                )
                nan = bool(np.isnan(energy.real))
                if ((time_due and (step + 1) % cfg.log.save_step_interval == 0)
                        or nan or step == cfg.optim.iterations - 1 or kill_now):
                    last_save_time = time.time()
                    writer.force_flush()
                    log_manager.save_checkpoint(step, state)
                if kill_now or nan:
                    raise SystemExit("=" * 30 + " ABORT " + "=" * 30)
    finally:
        killer.restore()
    return state
