"""Run directory, statistics CSV and checkpoints — mirror of deephall/log.py:86-222.

``StatsWriter`` restates the reference's StatsWriter (Copyright 2024-2025 Bytedance Ltd.
and/or its affiliates, Apache-2.0) to keep its CSV contract.

* ``StatsWriter`` (log.py:86-133): ``train_stats.csv`` with a header row written once
  (appending to an existing non-empty file keeps its header), the same row echoed to
  the log without the hidden fields, ``force_flush`` before checkpoints, the file
  removed if nothing was written.
* ``LogManager`` (log.py:136-222): save path ``DeepHall_n{N}l{flux}_{timestamp}`` unless
  given, ``config.yml`` (git commit + the config, a diff against the restored one on
  stderr), ``ckpt_{step:06d}.npz`` save / restore-newest with fallback to older files.

Checkpoint format.  The reference pickles the jax parameter tree into the npz
(log.py:174-178, restored with allow_pickle=True, SURVEY.md finding 6).  Here every
entry is a plain array under a flat key, readable with ``np.load(allow_pickle=False)``:
``step``, ``mcmc_width``, ``data`` [B_total, N, 2] (all ranks, gathered to rank 0),
``params/<Flax path>`` per leaf, ``opt_state/<name>`` (Adam: mu, nu, count — in the
flat reference-tree layout).  A restore re-shards ``data`` over the current ranks.
"""

from __future__ import annotations

import dataclasses
import datetime
import difflib
import enum
import logging
import subprocess
import sys
from contextlib import contextmanager
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

from . import constants
from .types import CheckpointState

logger = logging.getLogger("deephall_amd")


def init_logging():
    """log.py:70-83: INFO to stderr with a time stamp, no propagation."""
    logger.setLevel(logging.INFO)
    if any(getattr(h, "_dh_stderr", False) for h in logger.handlers):
        return
    handler = logging.StreamHandler(sys.stderr)
    handler._dh_stderr = True
    handler.setFormatter(logging.Formatter("%(asctime)s %(levelname)s: %(message)s"))
    handler.setLevel(logging.INFO)
    logger.setLevel(logging.INFO)
    logger.addHandler(handler)
    logger.propagate = False


class StatsWriter:
    """CSV + log writer with a header row and hidden-on-stderr fields (log.py:86-133)."""

    def __init__(self, stats_path: Path):
        self.stats_path = Path(stats_path)
        self.stats_file = None
        self.hidden_fields: set = set()

    def __enter__(self):
        self.should_write_head = not self.stats_path.exists() or self.stats_path.stat().st_size == 0
        self.stats_file = self.stats_path.open("a" if self.stats_path.exists() else "w", buffering=1)
        return self

    def hide(self, *args):
        self.hidden_fields.update(args)

    def log(self, **kwargs):
        if self.should_write_head:
            self.stats_file.write(",".join(kwargs.keys()) + "\n")
            self.should_write_head = False
        self.stats_file.write(",".join(kwargs.values()) + "\n")
        logger.info(", ".join(f"{k}={v}" for k, v in kwargs.items() if k not in self.hidden_fields))

    def force_flush(self):
        self.stats_file.close()
        self.stats_file = self.stats_path.open("a", buffering=1)

    def __exit__(self, exc_type, exc_value, traceback):
        self.stats_file.close()
        if self.should_write_head:  # nothing got written
            self.stats_path.unlink(missing_ok=True)


def _plain(obj):
    if dataclasses.is_dataclass(obj):
        return {f.name: _plain(getattr(obj, f.name)) for f in dataclasses.fields(obj)}
    if isinstance(obj, enum.Enum):
        return obj.value
    if isinstance(obj, tuple):
        return list(obj)
    return obj


def get_git_commit() -> str:
    try:
        return subprocess.check_output(["git", "rev-parse", "--short", "HEAD"], cwd=Path(__file__).parent, text=True,
                                       stderr=subprocess.DEVNULL).strip()
    except (subprocess.CalledProcessError, OSError):
        return "''"


def _gather_rows(t: torch.Tensor) -> np.ndarray:
    """Walkers of every rank, rank order (the reference's [ndev, B/ndev] data, flattened)."""
    n = constants.world_size()
    if n == 1:
        return t.detach().cpu().numpy()
    parts = [torch.empty_like(t) for _ in range(n)]
    dist.all_gather(parts, t.contiguous())
    return torch.cat(parts).cpu().numpy()


class LogManager:
    def __init__(self, cfg):
        if cfg.log.save_path is None:
            stamp = datetime.datetime.now().strftime("%Y%m%d_%H:%M:%S")
            self.save_path = Path(f"DeepHall_n{sum(cfg.system.nspins)}l{cfg.system.flux}_{stamp}")
        else:
            self.save_path = Path(cfg.log.save_path)
        self.explicit_restore = cfg.log.restore_path is not None
        if cfg.log.restore_path is None:
            self.restore_path = self.save_path
        else:
            self.restore_path = Path(cfg.log.restore_path)
            if not self.restore_path.exists():
                logger.warning("Restore path %s does not exist!", self.restore_path)
        self.rank0 = constants.rank() == 0
        if self.rank0:
            self.save_path.mkdir(parents=True, exist_ok=True)
            self.check_config(cfg)

    def check_config(self, cfg) -> None:
        """Save the config (with the git commit) and print its diff against the restored one."""
        import yaml

        current = [f"git_commit: {get_git_commit()}\n"]
        current.extend(yaml.safe_dump(_plain(cfg), sort_keys=False).splitlines(keepends=True))
        old_path = self.restore_path / "config.yml"
        original = old_path.read_text().splitlines(keepends=True) if old_path.exists() else []
        sys.stderr.writelines(difflib.ndiff(original, current))
        (self.save_path / "config.yml").write_text("".join(current))

    def save_checkpoint(self, step: int, state: CheckpointState) -> None:
        """ckpt_{step:06d}.npz with flat keys (collective: every rank must call it)."""
        data = _gather_rows(state.data)
        if not self.rank0:
            return
        arrays = {"step": np.asarray(step), "mcmc_width": np.asarray(float(state.mcmc_width)), "data": data}
        for k, v in state.params.items():
            arrays[f"params/{k}"] = v.detach().cpu().numpy()
        if state.opt_state is not None:
            for k, v in state.opt_state.state_dict().items():
                arrays[f"opt_state/{k}"] = v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v)
        path = self.save_path / f"ckpt_{step:06d}.npz"
        logger.info("Saving checkpoint %s", path)
        with path.open("wb") as f:
            np.savez_compressed(f, **arrays)

    def try_restore_checkpoint(self, model, device, opt_init=None):
        """Newest readable checkpoint in restore_path (or the file itself), else None.

        When ``log.restore_path`` was given explicitly and it holds checkpoints none of
        which can be read (e.g. a reference checkpoint with its pickled parameter tree,
        SURVEY.md finding 6), this raises instead of silently starting from random
        parameters; the implicit restore from ``save_path`` keeps the reference's
        fall-through (log.py:180-192)."""
        if not self.restore_path.exists():
            return None
        if self.restore_path.is_file():
            return self.restore_checkpoint(self.restore_path, model, device, opt_init)
        paths = sorted(self.restore_path.glob("ckpt_*.npz"), reverse=True)
        errors = []
        for path in paths:
            try:
                return self.restore_checkpoint(path, model, device, opt_init)
            except Exception as e:  # noqa: BLE001  (log.py:190: try older checkpoints)
                logger.warning("Error restoring checkpoint %s: %s", path, e)
                errors.append(f"{path.name}: {e}")
        if paths and self.explicit_restore:
            raise RuntimeError(f"log.restore_path={self.restore_path}: no checkpoint could be restored "
                               f"({'; '.join(errors)}); checkpoints of this library are flat-key npz files "
                               f"(INTEGRATION.md §3)")
        return None

    @staticmethod
    def restore_checkpoint(path, model, device, opt_init=None):
        """Returns (next step, CheckpointState) with this rank's walker shard."""
        with np.load(Path(path), allow_pickle=False) as f:
            step = int(f["step"]) + 1
            params = model.init(0, device=device)  # a ParamTree of the right layout
            for k in params:
                params[k].copy_(torch.as_tensor(f[f"params/{k}"]))
            data = f["data"]
            n, r = constants.world_size(), constants.rank()
            if data.shape[0] % n:
                raise ValueError(f"checkpoint has {data.shape[0]} walkers, not divisible by {n} ranks")
            per = data.shape[0] // n
            shard = torch.tensor(data[r * per : (r + 1) * per], dtype=torch.float32, device=device).contiguous()
            opt_state = None
            keys = [k for k in f.files if k.startswith("opt_state/")]
            if keys and opt_init is not None:
                opt_state = opt_init(params)
                if opt_state is not None:
                    saved = {k.split("/", 1)[1] for k in keys}
                    if saved != set(opt_state.state_dict()):
                        # a different optimizer wrote the checkpoint (e.g. an Adam checkpoint
                        # restored into a run with the KFAC default): keep the params, walkers
                        # and step, start the optimizer state afresh
                        logger.warning("Checkpoint %s: optimizer state keys %s do not match the current "
                                       "optimizer's %s; params, walkers and step restored, optimizer state "
                                       "re-initialised", path, sorted(saved), sorted(opt_state.state_dict()))
                    else:
                        # same optimizer: a wrong size or corrupt entry is an error, not a reset
                        opt_state.load_state_dict({k.split("/", 1)[1]: f[k] for k in keys})
            width = float(f["mcmc_width"])
        logger.info("Restored checkpoint %s", path)
        return step, CheckpointState(params, shard, opt_state, width)

    @contextmanager
    def create_writer(self):
        if not self.rank0:
            yield _NullWriter()
            return
        with StatsWriter(self.save_path / "train_stats.csv") as writer:
            yield writer


class _NullWriter:
    def hide(self, *args):
        pass

    def log(self, **kwargs):
        pass

    def force_flush(self):
        pass
