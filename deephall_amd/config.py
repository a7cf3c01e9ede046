"""Configuration dataclasses — the fields of deephall/config.py:56-214 the hot path reads.

Field names, defaults and meaning follow the reference exactly (System 56-79,
PsiformerNetwork 92-97, Network 100-104, MCMC 107-122, LearningRate / optimizers
125-165, Log 168-198, Config 201-214).  The
OmegaConf machinery is out of scope; ``Config.from_dict`` mirrors the reference's
``from_dict`` (config.py:23-48: nested dataclasses, extra keys ignored).
The reference needs Python >= 3.11 (``StrEnum``); these are ``str`` Enums.
"""

from __future__ import annotations

import enum
import time
from dataclasses import dataclass, field, fields, is_dataclass
from typing import Any, Optional, Tuple


def from_dict(cls, dikt: dict):
    try:
        ftypes = {f.name: f.type for f in fields(cls)}
        resolved = {f.name: f for f in fields(cls)}
        kwargs = {}
        for k, v in dikt.items():
            if k not in ftypes:
                continue  # allow extra keys (config.py:41)
            default = resolved[k].default_factory() if callable(resolved[k].default_factory) else None
            if is_dataclass(default) and isinstance(v, dict):
                kwargs[k] = from_dict(type(default), v)
            else:
                kwargs[k] = v
        return cls(**kwargs)
    except Exception as e:  # noqa: BLE001
        raise ValueError(f"Error converting dictionary to {cls.__name__}: {e}") from e


class InteractionType(str, enum.Enum):
    coulomb = "coulomb"
    harmonic = "harmonic"


class NetworkType(str, enum.Enum):
    psiformer = "psiformer"
    laughlin = "laughlin"


class OrbitalType(str, enum.Enum):
    full = "full"
    sparse = "sparse"


@dataclass
class System:
    flux: int = 2
    radius: Optional[float] = None
    nspins: Tuple[int, int] = (3, 0)
    interaction_strength: float = 1.0
    lz_center: float = 0.0
    lz_penalty: float = 0.0
    l2_penalty: float = 0.0
    interaction_type: InteractionType = InteractionType.coulomb


@dataclass
class PsiformerNetwork:
    num_heads: int = 4
    heads_dim: int = 64
    num_layers: int = 2
    determinants: int = 1


@dataclass
class Network:
    type: NetworkType = NetworkType.psiformer
    orbital: OrbitalType = OrbitalType.full
    psiformer: PsiformerNetwork = field(default_factory=PsiformerNetwork)


@dataclass
class MCMC:
    steps: int = 10
    width: float = 0.1
    burn_in: int = 200
    adapt_frequency: int = 100


@dataclass
class LearningRate:
    """rate * (1 / (1 + t / delay)) ** decay (config.py:125-137)."""

    rate: float = 0.005
    decay: float = 1.0
    delay: float = 2000.0

    def schedule(self, t):
        return self.rate * (1.0 / (1.0 + (t / self.delay))) ** self.decay


class OptimizerName(str, enum.Enum):
    adam = "adam"
    kfac = "kfac"
    none = "none"


@dataclass
class OptimizerAdam:
    lr: LearningRate = field(default_factory=LearningRate)


@dataclass
class OptimizerKfac:
    lr: LearningRate = field(default_factory=lambda: LearningRate(rate=0.05))


@dataclass
class Optim:
    """config.py:160-165.  The default optimizer is KFAC, as in the reference
    (optimizers.py: make_kfac_training_step on the dh_kfac_* kernels)."""

    iterations: int = 1000
    optimizer: Optional[OptimizerName] = OptimizerName.kfac
    adam: OptimizerAdam = field(default_factory=OptimizerAdam)
    kfac: OptimizerKfac = field(default_factory=OptimizerKfac)


@dataclass
class Log:
    """config.py:168-198."""

    save_path: Optional[str] = None
    restore_path: Optional[str] = None
    save_time_interval: int = 10 * 60
    save_step_interval: int = 1000
    initial_energy: bool = True


@dataclass
class Config:
    batch_size: int = 3360
    seed: int = field(default_factory=lambda: int(time.time()))
    system: System = field(default_factory=System)
    network: Network = field(default_factory=Network)
    mcmc: MCMC = field(default_factory=MCMC)
    optim: Optim = field(default_factory=Optim)
    log: Log = field(default_factory=Log)

    @classmethod
    def from_dict(cls, dikt: dict[str, Any]) -> "Config":
        return from_dict(cls, dikt)
