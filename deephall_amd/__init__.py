"""deephall_amd — MI355X-native VMC inner loop for DeepHall (Psiformer log psi,
Metropolis walker update, local energy) behind the reference's Python API.

Public names mirror the reference package:
  make_network           deephall.networks.make_network
  local_energy           deephall.hamiltonian.local_energy   (alias make_local_energy)
  make_local_kinetic_energy, make_potential
  make_mcmc_step, update_mcmc_width   deephall.mcmc
  make_loss_fn, LossMode              deephall.loss (statistics + parameter gradient)
  make_optimizer_step                 deephall.optimizers (KFAC = the default, Adam, none)
  train, init_guess, initalize_state, setup_mcmc, vmc   deephall.train
All compute runs in the HIP library deephall_amd/_lib/libdeephall_amd.so.
"""

from .config import MCMC, Config, InteractionType, Network, NetworkType, OrbitalType, PsiformerNetwork, System
from .hamiltonian import local_energy, make_local_energy, make_local_kinetic_energy, make_potential
from .loss import LossMode, make_loss_fn
from .mcmc import make_mcmc_step, update_mcmc_width
from .networks import make_network
from .optimizers import make_optimizer_step
from .random import Key, PRNGKey
from .train import train

__all__ = [
    "Config",
    "System",
    "Network",
    "NetworkType",
    "OrbitalType",
    "PsiformerNetwork",
    "MCMC",
    "InteractionType",
    "make_network",
    "local_energy",
    "make_local_energy",
    "make_local_kinetic_energy",
    "make_potential",
    "make_mcmc_step",
    "update_mcmc_width",
    "make_loss_fn",
    "LossMode",
    "Key",
    "PRNGKey",
    "make_optimizer_step",
    "train",
]
