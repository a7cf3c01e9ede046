"""TEST/BENCH INFRASTRUCTURE ONLY — CPU timing of the reference algorithm (the port).

The reference JAX-CPU path cannot run here (no jax; Python 3.10), so bench.py's
``cpu_baseline`` times this repository's float32 restatement of it
(oracle/reference.py): the forward pass vmapped over walkers, and the local
energy with the full autograd Hessian exactly as hamiltonian.py:105-113
(``jax.hessian`` -> torch.func.hessian), vmapped over walkers like loss.py:51.
One VMC iteration per walker = (steps + 1) forwards (mcmc.py:142-145) + one E_L.
"""

from __future__ import annotations

import time

import numpy as np
import torch
from torch.func import vmap

from . import reference as R


def measure(cfg: R.OracleConfig, steps: int = 10, el_batch: int = 16, fwd_batch: int = 256, budget_s: float = 15.0,
            threads: int | None = None, seed: int = 0) -> dict:
    if threads:
        torch.set_num_threads(int(threads))
    p = {k: v.float() for k, v in R.init_params(cfg, seed=42).items()}
    rng = np.random.default_rng(seed)
    N = cfg.nelec

    def walkers(B):
        return torch.tensor(R.init_guess_from_uniforms(rng.random((B, N)), rng.random((B, N))), dtype=torch.float32)

    f = lambda y: R.logpsi(p, cfg, y)  # noqa: E731
    ke = R.make_local_kinetic_energy(lambda pp, y: R.logpsi(pp, cfg, y), cfg.Q, cfg.r)
    fwd = vmap(f)
    el = vmap(lambda y: ke(p, y))
    # warm up (first vmap trace)
    fwd(walkers(8))
    el(walkers(2))
    t_fwd, n_fwd = 0.0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s / 3:
        x = walkers(fwd_batch)
        a = time.perf_counter()
        fwd(x)
        t_fwd += time.perf_counter() - a
        n_fwd += fwd_batch
    t_el, n_el = 0.0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2 * budget_s / 3 or n_el == 0:
        x = walkers(el_batch)
        a = time.perf_counter()
        el(x)
        t_el += time.perf_counter() - a
        n_el += el_batch
    per_fwd = t_fwd / n_fwd
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), model)
    except OSError:
        pass
    per_el = t_el / n_el
    per_iter = per_el + (steps + 1) * per_fwd
    return {
        "local_energies_per_sec": 1.0 / per_iter,
        "el_only_per_sec": 1.0 / per_el,
        "walker_steps_per_sec": 1.0 / per_fwd,
        "threads": torch.get_num_threads(),
        "cpu_model": model,
        "host_cpus": __import__("os").cpu_count(),
        "sample": f"{n_el} local energies (full autograd Hessian, f32, vmap batch {el_batch}) + "
        f"{n_fwd} forwards (vmap batch {fwd_batch}); {t_el + t_fwd:.1f} s CPU",
    }
