"""Generate the golden vectors in tests/golden/ from the float64 oracle.

The reference (JAX/Flax, Python >= 3.11) cannot be imported in this container
(SURVEY.md §8c), so the vectors come from oracle/reference.py — the full-Hessian
restatement of hamiltonian.py — which is itself pinned by the reference's
analytic known answers (tests/test_oracle_kat.py).  Parameters are NOT stored:
they are regenerated from `param_seed` by oracle.reference.init_params (numpy
PCG64, stable) plus the perturbation in tests/helpers.make_params, rounded to
float32 so the GPU sees exactly the same weights.

Run:  python tests/golden/make_golden.py
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))
sys.path.insert(0, str(HERE.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from helpers import make_params, make_walkers, oracle_config  # noqa: E402
from oracle import reference as R  # noqa: E402


def local_energy_case(name, B, seed=1898, param_seed=42):
    cfg = oracle_config(name)
    p = make_params(cfg, seed=param_seed)
    x = make_walkers(B, cfg.nelec, seed=seed)
    xt = torch.tensor(x, dtype=torch.float64)
    lp = R.batch_logpsi(p, cfg, xt).numpy()
    e, o = R.local_energy(p, cfg, xt)
    np.savez_compressed(
        HERE / f"local_energy_{name}.npz",
        config=json.dumps(cfg.__dict__),
        param_seed=param_seed,
        x=x,
        logpsi=lp,
        e_l=e.numpy(),
        kinetic=o["kinetic"].numpy(),
        potential=o["potential"].numpy(),
        lz=o["angular_momentum_z"].numpy(),
        lz2=o["angular_momentum_z_square"].numpy(),
        l2=o["angular_momentum_square"].numpy(),
    )
    print("wrote", name, e.numpy()[:2])


def mcmc_case(name, B=16, steps=4, width=0.3, seed=7):
    cfg = oracle_config(name)
    p = make_params(cfg)
    N = cfg.nelec
    x0 = make_walkers(B, N, seed=seed)
    g = np.random.default_rng(seed + 100)
    while True:
        normals = g.standard_normal((steps, B, N)).astype(np.float32)
        uph = g.random((steps, B, N)).astype(np.float32)
        uacc = g.random((steps, B)).astype(np.float32)
        x = torch.tensor(x0, dtype=torch.float64)
        lpf = lambda y: 2.0 * R.batch_logpsi(p, cfg, y).real  # noqa: E731
        lp = lpf(x)
        margins, accs, n_acc = [], [], np.zeros(B, np.int32)
        for s in range(steps):
            x2 = R.sph_sampling(x, normals[s].astype(np.float64), uph[s].astype(np.float64), width)
            lp2 = lpf(x2)
            margins.append(np.abs((lp2 - lp).numpy() - np.log(uacc[s].astype(np.float64))))
            x, lp, cond = R.mh_accept(x, x2, lp, lp2, uacc[s].astype(np.float64))
            n_acc += cond.numpy().astype(np.int32)
        if min(m.min() for m in margins) > 1e-3:  # no borderline accept decisions
            break
    noise = np.concatenate([normals, uph, uacc[..., None]], -1)  # [steps, B, 2N+1]
    np.savez_compressed(
        HERE / f"mcmc_{name}.npz",
        config=json.dumps(cfg.__dict__),
        x0=x0,
        noise=noise,
        width=np.float32(width),
        x=x.numpy(),
        lp=lp.numpy(),
        n_acc=n_acc,
    )
    print("wrote mcmc", name, n_acc)


if __name__ == "__main__":
    torch.set_num_threads(8)
    local_energy_case("C1", 8)
    local_energy_case("C2", 6)
    local_energy_case("MIX", 6)
    mcmc_case("C1")
    mcmc_case("C2", B=8, steps=3)
