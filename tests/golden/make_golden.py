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


def pole_walkers(B, N, seed):
    """init_guess walkers with electron 0 within 0.15 rad of the north pole and electron 1
    within 0.15 rad of the south pole (theta in [1e-3, 0.15]): the cot / 1/sin^2 terms of
    hamiltonian.py:121-159 are largest there, and the reference samples the poles freely."""
    g = np.random.default_rng(seed)
    x = R.init_guess_from_uniforms(g.random((B, N)), g.random((B, N)))
    t = 10 ** g.uniform(-3, np.log10(0.15), size=(B, 2))
    x[:, 0, 0] = t[:, 0]
    if N > 1:
        x[:, 1, 0] = np.pi - t[:, 1]
    return x.astype(np.float32)


def energy_case(tag, name, B, seed=1898, param_seed=42, pole=False, **over):
    """Golden local energies with the float64 oracle AND the same full-Hessian algorithm run
    in float32 (the reference's own arithmetic): the tests bound the kernels' error by the
    error of that float32 run (the f32 floor) per observable."""
    cfg = oracle_config(name, **over)
    p = make_params(cfg, seed=param_seed)
    x = pole_walkers(B, cfg.nelec, seed) if pole else make_walkers(B, cfg.nelec, seed=seed)
    xt = torch.tensor(x, dtype=torch.float64)
    lp = R.batch_logpsi(p, cfg, xt).numpy()
    e, o = R.local_energy(p, cfg, xt)
    p32 = {k: v.float() for k, v in p.items()}
    x32 = torch.tensor(x, dtype=torch.float32)
    lp32 = R.batch_logpsi(p32, cfg, x32).detach().numpy()
    e32, o32 = R.local_energy(p32, cfg, x32)
    out = dict(config=json.dumps(cfg.__dict__), param_seed=param_seed, x=x, logpsi=lp, e_l=e.detach().numpy(),
               logpsi32=lp32, e_l32=e32.detach().numpy())
    for key, k in (("kinetic", "kinetic"), ("potential", "potential"), ("lz", "angular_momentum_z"),
                   ("lz2", "angular_momentum_z_square"), ("l2", "angular_momentum_square")):
        out[key] = o[k].detach().numpy()
        out[key + "32"] = o32[k].detach().numpy()
    np.savez_compressed(HERE / f"energy_{tag}.npz", **out)
    print("wrote", tag, e.detach().numpy()[:2])


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


def round1():
    local_energy_case("C1", 8)
    local_energy_case("C2", 6)
    local_energy_case("MIX", 6)
    mcmc_case("C1")
    mcmc_case("C2", B=8, steps=3)


def round2():
    """Near-pole walkers, harmonic potential, explicit radius, C4 / C5 batches, each with
    the float32 run of the same full-Hessian algorithm beside the float64 one."""
    energy_case("C1_pole", "C1", 32, seed=31, pole=True)
    energy_case("C2_pole", "C2", 16, seed=32, pole=True)
    energy_case("MIX_pole", "MIX", 16, seed=33, pole=True)
    energy_case("C1_harmonic", "C1", 16, seed=34, interaction_type="harmonic", interaction_strength=0.7)
    energy_case("C2_harmonic_radius", "C2", 16, seed=35, interaction_type="harmonic", radius=2.5)
    energy_case("C2_radius", "C2", 16, seed=36, radius=3.1)
    energy_case("C2", "C2", 32, seed=37)
    energy_case("C4", "C4", 128, seed=38)  # 128 walkers: the p90 of a 32-walker batch is its 4th-worst walker
    energy_case("C5", "C5", 32, seed=39)
    mcmc_case("C4", B=16, steps=3)


def round4():
    """The f32-floor gate on real sample sizes (round-3 verdict, weak item 1): with 16-32
    walkers the "p90" is the 2nd-4th worst walker and a 1-ulp change of one kernel flipped
    the gate.  Same seeds as round 2, larger batches (new walkers), and "sparse"-orbital
    fixtures (blocks.py:52-62) beside the dense ones."""
    energy_case("C1_pole", "C1", 64, seed=31, pole=True)
    energy_case("C2_pole", "C2", 64, seed=32, pole=True)
    energy_case("MIX_pole", "MIX", 64, seed=33, pole=True)
    energy_case("C2", "C2", 256, seed=37)
    energy_case("C5", "C5", 128, seed=39)
    energy_case("C1_sparse", "C1", 96, seed=40, orbital="sparse")
    energy_case("C2_sparse", "C2", 64, seed=41, orbital="sparse")
    energy_case("MIX_sparse", "MIX", 64, seed=42, orbital="sparse")


def round6():
    """The injected-noise MCMC golden at N = 20 (round-5 verdict, weak 1c): the accept fused
    into the value kernel's epilogue and the N = 20 value kernel (det_value<MGV>) against
    mcmc.py:25-64 run by the float64 oracle."""
    mcmc_case("C5", B=8, steps=3)


if __name__ == "__main__":
    torch.set_num_threads(8)
    # python make_golden.py [round1] [round2] [round4] [round6]   (default: all; round4 rewrites
    # round 2's pole / C2 / C5 fixtures at the larger sizes)
    for part in sys.argv[1:] or ["round1", "round2", "round4", "round6"]:
        {"round1": round1, "round2": round2, "round4": round4, "round6": round6}[part]()
