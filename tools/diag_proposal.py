"""Proposal (sph_sampling) accuracy: GPU f32 vs the float64 oracle, accept-all noise."""

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from deephall_amd.mcmc import make_mcmc_step  # noqa: E402
from deephall_amd.random import Key  # noqa: E402
from helpers import make_params, make_walkers, oracle_config, to_device_params  # noqa: E402
from oracle import reference as R  # noqa: E402
from test_gpu_parity import build, cart_err  # noqa: E402

ocfg = oracle_config("C1")
system, model = build(ocfg)
params = to_device_params(make_params(ocfg))
B, N = 4096, 3
x0 = make_walkers(B, N, seed=4, margin=0.0)
g = np.random.default_rng(5)
noise = np.concatenate([g.standard_normal((1, B, N)), g.random((1, B, N)), np.zeros((1, B, 1))], -1).astype(np.float32)
step = make_mcmc_step(model, batch_per_device=B, steps=1)
xg, _ = step(params, torch.tensor(x0, device="cuda"), Key(0), 0.3, noise=torch.tensor(noise, device="cuda"))
xr = R.sph_sampling(torch.tensor(x0, dtype=torch.float64), noise[0, :, :N].astype(np.float64),
                    noise[0, :, N : 2 * N].astype(np.float64), 0.3).numpy()
x32 = R.sph_sampling(torch.tensor(x0), noise[0, :, :N], noise[0, :, N : 2 * N], 0.3).numpy()
xg = xg.cpu().numpy()
errs = np.array([cart_err(xg[b], xr[b]) for b in range(B)])
e32 = np.array([cart_err(x32[b], xr[b]) for b in range(B)])
print("gpu max", errs.max(), "median", np.median(errs), " torch-f32 max", e32.max())
for b in np.argsort(-errs)[:4]:
    print(b, errs[b], "x0", x0[b].tolist(), "gpu", xg[b].tolist(), "ref", xr[b].tolist(), "noise", noise[0, b].tolist())
