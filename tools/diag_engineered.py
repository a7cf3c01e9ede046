"""Dump the worst walkers of the engineered-Psiformer known-answer test (GPU box)."""

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from deephall_amd import hamiltonian  # noqa: E402
from helpers import make_walkers, oracle_config, to_device_params  # noqa: E402
from test_gpu_parity import build  # noqa: E402
from test_oracle_kat import engineered_params  # noqa: E402

ocfg = oracle_config("C2", interaction_strength=0.0)
p = engineered_params(ocfg)
system, model = build(ocfg)
params = to_device_params(p)
x = make_walkers(4096, ocfg.nelec, seed=3, margin=0.3)
e, o = hamiltonian.local_energy(model, system)(params, torch.tensor(x, device="cuda"))
ke = o["kinetic"].cpu().numpy()
err = np.abs(ke - 3)
idx = np.argsort(-err)[:8]
np.savez("gpurun_out/engineered_worst.npz", x=x[idx], ke=ke[idx], l2=o["angular_momentum_square"].cpu().numpy()[idx])
print("worst", err[idx])
print("median err", np.median(err), "p99", np.percentile(err, 99))
# like-for-like with the float32 full-Hessian reference on the first 300 walkers
xs = torch.tensor(x[:300], dtype=torch.float64)
st = torch.sin(xs[..., 0])
geo = (ocfg.Q**2 / st**2).sum(-1).numpy() / (2 * ocfg.r**2)
rh = torch.stack([torch.sin(xs[..., 0]) * torch.cos(xs[..., 1]), torch.sin(xs[..., 0]) * torch.sin(xs[..., 1]), torch.cos(xs[..., 0])], -1)
dmin = (torch.cdist(rh, rh) + 9 * torch.eye(6)).amin(dim=(1, 2)).numpy()
e300 = np.abs(ke[:300] - 3) / np.maximum(3, geo)
print("gpu first300: max sep", e300[dmin > 0.3].max(), "median", np.median(e300), "p99", np.percentile(e300, 99))
np.save("gpurun_out/eng_gpu_err.npy", e300)
