"""Run the local energy a few times (profiling target for rocprofv3 --pmc).

usage: run_el.py [B] [reps]; NSPINS="6 0" FLUX=15 select the system (default C2)."""

import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from deephall_amd import config  # noqa: E402
from deephall_amd.hamiltonian import _run_local_energy  # noqa: E402
from deephall_amd.networks import make_network  # noqa: E402
from deephall_amd.random import Key, PRNGKey  # noqa: E402
from deephall_amd.train import init_guess  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
nspins = tuple(int(v) for v in os.environ.get("NSPINS", "6 0").split())
flux = int(os.environ.get("FLUX", "15"))
model = make_network(config.System(nspins=nspins, flux=flux), config.Network())
params = model.init(PRNGKey(42), device="cuda")
x = init_guess(Key(1), B, sum(nspins), "cuda", network=model)
for _ in range(reps):
    _run_local_energy(model, params, x)
torch.cuda.synchronize()
print("done")
