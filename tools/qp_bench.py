"""Laughlin quasiparticle local energy: native kernel (laughlin.hip) vs the callable route
(torch.func derivatives of the reference's slogdet form).  Prints one line per N."""
import sys
import time

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from deephall_amd import config, hamiltonian, make_network  # noqa: E402
from deephall_amd.networks import LaughlinQuasiparticle  # noqa: E402
from helpers import make_walkers  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


for N, B in ((4, 4096), (6, 4096), (8, 4096), (10, 4096), (16, 4096)):
    flux = 3 * (N - 1) - 1
    system = config.System(nspins=(N, 0), flux=flux, lz_center=1.0)
    net = config.Network()
    net.type = config.NetworkType.laughlin
    model = make_network(system, net)
    x = torch.tensor(make_walkers(B, N, seed=5, margin=0.05), device="cuda")
    p = model.init(0, device="cuda")
    el = hamiltonian.local_energy(model, system)
    tn = timed(lambda: el(p, x), 10)
    qp = LaughlinQuasiparticle(flux=flux, nspins=(N, 0), excitation_lz=1.0, system=system)
    elq = hamiltonian.local_energy(qp, system)
    tc = timed(lambda: elq({}, x), 2) if N <= 10 else float("nan")
    print(f"quasiparticle N={N:2d} B={B}: native {tn * 1e3:8.3f} ms ({B / tn:,.0f} E_L/s)   "
          f"callable {tc * 1e3:9.2f} ms   ratio {tc / tn:6.1f}x", flush=True)
