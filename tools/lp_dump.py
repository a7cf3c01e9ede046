"""log psi of a fixed walker batch through the library named by DH_LIB_PATH, saved to a .npy
file, so two builds can be compared bitwise:  DH_LIB_PATH=ab/X.so python tools/lp_dump.py
out.npy [N] [B] [el].  Includes walkers with two coincident electrons (psi = 0).  With "el"
the local energies of the same walkers are saved instead."""

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from deephall_amd import config, make_network  # noqa: E402
from helpers import make_walkers  # noqa: E402


def main():
    out = sys.argv[1]
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    system = config.System(nspins=(N, 0), flux={6: 15, 3: 2, 10: 23, 20: 57}[N])
    model = make_network(system, config.Network())
    params = model.init(1, device="cuda")
    x = make_walkers(B, N, seed=5)
    x[::97, 1] = x[::97, 0]  # coincident electrons
    lp = model.apply(params, torch.tensor(x, device="cuda"))
    res = lp.detach().cpu().numpy()
    if len(sys.argv) > 4 and sys.argv[4] == "el":  # the local energies of the same walkers instead
        from deephall_amd import hamiltonian
        el = hamiltonian.local_energy(model.apply, system)(params, torch.tensor(x, device="cuda"))
        e, o = el
        cols = [e.real, e.imag, o["kinetic"].real, o["kinetic"].imag, o["potential"], o["angular_momentum_z"],
                o["angular_momentum_z_square"], o["angular_momentum_square"]]
        res = torch.stack([c.float() for c in cols], 1).detach().cpu().numpy()
    np.save(out, res)
    print(out, "non-finite:", int((~np.isfinite(res)).sum()))


if __name__ == "__main__":
    main()
