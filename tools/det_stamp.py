"""Phase stamps of det_value_kernel (inside an MCMC step) and det_energy_wave_kernel (inside a
local-energy call) at the bench batch: build with  FILE=det.hip bash tools/build_variant.sh
det_stamp -DDET_STAMP=1  and run  DH_LIB_PATH=ab/det_stamp.so python tools/det_stamp.py [N] [B]
on the GPU box.  Mean over workgroups of each phase in shader-clock cycles (s_memtime)."""

import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from deephall_amd import PRNGKey, _lib, config, hamiltonian, make_mcmc_step, make_network  # noqa: E402
from helpers import make_walkers  # noqa: E402

NAMES = {0: ["envelope leaves + cartesian", "Jastrow", "orbital contraction", "elimination", "log-sum-exp + MCMC epilogue",
             "(end)"],
         1: ["geometry + first row loads", "envelope leaves + channel contraction", "B = Phi0^-1",
             "traces + sums", "f64 energy assembly"]}


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    lib = _lib.load()
    fn = lib.dh_debug_det_stamps
    fn.argtypes = [C.c_void_p, C.c_int]
    system = config.System(nspins=(N, 0), flux={6: 15, 3: 2, 10: 23, 20: 57}[N])
    model = make_network(system, config.Network())
    params = model.init(1, device="cuda")
    x = torch.tensor(make_walkers(B, N, seed=3), device="cuda")
    step = make_mcmc_step(model, batch_per_device=B, steps=2)
    el = hamiltonian.local_energy(model.apply, system)
    for r in range(3):
        step(params, x, PRNGKey(r), 0.1)
        el(params, x)
    torch.cuda.synchronize()
    WG, NS = 1024, 12
    buf = np.zeros(2 * WG * NS, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0
    st = buf.reshape(2, WG, NS).astype(np.int64)
    for slot, name in ((0, "det_value_kernel"), (1, "det_energy_wave_kernel")):
        t = st[slot]
        t = t[t[:, 0] > 0]
        if not len(t):
            print(f"== {name}: no stamps")
            continue
        last = max(i for i in range(NS) if (t[:, i] > 0).all())
        tot = (t[:, last] - t[:, 0]).mean()
        print(f"== {name}: {len(t)} workgroups, span {tot:.0f} cycles (stamps 0..{last})")
        for i in range(last):
            d = (t[:, i + 1] - t[:, i]).mean()
            nm = NAMES[slot][i] if i < len(NAMES[slot]) else f"phase {i}"
            print(f"   {nm:40s} {d:9.0f} cycles  {100 * d / tot:5.1f} %")


if __name__ == "__main__":
    main()
