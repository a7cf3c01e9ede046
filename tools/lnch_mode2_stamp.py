"""Phase stamps of gemm_lnch MODE 2 (layer 1 whole) inside the C2 local energy: run with a
LNCH_STAMP=1 LNCH_STAMP_MODE=2 build (tools/build_variant.sh) through DH_LIB_PATH.
usage: python tools/lnch_mode2_stamp.py [B]"""
import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from deephall_amd import _lib, config, hamiltonian, make_network  # noqa: E402
from deephall_amd.random import Key, PRNGKey  # noqa: E402
from deephall_amd.train import init_guess  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
system = config.System(nspins=(6, 0), flux=15)
model = make_network(system, config.Network())
params = model.init(PRNGKey(7), device="cuda")
x = init_guess(Key(3), B, 6, "cuda", network=model)
for _ in range(3):
    hamiltonian.local_energy(model, system)(params, x)
torch.cuda.synchronize()
lib = _lib.load()
NS = 16
buf = (C.c_ulonglong * (4096 * NS))()
assert lib.dh_debug_lnch_stamps(buf, 4096 * NS) == 0
nwg = min((B * 6 + 15) // 16, 4096)
st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, NS)[:nwg].astype(np.float64)
f = np.median((st[:, 6] - st[:, 0]) / ((st[:, 9] - st[:, 8]) / 100e6))
order = [(0, 1, "prologue"), (1, 2, "pass 1 (o~ U)"), (2, 4, "f W0 + reduce means"), (4, 5, "zh + reduce 2"),
         (5, 10, "scalars + r rows"), (10, 11, "pass V"), (11, 12, "tanh_ch"), (12, 13, "pass B + barrier"),
         (13, 14, "LN2 reductions"), (14, 6, "LN2 + stores")]
print(f"MODE 2 stamps: clock {f / 1e9:.2f} GHz, {nwg} workgroups, per-WG span {np.median((st[:, 6] - st[:, 0]) / f * 1e6):.1f} us")
for a, b, n in order:
    d = (st[:, b] - st[:, a]) / f * 1e6
    print(f"  {n:22s} median {np.median(d):7.2f} us  p90 {np.percentile(d, 90):7.2f}")
