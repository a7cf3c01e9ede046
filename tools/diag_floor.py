"""Per-observable errors of one golden fixture against its float64 values (and the f32 run).

usage: diag_floor.py TAG  (e.g. C4); env knobs (DH_GEMM=f32, DH_ATTN_MFMA=0, DH_DET_PC=0/1)
select kernel variants.  Prints max / p90 / median relative errors and the worst walkers."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from deephall_amd import hamiltonian  # noqa: E402
from helpers import cancellation_scales, make_params, to_device_params  # noqa: E402
from oracle import reference as R  # noqa: E402
from test_gpu_parity import build  # noqa: E402

tag = sys.argv[1]
g = np.load(ROOT / "tests" / "golden" / f"energy_{tag}.npz")
ocfg = R.OracleConfig(**json.loads(str(g["config"])))
ocfg.nspins = tuple(ocfg.nspins)
system, model = build(ocfg)
params = to_device_params(make_params(ocfg, seed=int(g["param_seed"])))
x = torch.tensor(g["x"], device="cuda")
e, o = hamiltonian.local_energy(model, system)(params, x)
got = {"e_l": e.cpu().numpy(), "kinetic": o["kinetic"].cpu().numpy(), "lz": o["angular_momentum_z"].cpu().numpy(),
       "lz2": o["angular_momentum_z_square"].cpu().numpy(), "l2": o["angular_momentum_square"].cpu().numpy()}
for k in got:
    ref, r32 = g[k], g[k + "32"]
    eh = np.abs(got[k] - ref) / np.maximum(np.abs(ref), 1.0)
    e32 = np.abs(r32 - ref) / np.maximum(np.abs(ref), 1.0)
    worst = np.argsort(eh)[-4:][::-1]
    print(f"{k:8s} HIP max {eh.max():.2e} p90 {np.percentile(eh, 90):.2e} med {np.median(eh):.2e} | "
          f"f32 max {e32.max():.2e} p90 {np.percentile(e32, 90):.2e} | worst {worst.tolist()} "
          f"{np.round(eh[worst] / np.maximum(e32[worst], 1e-12), 1).tolist()} x f32", flush=True)

# the worst walkers against the size of the terms that cancel in each observable (float64
# channel oracle): an error that is eps_f32 x that scale is the f32 floor of the walker
p64 = make_params(ocfg, seed=int(g["param_seed"]))
sc = cancellation_scales(p64, ocfg, g["x"])
for k, key in (("kinetic", "kinetic"), ("lz2", "angular_momentum_z_square"), ("l2", "angular_momentum_square"),
               ("lz", "angular_momentum_z")):
    ref, r32 = g[k], g[k + "32"]
    ah, a32 = np.abs(got[k] - ref), np.abs(r32 - ref)
    s = np.maximum(sc[key], 1.0)
    worst = np.argsort(ah / np.maximum(np.abs(ref), 1.0))[-3:][::-1]
    print(f"{k:8s} err/scale HIP max {np.max(ah / s):.2e} med {np.median(ah / s):.2e} | f32 max {np.max(a32 / s):.2e} "
          f"med {np.median(a32 / s):.2e} | worst walkers {worst.tolist()} |ref| {np.abs(ref[worst]).round(3).tolist()} "
          f"scale {s[worst].round(1).tolist()} HIP {ah[worst].tolist()} f32 {a32[worst].tolist()}", flush=True)
