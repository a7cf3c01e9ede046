import sys, numpy as np, torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from test_gpu_lnch import run, rel, OBS
from test_gpu_parity import build
from helpers import make_params, make_walkers, to_device_params
from oracle import reference as R
for kw, B in [(dict(nspins=(2, 0), flux=3), 13), (dict(nspins=(3, 0), flux=2), 37), (dict(nspins=(6, 0), flux=15), 43)]:
    ocfg = R.OracleConfig(**kw)
    system, model = build(ocfg)
    params = to_device_params(make_params(ocfg, seed=11))
    N = sum(kw["nspins"])
    x = torch.tensor(make_walkers(B, N, seed=5 + B), device="cuda")
    split = run(model, system, params, x, "x6all_unfused")
    for rep in range(3):
        fused = run(model, system, params, x, "x6all")
        err = np.max([rel(fused[k], split[k]) for k in fused], axis=0)
        bad = np.where(err > 1e-3)[0]
        print(kw["nspins"], B, "rep", rep, "bad walkers", bad.tolist(), "electrons", [(b * N, b * N + N - 1) for b in bad], "err", err[bad].tolist(), flush=True)
