"""Layer-by-layer diagnostic: GPU trunk activations vs the channel oracle (GPU box only)."""

from __future__ import annotations

import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from deephall_amd import config, make_network  # noqa: E402
from deephall_amd.networks.psiformer import _ptr, _stream  # noqa: E402
from helpers import make_params, make_walkers, oracle_config, to_device_params  # noqa: E402
from oracle import channels as CH  # noqa: E402
from oracle import reference as R  # noqa: E402


def run(name, B=3):
    ocfg = oracle_config(name)
    p64 = make_params(ocfg)
    x = make_walkers(B, ocfg.nelec)
    sysc = config.System(nspins=ocfg.nspins, flux=ocfg.flux)
    net = config.Network()
    net.psiformer.num_heads, net.psiformer.heads_dim = ocfg.num_heads, ocfg.heads_dim
    net.psiformer.num_layers, net.psiformer.determinants = ocfg.num_layers, ocfg.determinants
    model = make_network(sysc, net)
    params = to_device_params(p64)
    xd = torch.tensor(x, device="cuda")
    h = model.prepare(params, xd.device)
    N, D = ocfg.nelec, ocfg.num_heads * ocfg.heads_dim
    for op in (0, 1):
        Cn = 1 if op == 0 else 2 * N + 5
        nb = h.lib.dh_workspace_bytes(h.h, B, op)
        ws = h.workspace(nb)
        rc = h.lib.dh_debug_trunk(h.h, _ptr(xd), B, op, _ptr(ws), ws.numel(), _stream(xd.device))
        assert rc == 0, h.lib.dh_last_error()
        torch.cuda.synchronize()
        wf = ws.view(torch.float32)
        rows = B * N * Cn
        hg = wf[: rows * D].reshape(B, N, Cn, D).double().cpu()
        X, _ = CH.trunk_channels(p64, ocfg, torch.tensor(x, dtype=torch.float64))
        Xr = X[:, :, :Cn]
        err = (hg - Xr).abs().amax(dim=(0, 1, 3))
        scale = Xr.abs().amax(dim=(0, 1, 3))
        print(f"{name} op={op} trunk max|err| per channel:", [f"{e:.1e}/{s:.1e}" for e, s in zip(err, scale)])
    lp = model.apply(params, xd).cpu()
    ref = R.batch_logpsi(p64, ocfg, torch.tensor(x, dtype=torch.float64))
    print(name, "logpsi gpu", lp.numpy(), "\n   ref", ref.numpy())
    from deephall_amd import hamiltonian

    e, o = hamiltonian.local_energy(model, sysc)(params, xd)
    lp2, ke, o2, raw = CH.local_energy(p64, ocfg, torch.tensor(x, dtype=torch.float64))
    print(name, "KE gpu", o["kinetic"].cpu().numpy(), "\n   ref", ke.numpy())
    for k in ("angular_momentum_z", "angular_momentum_z_square", "angular_momentum_square"):
        print("  ", k, o[k].cpu().numpy(), o2[k].numpy())


if __name__ == "__main__":
    for n in sys.argv[1:] or ["C1", "C2"]:
        run(n)
