"""Local-energy time vs walker chunk size (workspace budget) on the GPU box.

Smaller chunks keep a chunk's activations (h, o, t, q|k|v) inside the 256 MB Infinity
Cache; larger chunks give the GEMMs more tiles.  usage: chunk_bench.py [B] [NSPINS FLUX]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from deephall_amd import config  # noqa: E402
from deephall_amd import _lib  # noqa: E402
from deephall_amd.networks.psiformer import _ptr, _stream  # noqa: E402
from deephall_amd.networks import make_network  # noqa: E402
from deephall_amd.random import Key, PRNGKey  # noqa: E402
from deephall_amd.train import init_guess  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
nspins = (int(sys.argv[2]), 0) if len(sys.argv) > 2 else (6, 0)
flux = int(sys.argv[3]) if len(sys.argv) > 3 else 15
model = make_network(config.System(nspins=nspins, flux=flux), config.Network())
params = model.init(PRNGKey(42), device="cuda")
x = init_guess(Key(1), B, sum(nspins), "cuda", network=model)
h = model.prepare(params, x.device)
e_l = torch.empty(B, 2, device="cuda")
obs = torch.empty(B, 8, device="cuda")
ws_all = torch.empty(h.lib.dh_workspace_bytes(h.h, B, 1), dtype=torch.uint8, device="cuda")


def _run_local_energy(model, params, x, ws_budget):
    ws = ws_all[:ws_budget]
    _lib.check(h.lib.dh_local_energy(h.h, _ptr(x), B, _ptr(e_l), _ptr(obs), _ptr(ws), ws.numel(), _stream(x.device)))


for chunk in (B, B // 2, B // 4, B // 8, B // 16):
    budget = h.lib.dh_workspace_bytes(h.h, chunk, 1)
    for _ in range(2):
        _run_local_energy(model, params, x, ws_budget=budget)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        _run_local_energy(model, params, x, ws_budget=budget)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print(f"chunk {chunk:5d} walkers, workspace {budget / 2**20:8.1f} MiB: {ms:7.3f} ms  {B / ms * 1e3:10.0f} E_L/s", flush=True)
