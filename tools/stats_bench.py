"""Time dh_energy_stats alone (B walkers, random E_L / observables with NaN walkers and
outliers) through the library named by DH_LIB_PATH:  python tools/stats_bench.py [B] [calls]
[out.npy] [penalties].  Ablation builds (STATS_ABL) show where the single-workgroup kernel's
time goes; out.npy (the DH_STAT_* vector) lets two builds be compared bitwise."""

import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT)]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from deephall_amd import _lib  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    lib = _lib.load()
    g = torch.Generator().manual_seed(0)
    e_l = torch.randn(B, 2, generator=g)
    obs = torch.randn(B, 8, generator=g)
    e_l[::97, 0] = float("nan")
    e_l[5::131, 1] = 1e6
    obs[3::89, 5] = -5e4
    e_l = torch.round(e_l * 64) / 64  # ties
    e_l, obs = e_l.cuda(), obs.cuda()
    pen = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    nacc = torch.randint(0, 10, (B,), dtype=torch.int32, generator=g).cuda()
    out = torch.empty(_lib.DH_NSTATS, dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    args = (None, C.c_void_p(e_l.data_ptr()), C.c_void_p(obs.data_ptr()), C.c_void_p(nacc.data_ptr()), B, 10, pen,
            C.c_void_p(out.data_ptr()), C.c_void_p(st))
    for _ in range(10):
        assert lib.dh_energy_stats(*args) == 0
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(calls):
        lib.dh_energy_stats(*args)
    t1.record()
    torch.cuda.synchronize()
    if len(sys.argv) > 3:
        np.save(sys.argv[3], out.cpu().numpy())
    print(f"B={B} pen={pen} dh_energy_stats {1000 * t0.elapsed_time(t1) / calls:.1f} us per call ({os.environ.get('DH_LIB_PATH', 'in-tree')})")


if __name__ == "__main__":
    import os
    main()
