"""Time (HIP events) the fused channel GEMM + LayerNorm kernel at a hot-path shape, or run it
a few times for rocprofv3 --pmc.  Usage: python tools/lnch_one.py N B mode reps"""
import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from deephall_amd import _lib  # noqa: E402

N, B, mode, reps = (int(a) for a in sys.argv[1:5])
lib = _lib.load()
p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
Cc, D = 2 * N + 5, 256
ne = B * N
rows = ne * Cc
X = torch.randn(rows, D, device="cuda")
h0 = torch.randn(rows, D, device="cuda")
h = h0.clone()
Wt = torch.randn(256, 256, device="cuda") / 16
ldp = lib.dh_debug_x6_plane_rows(256)
Wp = torch.empty(3 * ldp * 256, dtype=torch.int16, device="cuda")
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
assert lib.dh_debug_split_planes(p(Wt), 256, 256, 256, p(Wp), s) == 0
b = torch.randn(256, device="cuda") * 0.1
ln = torch.cat([torch.ones(256, device="cuda"), torch.zeros(256, device="cuda")])
th = torch.rand(ne, device="cuda") * 3.0 + 0.07
ph = torch.rand(ne, device="cuda") * 6.28
geo = torch.stack([th.sin(), th.cos(), ph.sin(), ph.cos()], 1).contiguous()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
for i in range(reps + 1):
    h.copy_(h0)
    if i:
        ev[2 * i - 2].record()
    assert lib.dh_debug_gemm_lnch(N, mode, p(X), p(Wp), ldp, p(b), p(ln), p(geo), p(h), ne, s) == 0
    if i:
        ev[2 * i - 1].record()
torch.cuda.synchronize()
ts = [ev[2 * i].elapsed_time(ev[2 * i + 1]) * 1e3 for i in range(reps)]
print(f"gemm_lnch N={N} B={B} mode={mode}: {sum(ts) / len(ts):.1f} us per launch (min {min(ts):.1f})")
if hasattr(lib, "dh_debug_lnch_stamps"):  # LNCH_STAMP=1 diagnostic build: phase breakdown of the last launch
    import numpy as np

    nwg = min((ne + 15) // 16, 4096)
    buf = (C.c_ulonglong * (4096 * 10))()
    assert lib.dh_debug_lnch_stamps(buf, 4096 * 10) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 10)[:nwg].astype(np.float64)
    clk = (st[:, 6] - st[:, 0]) / ((st[:, 9] - st[:, 8]) / 100e6)  # shader clock, Hz
    f = np.median(clk)
    names = ["prologue", "k loop", "residual", "reduce 1", "reduce 2", "LN + stores"]
    d = np.diff(st[:, :7], axis=1) / f * 1e6
    print(f"stamps: clock {f / 1e9:.2f} GHz, {nwg} workgroups, per-WG span {np.median((st[:, 6] - st[:, 0]) / f * 1e6):.1f} us "
          f"(launch span {(st[:, 9].max() - st[:, 8].min()) / 100:.1f} us)")
    for i, n in enumerate(names):
        print(f"  {n:12s} median {np.median(d[:, i]):7.2f} us  p90 {np.percentile(d[:, i], 90):7.2f}")
