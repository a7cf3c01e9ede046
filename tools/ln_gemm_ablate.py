"""Log-psi GEMM + LayerNorm (mode 1: h = LN(h + tanh(h W + b))) at the walker-row counts of
C2 / C4 / C5 (B = 4096 x N = 6 / 10 / 20), GPU box: microseconds per launch of the production
form and of its ablations (launch_gemm_x6_ln codes 32-41; caller pads rows to 768):
  abl 1 no DMA / barriers, 2 + no split, 3 + no LDS reads, 4 MFMAs only, 5 full loop no epilogue,
  6 epilogue without the row reductions, 7 epilogue without tanh."""

import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from deephall_amd import _lib  # noqa: E402

lib = _lib.load()
K = D = 256
FORMS = {
    "prod": 0,
    "64r": 2, "64r abl1": 32, "64r abl2": 33, "64r abl3": 34, "64r abl4": 35, "64r abl5": 40,
    "96r": 36, "96r abl4": 37, "96r abl5": 41, "96r noreduce": 42, "96r notanh": 43,
    "128r": 38, "128r abl4": 39,
}


def p(t):
    return C.c_void_p(t.data_ptr())


def timed(fn, reps=50):
    for _ in range(5):
        assert fn() == 0
    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    z.record()
    torch.cuda.synchronize()
    return 1e3 * a.elapsed_time(z) / reps


s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
W = torch.randn(K, D, device="cuda") / 16
ldp = lib.dh_debug_x6_plane_rows(D)
Wp = torch.empty(3 * ldp * K, dtype=torch.int16, device="cuda")
assert lib.dh_debug_split_planes(p(W.t().contiguous()), K, D, K, p(Wp), s) == 0
b = torch.randn(D, device="cuda")
ln = torch.cat([torch.ones(D), torch.zeros(D)]).cuda()
for rows in [int(a) for a in sys.argv[1:]] or [24576, 40960, 81920]:
    rp = (rows + 767) // 768 * 768
    h = torch.randn(rp, D, device="cuda")
    fl = 2.0 * rows * D * K
    line = []
    for name, nw in FORMS.items():
        us = timed(lambda: lib.dh_debug_gemm_x6_ln(1, nw, p(h), K, p(Wp), ldp, p(b), p(ln), p(h), rows, K, s))
        line.append(f"{name} {us:6.1f}us {fl / us / 1e6:5.1f}TF")
    print(f"rows {rows}: " + " | ".join(line), flush=True)
