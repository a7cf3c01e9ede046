"""Log-psi GEMM + LayerNorm forms on the C2 shape (24576 x 256 x 256), GPU box: microseconds
per launch of the split-bf16 GEMM alone, the split-bf16 GEMM with the LayerNorm epilogue
(tile heights 96 / 128) and the exact-f32 GEMM with the LayerNorm epilogue."""

import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from deephall_amd import _lib  # noqa: E402

lib = _lib.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 24576
K = D = 256
rp = (rows + 767) // 768 * 768
X = torch.randn(rp, K, device="cuda")
W = torch.randn(K, D, device="cuda") / 16
Wt = W.t().contiguous()
b = torch.randn(D, device="cuda")
ln = torch.cat([torch.ones(D), torch.zeros(D)]).cuda()
h = torch.randn(rp, D, device="cuda")
Y = torch.empty(rp, D, device="cuda")
ldp = lib.dh_debug_x6_plane_rows(D)
Wp = torch.empty(3 * ldp * K, dtype=torch.int16, device="cuda")
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)


def p(t):
    return C.c_void_p(t.data_ptr())


assert lib.dh_debug_split_planes(p(Wt), K, D, K, p(Wp), s) == 0


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


flops = 2.0 * rows * D * K
for n in (256, 768, 192):
    Wn = torch.randn(K, n, device="cuda") / 16
    ldn = lib.dh_debug_x6_plane_rows(n)
    Wpn = torch.empty(3 * ldn * K, dtype=torch.int16, device="cuda")
    assert lib.dh_debug_split_planes(p(Wn.t().contiguous()), K, n, K, p(Wpn), s) == 0
    bn = torch.randn(n, device="cuda")
    Yn = torch.empty(rp, n, device="cuda")
    fl = 2.0 * rows * n * K
    for v in (-1, 44, 46, 60, 61, 62):
        us = timed(lambda: lib.dh_debug_gemm_x6(v, p(X), K, p(Wpn), ldn, p(bn), None, n, p(Yn), n, rows, n, K, 1, s))
        print(f"x6 gemm {rows}x{n}x{K} variant {v:3d}: {us:7.1f} us  {fl / us / 1e6:6.1f} TF/s")
for nw in (1, 2, 3, 4):
    for mode in (0, 1):
        us = timed(lambda: lib.dh_debug_gemm_x6_ln(mode, nw, p(X), K, p(Wp), ldp, p(b), p(ln), p(h), rows, K, s))
        print(f"x6 gemm+LN nw={nw} mode={mode}: {us:7.1f} us  {flops / us / 1e6:6.1f} TF/s")
for mode in (0, 1):
    us = timed(lambda: lib.dh_debug_gemm_ln(mode, 0, p(X), K, p(Wt), K, p(b), p(ln), p(h), rows, K, s))
    print(f"f32 gemm+LN mode={mode}: {us:7.1f} us  {flops / us / 1e6:6.1f} TF/s")
