"""Ring depth of the split-bf16 log-psi GEMMs (gemm_x6d_kernel ST): microseconds per launch
and max error vs float64 on the C2 log-psi shapes (24576 rows), GPU box.
  plain GEMM: variants 44 / 46 (ST 2) vs 70-75 (ST 4-5)
  LayerNorm GEMM: nw 1 (96 rows, ST 3) vs 5 / 6 (ST 5 / 4), 7 (64 rows, ST 5)"""

import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from deephall_amd import _lib  # noqa: E402

lib = _lib.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 24576
K = 256
rp = (rows + 767) // 768 * 768
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
X = torch.randn(rp, K, device="cuda")


def timed(fn, reps=50):
    for _ in range(5):
        assert fn() == 0, lib.dh_last_error()
    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    z.record()
    torch.cuda.synchronize()
    return 1e3 * a.elapsed_time(z) / reps


out = {}
for n in (256, 768, 192):
    W = torch.randn(K, n, device="cuda") / 16
    ldn = lib.dh_debug_x6_plane_rows(n)
    Wp = torch.empty(3 * ldn * K, dtype=torch.int16, device="cuda")
    assert lib.dh_debug_split_planes(p(W.t().contiguous()), K, n, K, p(Wp), s) == 0
    b = torch.randn(n, device="cuda")
    ref = (X[:rows].double() @ W.double() + b.double())
    for v in (-1, 44, 46, 70, 71, 72, 73, 74, 75):
        Y = torch.zeros(rp, n, device="cuda")
        us = timed(lambda: lib.dh_debug_gemm_x6(v, p(X), K, p(Wp), ldn, p(b), None, n, p(Y), n, rows, n, K, 1, s))
        err = ((Y[:rows].double() - ref).abs().max() / ref.abs().max()).item()
        out[f"gemm n={n} v={v}"] = {"us": round(us, 2), "tflops": round(2 * rows * n * K / us / 1e6, 1),
                                    "max_rel_err": err}
D = 256
W = torch.randn(K, D, device="cuda") / 16
ldp = lib.dh_debug_x6_plane_rows(D)
Wp = torch.empty(3 * ldp * K, dtype=torch.int16, device="cuda")
assert lib.dh_debug_split_planes(p(W.t().contiguous()), K, D, K, p(Wp), s) == 0
b = torch.randn(D, device="cuda")
ln = torch.cat([torch.ones(D), torch.zeros(D)]).cuda()
h0 = torch.randn(rp, D, device="cuda")
for mode in (0, 1):
    Xm = X if mode == 0 else h0
    z = Xm[:rows].double() @ W.double() + b.double()
    pre = h0[:rows].double() + (z if mode == 0 else torch.tanh(z))
    mu = pre.mean(-1, keepdim=True)
    ref = (pre - mu) / torch.sqrt(((pre - mu) ** 2).mean(-1, keepdim=True) + 1e-5)
    for nw in (1, 5, 6, 7):
        h = h0.clone()
        assert lib.dh_debug_gemm_x6_ln(mode, nw, p(Xm), K, p(Wp), ldp, p(b), p(ln), p(h), rows, K, s) == 0
        torch.cuda.synchronize()
        err = (h[:rows].double() - ref).abs().max().item()
        hh = h0.clone()
        us = timed(lambda: lib.dh_debug_gemm_x6_ln(mode, nw, p(Xm), K, p(Wp), ldp, p(b), p(ln), p(hh), rows, K, s))
        out[f"ln mode={mode} nw={nw}"] = {"us": round(us, 2), "max_abs_err": err}
print(json.dumps(out, indent=1))
