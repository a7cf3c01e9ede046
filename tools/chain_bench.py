"""Chained log-psi layer tail (dh_debug_chain_x6) at the C2 / C4 walker rows, GPU box:
microseconds per launch and algorithmic TF/s (2 rows 256 (512 + n3) flops), beside the
separate kernels (two LayerNorm GEMMs + the plain GEMM).  DH_CHAIN=2 selects the LDS-ring
form of the chain."""

import ctypes as C
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from deephall_amd import _lib  # noqa: E402

lib = _lib.load()
K = D = 256


def p(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def timed(fn, reps=30):
    for _ in range(3):
        assert fn() == 0
    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    z.record()
    torch.cuda.synchronize()
    return 1e3 * a.elapsed_time(z) / reps


s = C.c_void_p(torch.cuda.current_stream().cuda_stream)


def planes(W, n):
    ldp = lib.dh_debug_x6_plane_rows(n)
    Wp = torch.empty(3 * ldp * K, dtype=torch.int16, device="cuda")
    assert lib.dh_debug_split_planes(p(W.t().contiguous()), K, n, K, p(Wp), s) == 0
    return Wp, ldp


W1, W2 = (torch.randn(K, D, device="cuda") / 16 for _ in range(2))
Wp1, ldp = planes(W1, D)
Wp2, _ = planes(W2, D)
b = torch.randn(3 * D, device="cuda")
ln = torch.cat([torch.ones(D), torch.zeros(D)]).cuda()
form = "ring" if os.environ.get("DH_CHAIN") == "2" else "reg"
for rows in [int(a) for a in sys.argv[1:]] or [24576, 40960]:
    rp = (rows + 767) // 768 * 768
    X1 = torch.randn(rp, K, device="cuda")
    h = torch.randn(rp, D, device="cuda")
    for n3 in (768, 192, 480):
        W3 = torch.randn(K, n3, device="cuda") / 16
        Wp3, ldp3 = planes(W3, n3)
        Y = torch.empty(rp, n3, device="cuda")
        fl = 2.0 * rows * 256 * (512 + n3)
        us = timed(lambda: lib.dh_debug_chain_x6(p(X1), p(Wp1), ldp, p(b), p(ln), p(Wp2), ldp, p(b), p(ln), p(Wp3),
                                                 ldp3, p(b), n3, p(Y), n3, p(h), rows, s))
        us2 = timed(lambda: lib.dh_debug_chain_x6(p(X1), p(Wp1), ldp, p(b), p(ln), p(Wp2), ldp, p(b), p(ln), None,
                                                  0, None, 0, None, 0, p(h), rows, s))

        def sep():
            r = lib.dh_debug_gemm_x6_ln(0, 0, p(X1), K, p(Wp1), ldp, p(b), p(ln), p(h), rows, K, s)
            r |= lib.dh_debug_gemm_x6_ln(1, 0, p(h), K, p(Wp2), ldp, p(b), p(ln), p(h), rows, K, s)
            r |= lib.dh_debug_gemm_x6(-1, p(h), K, p(Wp3), ldp3, p(b), None, 0, p(Y), n3, rows, n3, K, 1, s)
            return r

        us3 = timed(sep)
        print(f"rows {rows} n3 {n3:4d} [{form}]: chain {us:6.1f} us {fl / us / 1e6:5.1f} TF/s | "
              f"P1+P2 only {us2:6.1f} us | separate {us3:6.1f} us", flush=True)
