"""One chained log-psi layer tail shape, launched 20 times (GPU box, for rocprofv3 --pmc):
python tools/chain_one.py [rows] [n3]."""

import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from deephall_amd import _lib  # noqa: E402

lib = _lib.load()
K = D = 256
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 24576
n3 = int(sys.argv[2]) if len(sys.argv) > 2 else 768
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)


def p(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def planes(W, n):
    ldp = lib.dh_debug_x6_plane_rows(n)
    Wp = torch.empty(3 * ldp * K, dtype=torch.int16, device="cuda")
    assert lib.dh_debug_split_planes(p(W.t().contiguous()), K, n, K, p(Wp), s) == 0
    return Wp, ldp


rp = (rows + 767) // 768 * 768
Wp1, ldp = planes(torch.randn(K, D, device="cuda") / 16, D)
Wp2, _ = planes(torch.randn(K, D, device="cuda") / 16, D)
Wp3, ldp3 = planes(torch.randn(K, n3, device="cuda") / 16, n3)
b = torch.randn(max(n3, D), device="cuda")
ln = torch.cat([torch.ones(D), torch.zeros(D)]).cuda()
X1, h = torch.randn(rp, K, device="cuda"), torch.randn(rp, D, device="cuda")
Y = torch.empty(rp, n3, device="cuda")
for _ in range(20):
    assert lib.dh_debug_chain_x6(p(X1), p(Wp1), ldp, p(b), p(ln), p(Wp2), ldp, p(b), p(ln), p(Wp3), ldp3, p(b), n3,
                                 p(Y), n3, p(h), rows, s) == 0
torch.cuda.synchronize()
print("ok")
