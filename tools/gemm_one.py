"""Run one GEMM variant on one C2 hot-path shape a few times (for rocprofv3 --pmc).

variant < 200: dh_debug_gemm (>= 100: NT kernels); variant >= 200: split-bf16 kernel
variant - 200 through dh_debug_gemm_x6 (199 = automatic choice)."""
import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from deephall_amd import _lib  # noqa: E402

v, rows, n, K, reps = (int(a) for a in sys.argv[1:6])
lib = _lib.load()
p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
rp = (rows + 255) // 256 * 256
X = torch.randn(rp, K, device="cuda")
W = torch.randn(K, n, device="cuda") / 16
Wt = torch.zeros((n + 255) // 256 * 256, K, device="cuda")
Wt[:n] = W.t()
Y = torch.empty(rp, n, device="cuda")
b = torch.randn(n, device="cuda")  # a bias, as on the hot path
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
null = C.c_void_p(0)
if v >= 199:
    ldp = lib.dh_debug_x6_plane_rows(n)
    Wp = torch.empty(3 * ldp * K, dtype=torch.int16, device="cuda")
    assert lib.dh_debug_split_planes(p(Wt), K, n, K, p(Wp), s) == 0
    for _ in range(reps):
        assert lib.dh_debug_gemm_x6(v - 200, p(X), K, p(Wp), ldp, p(b), null, 0, p(Y), n, rows, n, K, 1, s) == 0
else:
    Wa, ldw = (Wt, K) if v >= 100 else (W, n)
    for _ in range(reps):
        assert lib.dh_debug_gemm(v, p(X), K, p(Wa), ldw, p(b), null, 0, p(Y), n, rows, n, K, 1, s) == 0
torch.cuda.synchronize()
