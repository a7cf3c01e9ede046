"""GEMM kernel variants on the shapes of the C2 hot path (GPU box): TFLOP/s + correctness."""

import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from deephall_amd import _lib  # noqa: E402

lib = _lib.load()
SHAPES = {
    "fwd_qkv": (24576, 768, 256, 1),
    "fwd_d": (24576, 256, 256, 1),
    "fwd_orb": (24576, 192, 256, 1),
    "el_qkv": (417792, 768, 256, 17),
    "el_d": (417792, 256, 256, 17),
    "el_m": (417792, 256, 256, 17),
    "el_orb": (417792, 192, 256, 17),
}


def p(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def run(variant, rows, ncols, K, Cc, reps=20, check=False, residual=False):
    rp = (rows + 255) // 256 * 256
    X = torch.randn(rp, K, device="cuda")
    W = torch.randn(K, ncols, device="cuda") / 16
    b = torch.randn(ncols, device="cuda")
    R = torch.randn(rp, ncols, device="cuda") if residual else None
    ldy = (ncols + 255) // 256 * 256 if 120 <= variant < 200 else ncols  # persistent: padded Y
    Yb = torch.empty(rp, ldy, device="cuda")
    Y = Yb[:, :ncols]
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    fn = lib.dh_debug_gemm
    if variant >= 200:  # split-bf16 kernels (variant 200 + v; 199 = automatic)
        ldp = lib.dh_debug_x6_plane_rows(ncols)
        Wt = W.t().contiguous()
        Wp = torch.empty(3 * ldp * K, dtype=torch.int16, device="cuda")
        assert lib.dh_debug_split_planes(p(Wt), K, ncols, K, p(Wp), s) == 0
        args = (variant - 200, p(X), K, p(Wp), ldp, p(b), p(R), ncols, p(Y), ncols, rows, ncols, K, Cc, s)
        fn = lib.dh_debug_gemm_x6
    elif variant >= 100:  # NT kernels take the transposed weight, rows padded to 256
        Wt = torch.zeros((ncols + 255) // 256 * 256, K, device="cuda")
        Wt[:ncols] = W.t()
        args = (variant, p(X), K, p(Wt), K, p(b), p(R), ncols, p(Yb), ldy, rows, ncols, K, Cc, s)
    else:
        args = (variant, p(X), K, p(W), ncols, p(b), p(R), ncols, p(Y), ncols, rows, ncols, K, Cc, s)
    assert fn(*args) == 0
    if check:
        ref = X[:rows].double() @ W.double()
        ref[torch.arange(rows, device="cuda") % Cc == 0] += b.double()
        if R is not None:
            ref += R[:rows].double()
        err = (Y[:rows].double() - ref).abs().max().item()
        assert err < 1e-3, err
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn(*args)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return ms, 2.0 * rows * ncols * K / (ms * 1e-3) / 1e12


if __name__ == "__main__":
    variants = [int(v) for v in sys.argv[1:]] or [0, 1, 2, 3, 4, 5]
    for name, (rows, n, k, cc) in SHAPES.items():
        line = [f"{name:8s}"]
        for v in variants:
            try:
                ms, tf = run(v, rows, n, k, cc, check=not (290 <= v < 300 or 286 <= v <= 289), residual=name in ("el_d", "fwd_d"))
                line.append(f"v{v}: {ms * 1e3:8.1f}us {tf:6.1f}TF")
            except AssertionError as e:
                line.append(f"v{v}: WRONG {e}")
        print("  ".join(line), flush=True)
