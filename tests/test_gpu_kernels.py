"""GPU unit tests of the GEMM kernels through the C ABI test hooks, against float64 torch.

Every tile variant of the register-staged GEMM (dh_debug_gemm 0..11), of the LDS-DMA
NT GEMM (100+), and the log-psi GEMM with the LayerNorm fused into its epilogue
(dh_debug_gemm_ln), on hot-path shapes including ragged rows / columns, the
channel-row bias rule (bias on rows r % C == 0 only) and the residual.
Tolerance: f32 products of K = 256 terms, |err| <= 2e-5 * (sum_k |x w| + 1).
"""

from __future__ import annotations

import ctypes as C

import numpy as np
import pytest
import torch

from deephall_amd import _lib

pytestmark = pytest.mark.gpu


def _p(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ref(X, W, b, R, rows, Cc):
    y = X[:rows].double() @ W.double()
    mask = (torch.arange(rows, device=X.device) % Cc == 0).double()[:, None]
    if b is not None:
        y = y + mask * b.double()
    if R is not None:
        y = y + R[:rows].double()
    scale = X[:rows].double().abs() @ W.double().abs() + 1.0
    return y, scale


SHAPES = [(1000, 256, 256, 17), (24576 // 8, 768, 256, 1), (777, 192, 256, 17), (300, 100, 256, 1)]
VARIANTS = list(range(12)) + [100 + v for v in (0, 1, 2, 3, 4, 5, 6, 7, 10, 11, 14, 15, 16, 17, 18)]
PERSISTENT = [120 + v for v in range(7)]  # write padding rows / columns (Y padded to 256 x 256)
VARIANTS += PERSISTENT


@pytest.mark.parametrize("variant", VARIANTS)
def test_gemm_variants(cuda, variant):
    lib = _lib.load()
    g = torch.Generator(device="cpu").manual_seed(variant)
    for rows, n, K, Cc in SHAPES:
        rp = (rows + 255) // 256 * 256
        X = torch.randn(rp, K, generator=g).cuda()
        W = (torch.randn(K, n, generator=g) / 16).cuda()
        b = torch.randn(n, generator=g).cuda()
        R = torch.randn(rp, n, generator=g).cuda() if n == 256 else None
        ldy = (n + 255) // 256 * 256 if variant in PERSISTENT else n
        Yb = torch.full((rp, ldy), float("nan"), device="cuda")
        Y = Yb[:, :n]
        if variant >= 100:
            Wt = torch.zeros((n + 255) // 256 * 256, K, device="cuda")
            Wt[:n] = W.t()
            rc = lib.dh_debug_gemm(variant, _p(X), K, _p(Wt), K, _p(b), _p(R), n, _p(Yb), ldy, rows, n, K, Cc,
                                   _stream())
        else:
            rc = lib.dh_debug_gemm(variant, _p(X), K, _p(W), n, _p(b), _p(R), n, _p(Y), n, rows, n, K, Cc, _stream())
        assert rc == 0
        torch.cuda.synchronize()
        ref, scale = _ref(X, W, b, R, rows, Cc)
        err = ((Y[:rows].double() - ref).abs() / scale).max().item()
        assert err < 2e-5, (variant, rows, n, err)
        if variant not in PERSISTENT:
            assert torch.isnan(Y[rows:]).all()  # rows past `rows` untouched


X6_VARIANTS = [-1, 0, 12, 40, 41, 43, 44, 45, 46, 50, 51, 52, 56, 57, 60, 61, 62, 76, 77, 78, 79, 80, 81, 82, 83, 84, 85, 90]


def _x6_planes(lib, W, n, K):
    ldp = lib.dh_debug_x6_plane_rows(n)
    Wt = W.t().contiguous()
    Wp = torch.empty(3 * ldp * K, dtype=torch.int16, device="cuda")
    assert lib.dh_debug_split_planes(_p(Wt), K, n, K, _p(Wp), _stream()) == 0
    return Wp, ldp


def test_x6_split_planes_exact(cuda):
    """The three bf16 planes sum exactly to the f32 weight (and zero-pad rows >= ncols)."""
    lib = _lib.load()
    g = torch.Generator(device="cpu").manual_seed(3)
    K, n = 256, 192
    W = (torch.randn(K, n, generator=g) * torch.exp(4 * torch.randn(K, n, generator=g))).cuda()
    Wp, ldp = _x6_planes(lib, W, n, K)
    torch.cuda.synchronize()
    planes = Wp.view(3, ldp, K)
    # bf16 bit pattern -> f32: shift into the high half
    f = (planes.to(torch.int32) << 16).view(torch.float32).double()
    recon = f[0] + f[1] + f[2]
    assert torch.equal(recon[:n], W.t().double())
    assert (recon[n:] == 0).all()
    # the terms shrink by 2^-8 each (round to nearest)
    assert (f[1].abs() <= f[0].abs() * 2.0**-8).all() and (f[2].abs() <= f[1].abs() * 2.0**-8).all()


@pytest.mark.parametrize("variant", X6_VARIANTS)
def test_gemm_x6_variants(cuda, variant):
    """Split-bf16 GEMM: correct contract (bias rule, residual, ragged rows / columns) and an
    error vs float64 at the level of the exact-f32 MFMA kernel on the same data."""
    lib = _lib.load()
    g = torch.Generator(device="cpu").manual_seed(100 + variant)
    for rows, n, K, Cc in SHAPES + [(4096, 480, 256, 1), (2048, 256, 256, 17)]:
        rp = (rows + 255) // 256 * 256
        X = torch.randn(rp, K, generator=g).cuda()
        W = (torch.randn(K, n, generator=g) / 16).cuda()
        b = torch.randn(n, generator=g).cuda() if rows != 2048 else None  # one case without a bias
        R = torch.randn(rp, n, generator=g).cuda() if n == 256 else None
        Wp, ldp = _x6_planes(lib, W, n, K)
        Yb = torch.full((rp, n), float("nan"), device="cuda")
        rc = lib.dh_debug_gemm_x6(variant, _p(X), K, _p(Wp), ldp, _p(b), _p(R), n, _p(Yb), n, rows, n, K, Cc,
                                  _stream())
        assert rc == 0
        # exact-f32 MFMA kernel on the same data
        Wt = torch.zeros((n + 255) // 256 * 256, K, device="cuda")
        Wt[:n] = W.t()
        Yf = torch.full((rp, n), float("nan"), device="cuda")
        assert lib.dh_debug_gemm(106, _p(X), K, _p(Wt), K, _p(b), _p(R), n, _p(Yf), n, rows, n, K, Cc, _stream()) == 0
        torch.cuda.synchronize()
        ref, scale = _ref(X, W, b, R, rows, Cc)
        err = ((Yb[:rows].double() - ref).abs() / scale).max().item()
        err_f32 = ((Yf[:rows].double() - ref).abs() / scale).max().item()
        assert err < 2e-5, (variant, rows, n, err)
        assert err <= 2.0 * err_f32 + 1e-8, (variant, rows, n, err, err_f32)
        assert torch.isnan(Yb[rows:]).all()


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("bm", [0, 32, 64, 96])
@pytest.mark.parametrize("rows", [96, 1000, 24576])
def test_gemm_layernorm_fused(cuda, mode, bm, rows):
    lib = _lib.load()
    g = torch.Generator(device="cpu").manual_seed(17 * mode + bm + rows)
    K, D = 256, 256
    rp = (rows + 767) // 768 * 768  # readable rows for every tile height (lcm of 256 and 96)
    X = torch.randn(rp, K, generator=g).cuda()
    W = (torch.randn(K, D, generator=g) / 16).cuda()
    Wt = W.t().contiguous()
    b = torch.randn(D, generator=g).cuda()
    ln = torch.cat([1.0 + 0.1 * torch.randn(D, generator=g), 0.1 * torch.randn(D, generator=g)]).cuda()
    h0 = torch.randn(rp, D, generator=g).cuda()
    if mode == 1:
        X = h0  # the MLP reads h and writes LN(h + tanh(h W + b)) over it
    h = h0.clone()
    Xin = h if mode == 1 else X
    assert lib.dh_debug_gemm_ln(mode, bm, _p(Xin), K, _p(Wt), K, _p(b), _p(ln), _p(h), rows, K, _stream()) == 0
    torch.cuda.synchronize()
    z = X[:rows].double() @ W.double() + b.double()
    y = h0[:rows].double() + (z if mode == 0 else torch.tanh(z))
    mu = y.mean(-1, keepdim=True)
    var = ((y - mu) ** 2).mean(-1, keepdim=True)
    ref = (y - mu) / torch.sqrt(var + 1e-5) * ln[:D].double() + ln[D:].double()
    err = (h[:rows].double() - ref).abs().max().item()
    assert err < 2e-4, err
    assert torch.equal(h[rows:], h0[rows:])  # padding rows untouched


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("nw", [0, 1, 2, 3, 4, 8])
@pytest.mark.parametrize("rows", [96, 1000, 24576, 40960])
def test_gemm_x6_layernorm_fused(cuda, mode, nw, rows):
    """Split-bf16 log-psi GEMM with the LayerNorm in its epilogue (in place over h): same
    contract and tolerance as the exact-f32 gemm_ln_kernel above, against float64."""
    lib = _lib.load()
    g = torch.Generator(device="cpu").manual_seed(23 * mode + nw + rows)
    K, D = 256, 256
    rp = (rows + 767) // 768 * 768
    X = torch.randn(rp, K, generator=g).cuda()
    W = (torch.randn(K, D, generator=g) / 16).cuda()
    Wp, ldp = _x6_planes(lib, W, D, K)
    b = torch.randn(D, generator=g).cuda()
    ln = torch.cat([1.0 + 0.1 * torch.randn(D, generator=g), 0.1 * torch.randn(D, generator=g)]).cuda()
    h0 = torch.randn(rp, D, generator=g).cuda()
    if mode == 1:
        X = h0
    h = h0.clone()
    Xin = h if mode == 1 else X
    assert lib.dh_debug_gemm_x6_ln(mode, nw, _p(Xin), K, _p(Wp), ldp, _p(b), _p(ln), _p(h), rows, K, _stream()) == 0
    torch.cuda.synchronize()
    z = X[:rows].double() @ W.double() + b.double()
    y = h0[:rows].double() + (z if mode == 0 else torch.tanh(z))
    mu = y.mean(-1, keepdim=True)
    var = ((y - mu) ** 2).mean(-1, keepdim=True)
    ref = (y - mu) / torch.sqrt(var + 1e-5) * ln[:D].double() + ln[D:].double()
    err = (h[:rows].double() - ref).abs().max().item()
    assert err < 2e-4, err
    assert torch.equal(h[rows:], h0[rows:])


@pytest.mark.parametrize("n3", [0, 768, 192, 18])
@pytest.mark.parametrize("rows", [96, 1000, 24576, 40960])
def test_chain_x6_matches_separate_kernels(cuda, n3, rows):
    """The chained log-psi layer tail (one launch: LN1 GEMM, LN2 GEMM, next linear map)
    against the separate split-bf16 kernels (same products in the same k order; the
    LayerNorm sums in another order: f32 rounding) and the float64 layer."""
    lib = _lib.load()
    g = torch.Generator(device="cpu").manual_seed(rows + n3)
    K = D = 256
    rp = (rows + 767) // 768 * 768
    X1 = torch.randn(rp, K, generator=g).cuda()
    h0 = torch.randn(rp, D, generator=g).cuda()
    W1, W2 = ((torch.randn(K, D, generator=g) / 16).cuda() for _ in range(2))
    b1, b2 = (torch.randn(D, generator=g).cuda() for _ in range(2))
    ln1, ln2 = (torch.cat([1.0 + 0.1 * torch.randn(D, generator=g), 0.1 * torch.randn(D, generator=g)]).cuda()
                for _ in range(2))
    Wp1, ldp = _x6_planes(lib, W1, D, K)
    Wp2, _ = _x6_planes(lib, W2, D, K)
    ldy = (n3 + 3) // 4 * 4 if n3 else 4
    if n3:
        W3 = (torch.randn(K, n3, generator=g) / 16).cuda()
        b3 = torch.randn(n3, generator=g).cuda()
        Wp3, ldp3 = _x6_planes(lib, W3, n3, K)
    else:
        W3 = b3 = Wp3 = None
        ldp3 = 0
    # separate kernels
    h_sep = h0.clone()
    assert lib.dh_debug_gemm_x6_ln(0, 0, _p(X1), K, _p(Wp1), ldp, _p(b1), _p(ln1), _p(h_sep), rows, K, _stream()) == 0
    assert lib.dh_debug_gemm_x6_ln(1, 0, _p(h_sep), K, _p(Wp2), ldp, _p(b2), _p(ln2), _p(h_sep), rows, K, _stream()) == 0
    Y_sep = torch.zeros(rp, ldy, device="cuda")
    if n3:
        assert lib.dh_debug_gemm_x6(-1, _p(h_sep), K, _p(Wp3), ldp3, _p(b3), None, 0, _p(Y_sep), ldy, rows, n3, K, 1,
                                    _stream()) == 0
    # chain
    h_ch = h0.clone()
    Y_ch = torch.zeros(rp, ldy, device="cuda")
    assert lib.dh_debug_chain_x6(_p(X1), _p(Wp1), ldp, _p(b1), _p(ln1), _p(Wp2), ldp, _p(b2), _p(ln2), _p(Wp3), ldp3,
                                 _p(b3), n3, _p(Y_ch), ldy, _p(h_ch), rows, _stream()) == 0
    torch.cuda.synchronize()
    assert (h_ch[:rows] - h_sep[:rows]).abs().max().item() < 4e-6
    assert torch.equal(h_ch[rows:], h0[rows:])  # padding rows untouched
    if n3:
        ys = Y_sep[:rows, :n3]
        assert (Y_ch[:rows, :n3] - ys).abs().max().item() < 4e-6 * max(1.0, ys.abs().max().item())
    # float64 layer
    def ln(y, p):
        mu = y.mean(-1, keepdim=True)
        return (y - mu) / torch.sqrt(((y - mu) ** 2).mean(-1, keepdim=True) + 1e-5) * p[:D].double() + p[D:].double()
    h1 = ln(h0[:rows].double() + X1[:rows].double() @ W1.double() + b1.double(), ln1)
    h2 = ln(h1 + torch.tanh(h1 @ W2.double() + b2.double()), ln2)
    assert (h_ch[:rows].double() - h2).abs().max().item() < 2e-4
    if n3:
        y = h2 @ W3.double() + b3.double()
        assert (Y_ch[:rows, :n3].double() - y).abs().max().item() < 2e-4 * max(1.0, y.abs().max().item())


def _env_leaf_f64(th, ph, M):
    """det.hip env_leaf in float64 (norm 1): [n][M][10] = e0, dth, dph, lb, d2th (re, im)."""
    th = th.astype(np.float64)[:, None]
    ph = ph.astype(np.float64)[:, None]
    ct32 = np.cos(th.astype(np.float32)).astype(np.float32)
    gauge = (np.float32(M - 1) * np.rint(np.float32(64.0) * ct32) * np.float32(1.0 / 128.0)).astype(np.float64)
    p = np.arange(M)[None, :].astype(np.float64)
    a, b = p, M - 1 - p
    m = 0.5 * (a - b) - gauge
    c, s = np.cos(0.5 * th), np.sin(0.5 * th)

    def pw(x, e):
        return np.where(e < 0, 0.0, np.power(x, np.maximum(e, 0)))

    R = pw(c, a) * pw(s, b)
    R1 = 0.5 * (b * pw(c, a + 1) * pw(s, b - 1) - a * pw(c, a - 1) * pw(s, b + 1))
    R2 = 0.25 * (b * (b - 1) * pw(c, a + 2) * pw(s, b - 2) - b * (a + 1) * R - a * (b + 1) * R
                 + a * (a - 1) * pw(c, a - 2) * pw(s, b + 2))
    cph, sph = np.cos(m * ph), np.sin(m * ph)
    st, ctd = np.sin(th), np.cos(th)
    e0 = (R * cph, R * sph)
    dth = (R1 * cph, R1 * sph)
    d2 = (R2 * cph, R2 * sph)
    dph = (-m * e0[1] / st, m * e0[0] / st)
    k2, cot = m * m / (st * st), ctd / st
    lb = (d2[0] - k2 * e0[0] + cot * dth[0], d2[1] - k2 * e0[1] + cot * dth[1])
    return np.stack([e0[0], e0[1], dth[0], dth[1], dph[0], dph[1], lb[0], lb[1], d2[0], d2[1]], -1)


@pytest.mark.parametrize("M", [16, 24, 58])
def test_env_leaf_powers(cuda, M):
    """The envelope leaves with integer powers by squaring (the production form of every
    determinant kernel, det.hip ipow_sq) against float64, beside the powf form: squaring
    carries about (e + popcount e) * 2^-24 relative error per power (e <= M - 1 = 57 at C5)
    where powf carries ~1 ulp.  Near the poles the leaves' own f32 formulas (m / sin, m^2 /
    sin^2, cot) dominate both forms' error (measured on the MI355X: max 1.8e-4 - 5.7e-4 of the
    component's scale for both at M = 16 .. 58), so the gate is relative: the squaring form's
    error distribution stays within that of powf (max 1.5x, p99 2x, plus 2e-6 of the scale)."""
    lib = _lib.load()
    g = np.random.default_rng(M)
    th = np.concatenate([g.uniform(1e-3, 0.15, 32), np.pi - g.uniform(1e-3, 0.15, 32), g.uniform(0.15, np.pi - 0.15, 64)])
    ph = g.uniform(0.0, 2 * np.pi, th.size)
    thph = torch.tensor(np.stack([th, ph], -1).astype(np.float32), device="cuda")
    th32, ph32 = thph[:, 0].cpu().numpy(), thph[:, 1].cpu().numpy()
    ref = _env_leaf_f64(th32, ph32, M)
    scale = np.abs(ref).max(axis=1, keepdims=True) + 1e-30  # per point and component, over p
    errs = {}
    for sq in (0, 1):
        out = torch.empty(th.size * M * 10, device="cuda")
        assert lib.dh_debug_env_leaf(_p(thph), th.size, M, sq, _p(out), _stream()) == 0
        torch.cuda.synchronize()
        got = out.cpu().numpy().reshape(th.size, M, 10).astype(np.float64)
        e = np.abs(got - ref) / scale
        errs[sq] = (np.median(e), np.percentile(e, 99), e.max())
    print(f"M={M}: env_leaf error / component scale (median, p99, max): powf {errs[0]}, squaring {errs[1]}")
    assert errs[1][2] <= 1.5 * errs[0][2] + 2e-6 and errs[1][1] <= 2.0 * errs[0][1] + 2e-6, errs
