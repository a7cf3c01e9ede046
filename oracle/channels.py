"""TEST INFRASTRUCTURE ONLY — forward-mode (2N+5)-channel restatement of E_L.

This is the algorithm the HIP kernels implement, written in plain
batched torch so every intermediate tensor can be compared with the kernels.
It is an *independent* route to the quantities of deephall/hamiltonian.py:96-170:
instead of the full [N,2,N,2] Hessian (jax.hessian, hamiltonian.py:112-113) it
propagates, through every layer, the channels

    c = 0            value
    c = 1 .. 2N      first-order tangents along the scaled seeds
                     d_{2i} = e_theta_i,  d_{2i+1} = e_phi_i / sin(theta_i)
    c = 2N+1         Laplace-Beltrami channel  sum_c d_c^T H d_c + sum_i cot(theta_i) d/dtheta_i
    c = 2N+2 .. 2N+4 second derivative along the rigid-rotation flow about x, y, z

and assembles KE / Lz / Lz^2 / L^2 from them (DESIGN.md §3.4 derives that this is
algebraically identical to hamiltonian.py:115-169).

Layout of an activation bundle: [B, N, C, D] (walker, electron, channel, feature).
"""

from __future__ import annotations

import math

import numpy as np
import torch
from scipy import special as ss

from .reference import OracleConfig

DT = torch.float64


def _ctype(x):
    return torch.complex128 if x.dtype == torch.float64 else torch.complex64


def n_channels(N):
    return 2 * N + 5


def geometry(x):
    """Per-electron geometry. x [B,N,2] -> dict of [B,N] tensors and alpha [B,3,2N]."""
    th, ph = x[..., 0], x[..., 1]
    st, ct, sp, cp = torch.sin(th), torch.cos(th), torch.sin(ph), torch.cos(ph)
    B, N = th.shape
    r_hat = torch.stack([st * cp, st * sp, ct], -1)  # [B,N,3]
    th_hat = torch.stack([ct * cp, ct * sp, -st], -1)
    ph_hat = torch.stack([-sp, cp, torch.zeros_like(ph)], -1)
    alpha = torch.zeros(B, 3, 2 * N, dtype=x.dtype)
    alpha[:, :, 0::2] = ph_hat.permute(0, 2, 1)
    alpha[:, :, 1::2] = -th_hat.permute(0, 2, 1)
    return dict(th=th, ph=ph, st=st, ct=ct, sp=sp, cp=cp, r_hat=r_hat, th_hat=th_hat, ph_hat=ph_hat, alpha=alpha)


def u_dirs(X, alpha):
    """First-order part along the three flow directions: sum_t alpha[k,t] X[:,:,1+t]."""
    T = alpha.shape[-1]
    return torch.einsum("bkt,bn...td->bn...kd", alpha, X[:, :, 1 : 1 + T])


# ------------------------------------------------------------------ input layer


def input_channels(x, nspins):
    """Feature channels [B,N,C,4] of [cos th, sin th cos ph, sin th sin ph, s] (psiformer.py:51-60)."""
    g = geometry(x)
    B, N = x.shape[:2]
    C = n_channels(N)
    F = torch.zeros(B, N, C, 4, dtype=x.dtype)
    rh, th_h, ph_h = g["r_hat"], g["th_hat"], g["ph_hat"]
    perm = [2, 0, 1]  # feature order z, x, y
    spins = torch.tensor([1.0] * nspins[0] + [-1.0] * nspins[1], dtype=x.dtype)
    F[:, :, 0, :3] = rh[..., perm]
    F[:, :, 0, 3] = spins
    for i in range(N):
        F[:, i, 1 + 2 * i, :3] = th_h[:, i][..., perm]
        F[:, i, 2 + 2 * i, :3] = ph_h[:, i][..., perm]
    F[:, :, 2 * N + 1, :3] = -2.0 * rh[..., perm]  # Laplace-Beltrami of r_hat
    for k in range(3):
        ek = torch.zeros(3, dtype=x.dtype)
        ek[k] = 1.0
        s = ek * rh[..., k : k + 1] - rh  # e_k (e_k . r) - r  (second flow derivative)
        F[:, :, 2 * N + 2 + k, :3] = s[..., perm]
    return F


# ------------------------------------------------------------------ channel ops


def linear(X, W, b=None):
    Y = X @ W
    if b is not None:
        Y[:, :, 0] = Y[:, :, 0] + b
    return Y


def tanh_ch(Z, alpha):
    N2 = alpha.shape[-1]
    Y = torch.empty_like(Z)
    y0 = torch.tanh(Z[:, :, 0])
    d1 = 1 - y0 * y0
    d2 = -2 * y0 * d1
    Y[:, :, 0] = y0
    Y[:, :, 1 : 1 + N2] = d1[:, :, None] * Z[:, :, 1 : 1 + N2]
    Y[:, :, 1 + N2] = d1 * Z[:, :, 1 + N2] + d2 * (Z[:, :, 1 : 1 + N2] ** 2).sum(2)
    U = u_dirs(Z, alpha)  # [B,N,3,D]
    Y[:, :, 2 + N2 :] = d1[:, :, None] * Z[:, :, 2 + N2 :] + d2[:, :, None] * U**2
    return Y


def layer_norm_ch(X, alpha, scale, bias, eps=1e-5):
    N2 = alpha.shape[-1]
    Z = X - X.mean(-1, keepdim=True)
    z0 = Z[:, :, 0]
    s = 1.0 / torch.sqrt((z0 * z0).mean(-1) + eps)  # [B,N]
    a = (z0[:, :, None] * Z).mean(-1) * (s * s)[:, :, None]  # [B,N,C]
    Y = torch.empty_like(Z)
    Y[:, :, 0] = s[..., None] * z0
    at = a[:, :, 1 : 1 + N2]
    Zt = Z[:, :, 1 : 1 + N2]
    Y[:, :, 1 : 1 + N2] = s[..., None, None] * (Zt - at[..., None] * z0[:, :, None])
    mt2 = (Zt * Zt).mean(-1)  # [B,N,2N]
    coefL = (3 * at * at - (s * s)[..., None] * mt2).sum(-1)  # [B,N]
    YL = Z[:, :, 1 + N2] - a[:, :, 1 + N2, None] * z0 - 2 * (at[..., None] * Zt).sum(2) + coefL[..., None] * z0
    Y[:, :, 1 + N2] = s[..., None] * YL
    U = u_dirs(Z, alpha)  # [B,N,3,D]
    au = torch.einsum("bkt,bnt->bnk", alpha, at)
    mu2 = (U * U).mean(-1)
    coefS = 3 * au * au - (s * s)[..., None] * mu2  # [B,N,3]
    YS = Z[:, :, 2 + N2 :] - a[:, :, 2 + N2 :, None] * z0[:, :, None] - 2 * au[..., None] * U + coefS[..., None] * z0[:, :, None]
    Y[:, :, 2 + N2 :] = s[..., None, None] * YS
    Y = Y * scale
    Y[:, :, 0] = Y[:, :, 0] + bias
    return Y


def attention_ch(Qc, Kc, Vc, alpha):
    """Channel self-attention. Q/K/V: [B,N,C,H,dh] (Q already scaled by 1/sqrt(dh))."""
    N2 = alpha.shape[-1]
    q0, k0, v0 = Qc[:, :, 0], Kc[:, :, 0], Vc[:, :, 0]  # [B,N,H,dh]
    S0 = torch.einsum("bihd,bjhd->bhij", q0, k0)
    A0 = torch.softmax(S0, -1)
    avg = lambda X: (A0 * X).sum(-1, keepdim=True)  # noqa: E731
    O = torch.empty_like(Vc)
    O[:, :, 0] = torch.einsum("bhij,bjhd->bihd", A0, v0)
    # tangents
    qt = Qc[:, :, 1 : 1 + N2]  # [B,N,T,H,dh]
    kt = Kc[:, :, 1 : 1 + N2]
    vt = Vc[:, :, 1 : 1 + N2]
    St = torch.einsum("bithd,bjhd->bthij", qt, k0) + torch.einsum("bihd,bjthd->bthij", q0, kt)
    Sbar = St - (A0[:, None] * St).sum(-1, keepdim=True)
    At = A0[:, None] * Sbar
    O[:, :, 1 : 1 + N2] = torch.einsum("bthij,bjhd->bithd", At, v0) + torch.einsum("bhij,bjthd->bithd", A0, vt)
    # Laplace-Beltrami channel
    SL = (
        torch.einsum("bihd,bjhd->bhij", Qc[:, :, 1 + N2], k0)
        + torch.einsum("bihd,bjhd->bhij", q0, Kc[:, :, 1 + N2])
        + 2 * torch.einsum("bithd,bjthd->bhij", qt, kt)
    )
    T2 = (Sbar * Sbar).sum(1)
    AL = A0 * ((SL - avg(SL)) + (T2 - avg(T2)))
    O[:, :, 1 + N2] = (
        torch.einsum("bhij,bjhd->bihd", AL, v0)
        + torch.einsum("bhij,bjhd->bihd", A0, Vc[:, :, 1 + N2])
        + 2 * torch.einsum("bthij,bjthd->bihd", At, vt)
    )
    # flow channels
    for k in range(3):
        al = alpha[:, k]  # [B,T]
        qu = torch.einsum("bt,bithd->bihd", al, qt)
        ku = torch.einsum("bt,bjthd->bjhd", al, kt)
        vu = torch.einsum("bt,bjthd->bjhd", al, vt)
        Su_bar = torch.einsum("bt,bthij->bhij", al, Sbar)
        Au = torch.einsum("bt,bthij->bhij", al, At)
        c = 2 + N2 + k
        SS = (
            torch.einsum("bihd,bjhd->bhij", Qc[:, :, c], k0)
            + torch.einsum("bihd,bjhd->bhij", q0, Kc[:, :, c])
            + 2 * torch.einsum("bihd,bjhd->bhij", qu, ku)
        )
        U2 = Su_bar * Su_bar
        AS = A0 * ((SS - avg(SS)) + (U2 - avg(U2)))
        O[:, :, c] = (
            torch.einsum("bhij,bjhd->bihd", AS, v0)
            + torch.einsum("bhij,bjhd->bihd", A0, Vc[:, :, c])
            + 2 * torch.einsum("bhij,bjhd->bihd", Au, vu)
        )
    return O


# ------------------------------------------------------------------ envelope / Jastrow leaves


def gauge_sign(x):
    """kappa_i / Q of each electron's gauge exp(-i kappa_i phi_i): kappa_i = Q cos(theta_i)
    rounded to 1/64 of Q, the envelope's dominant harmonic (det.hip env_gauge: +-Q at the
    poles, ~0 on the equator).  Any per-electron constant is exact; this one keeps the phi
    derivatives of the contracted orbitals small."""
    return torch.round(64 * torch.cos(x[..., 0])) / 64


def envelope_channels(x, Q, gauge=False):
    """Envelope env[i,m] = c_m u^(Q+m) v^(Q-m) and its leaf derivatives.

    Returns complex [B,N,M] tensors: e0, dth (d/dtheta), dph (d/dphi / sin theta),
    lb (Laplace-Beltrami incl. cot term), and sflow [B,N,3,M] (second derivative along
    the rotation flow about x,y,z).
    """
    g = geometry(x)
    th, ph, st, ct = g["th"], g["ph"], g["st"], g["ct"]
    M = int(round(2 * Q)) + 1
    a = torch.arange(M, dtype=x.dtype)  # Q+m
    b = (M - 1) - a  # Q-m
    m = a - Q
    if gauge:  # env * exp(-i kappa phi), kappa = Q gauge_sign(x)
        m = m - (gauge_sign(x) * Q)[..., None]
    norm = torch.tensor(np.sqrt(ss.comb(2 * Q, Q - np.arange(-Q, Q + 1))), dtype=x.dtype)
    c = torch.cos(th / 2)[..., None]
    s = torch.sin(th / 2)[..., None]

    def pw(base, e):
        return torch.where(e >= 0, base ** torch.clamp(e, min=0), torch.zeros_like(base))

    R = pw(c, a) * pw(s, b)
    # dR/dtheta = 1/2 [ b c^(a+1) s^(b-1) - a c^(a-1) s^(b+1) ]
    R1 = 0.5 * (b * pw(c, a + 1) * pw(s, b - 1) - a * pw(c, a - 1) * pw(s, b + 1))
    # d2R/dtheta2
    R2 = 0.25 * (
        b * (b - 1) * pw(c, a + 2) * pw(s, b - 2)
        - b * (a + 1) * pw(c, a) * pw(s, b)
        - a * (b + 1) * pw(c, a) * pw(s, b)
        + a * (a - 1) * pw(c, a - 2) * pw(s, b + 2)
    )
    phase = torch.exp(1j * m * ph[..., None].to(_ctype(x)))
    e0 = norm * R * phase
    d_th = norm * R1 * phase
    d_ph = 1j * m * e0  # d/dphi
    d_thth = norm * R2 * phase
    d_thph = 1j * m * d_th
    d_phph = -(m**2) * e0
    st_ = st[..., None]
    ct_ = ct[..., None]
    dph_s = d_ph / st_
    lb = d_thth + d_phph / st_**2 + (ct_ / st_) * d_th
    # flow: theta' = ph_hat_k, phi' = -th_hat_k / sin th ; accelerations
    sp, cp = g["sp"], g["cp"]
    cot = ct / st
    sflow = []
    for k in range(3):
        tdot = g["ph_hat"][..., k]
        pdot = -g["th_hat"][..., k] / st
        thp = [cp * cot, sp * cot, -torch.ones_like(th)]  # theta_hat / sin
        dthp_dth = [-cp / st**2, -sp / st**2, torch.zeros_like(th)]
        dthp_dph = [-sp * cot, cp * cot, torch.zeros_like(th)]
        cs = [cp, sp, torch.zeros_like(th)]
        tdd = cs[k] * thp[k]
        pdd = -(dthp_dth[k] * tdot - dthp_dph[k] * thp[k])
        tdot, pdot, tdd, pdd = (t[..., None] for t in (tdot, pdot, tdd, pdd))
        sflow.append(d_thth * tdot**2 + 2 * d_thph * tdot * pdot + d_phph * pdot**2 + d_th * tdd + d_ph * pdd)
    return e0, d_th, dph_s, lb, torch.stack(sflow, 2)


def jastrow_channels(x, nspins, a_par, a_anti):
    """Jastrow value, scaled gradient [B,2N] and Laplace-Beltrami (blocks.py:76-121)."""
    g = geometry(x)
    B, N = x.shape[:2]
    rh, thh, phh = g["r_hat"], g["th_hat"], g["ph_hat"]
    J = torch.zeros(B, dtype=x.dtype)
    grad = torch.zeros(B, 2 * N, dtype=x.dtype)
    lb = torch.zeros(B, dtype=x.dtype)
    n_up = nspins[0]
    for i in range(N):
        for j in range(i + 1, N):
            same = (i < n_up) == (j < n_up)
            al = a_par if same else a_anti
            cst = 0.25 if same else 0.5
            u = (rh[:, i] * rh[:, j]).sum(-1)
            r = torch.sqrt(torch.clamp(2 - 2 * u, min=0))
            f = -(cst * al * al) / (al + r)
            f1 = (cst * al * al) / (al + r) ** 2
            f2 = -2 * (cst * al * al) / (al + r) ** 3
            J = J + f
            gu = -f1 / r  # dJ/du
            grad[:, 2 * i] += gu * (rh[:, j] * thh[:, i]).sum(-1)
            grad[:, 2 * i + 1] += gu * (rh[:, j] * phh[:, i]).sum(-1)
            grad[:, 2 * j] += gu * (rh[:, i] * thh[:, j]).sum(-1)
            grad[:, 2 * j + 1] += gu * (rh[:, i] * phh[:, j]).sum(-1)
            lb = lb + 2 * ((4 - r * r) * r * f2 + (4 - 3 * r * r) * f1) / (4 * r)
    return J, grad, lb


# ------------------------------------------------------------------ full pipeline


def split_heads(X, H, dh):
    return X.reshape(*X.shape[:-1], H, dh)


def trunk_channels(params, cfg: OracleConfig, x):
    N = cfg.nelec
    g = geometry(x)
    alpha = g["alpha"]
    H, dh = cfg.num_heads, cfg.heads_dim
    D = H * dh
    p = "PsiformerLayers_0/"
    X = input_channels(x, cfg.nspins) @ params[p + "Dense_0/kernel"]
    inter = [X]
    for l in range(cfg.num_layers):
        mha = p + f"MultiHeadAttention_{l}/"
        Wq = params[mha + "query/kernel"].reshape(D, D) / math.sqrt(dh)
        bq = params[mha + "query/bias"].reshape(D) / math.sqrt(dh)
        Qc = split_heads(linear(X, Wq, bq), H, dh)
        Kc = split_heads(linear(X, params[mha + "key/kernel"].reshape(D, D), params[mha + "key/bias"].reshape(D)), H, dh)
        Vc = split_heads(linear(X, params[mha + "value/kernel"].reshape(D, D), params[mha + "value/bias"].reshape(D)), H, dh)
        O = attention_ch(Qc, Kc, Vc, alpha).reshape(*X.shape)
        A = linear(O, params[mha + "out/kernel"].reshape(D, D), params[mha + "out/bias"])
        X = X + A @ params[p + f"Dense_{2 * l + 1}/kernel"]
        X = layer_norm_ch(X, alpha, params[p + f"LayerNorm_{2 * l}/scale"], params[p + f"LayerNorm_{2 * l}/bias"])
        Z = linear(X, params[p + f"Dense_{2 * l + 2}/kernel"], params[p + f"Dense_{2 * l + 2}/bias"])
        X = X + tanh_ch(Z, alpha)
        X = layer_norm_ch(X, alpha, params[p + f"LayerNorm_{2 * l + 1}/scale"], params[p + f"LayerNorm_{2 * l + 1}/bias"])
        inter.append(X)
    return X, inter


def local_energy(params, cfg: OracleConfig, x, gauge=False):
    """Batched E_L by channel propagation. x [B,N,2] float64.

    Returns (logpsi [B] complex, E_L [B] complex, obs dict, raw dict)."""
    N, K = cfg.nelec, cfg.determinants
    Q, r = cfg.Q, cfg.r
    M = int(round(cfg.flux)) + 1
    T = 2 * N
    C = n_channels(N)
    g = geometry(x)
    alpha = g["alpha"]
    Xh, _ = trunk_channels(params, cfg, x)  # [B,N,C,D]
    ob = "Orbitals_0/featured_orbitals/"
    n_up = cfg.nspins[0]

    def orb(blk, Xs):
        Wr = params[ob + f"DenseGeneral_{2 * blk}/kernel"]
        Wi = params[ob + f"DenseGeneral_{2 * blk + 1}/kernel"]
        Fr = torch.einsum("bncd,dmjk->bncmjk", Xs, Wr)
        Fi = torch.einsum("bncd,dmjk->bncmjk", Xs, Wi)
        Fr[:, :, 0] += params[ob + f"DenseGeneral_{2 * blk}/bias"]
        Fi[:, :, 0] += params[ob + f"DenseGeneral_{2 * blk + 1}/bias"]
        return torch.complex(Fr, Fi)

    parts = [orb(0, Xh[:, :n_up])]
    if cfg.nspins[1] > 0:
        parts.append(orb(1, Xh[:, n_up:]))
    F = torch.cat(parts, 1)  # [B,N(i),C,M,N(j),K]
    e0, dth, dph, elb, esf = envelope_channels(x, Q, gauge)  # [B,N,M]
    ctr = lambda Fc, e: torch.einsum("bimjk,bim->bkij", Fc, e)  # noqa: E731
    Phi0 = ctr(F[:, :, 0], e0)  # [B,K,N,N]
    Phit = torch.zeros(x.shape[0], T, K, N, N, dtype=_ctype(x))
    for t in range(T):
        i = t // 2
        de = dth if t % 2 == 0 else dph
        Phit[:, t] = ctr(F[:, :, 1 + t], e0)
        Phit[:, t, :, i, :] += torch.einsum("bmjk,bm->bkj", F[:, i, 0], de[:, i])
    PhiL = ctr(F[:, :, 1 + T], e0) + ctr(F[:, :, 0], elb)
    for i in range(N):
        PhiL[:, :, i, :] += 2 * (
            torch.einsum("bmjk,bm->bkj", F[:, i, 1 + 2 * i], dth[:, i])
            + torch.einsum("bmjk,bm->bkj", F[:, i, 2 + 2 * i], dph[:, i])
        )
    Binv = torch.linalg.inv(Phi0)
    sign, logabs = torch.linalg.slogdet(Phi0)
    ell0 = logabs + torch.log(sign)  # [B,K]
    Mt = torch.einsum("bkij,btkjl->btkil", Binv, Phit)
    tr = lambda Mx: torch.diagonal(Mx, dim1=-2, dim2=-1).sum(-1)  # noqa: E731
    ell_t = tr(Mt)  # [B,T,K]
    ell_L = tr(torch.einsum("bkij,bkjl->bkil", Binv, PhiL)) - tr(Mt @ Mt).sum(1)
    ell_S = []
    alc = alpha.to(_ctype(x))
    for k in range(3):
        flow1 = g["ph_hat"][..., k, None] * dth - g["th_hat"][..., k, None] * dph  # [B,N,M]
        Fu = torch.einsum("bt,bitmjl->bimjl", alc[:, k], F[:, :, 1 : 1 + T])
        PhiS = ctr(F[:, :, 2 + T + k], e0) + ctr(F[:, :, 0], esf[:, :, k]) + 2 * ctr(Fu, flow1)
        Mu = torch.einsum("bt,btkil->bkil", alc[:, k], Mt)
        ell_S.append(tr(torch.einsum("bkij,bkjl->bkil", Binv, PhiS)) - tr(Mu @ Mu))
    ell_S = torch.stack(ell_S, 1)  # [B,3,K]
    # combine determinants (log-sum-exp, psiformer.py:74-76)
    lmax = ell0.real.max(-1, keepdim=True).values
    w = torch.exp(ell0 - lmax)
    Z = w.sum(-1)
    p = w / Z[..., None]  # [B,K]
    val = torch.log(Z) + lmax[..., 0]
    g1 = (p[:, None] * ell_t).sum(-1)  # [B,T]
    mean_t = lambda X: (p[:, None] * X).sum(-1)  # noqa: E731
    LB = (p * ell_L).sum(-1) + (p[:, None] * ell_t**2).sum(-1).sum(-1) - (g1**2).sum(-1)
    gu = torch.einsum("bkt,btd->bkd", alc, ell_t)  # [B,3,K] first order along flows per det
    S = mean_t(ell_S) + mean_t(gu**2) - mean_t(gu) ** 2
    # Jastrow (additive in log psi)
    J, Jg, Jlb = jastrow_channels(x, cfg.nspins, params["Jastrow_0/ee_par"][0], params["Jastrow_0/ee_anti"][0])
    logpsi = val + J
    tg = g1 + Jg
    if gauge:  # add back A = i Q sum_i sigma_i phi_i analytically
        sg = gauge_sign(x)
        st_, ct_, sp_, cp_ = g["st"], g["ct"], g["sp"], g["cp"]
        cot_ = ct_ / st_
        logpsi = logpsi + 1j * Q * (sg * x[..., 1]).sum(-1)
        tg = tg.clone()
        tg[:, 1::2] = tg[:, 1::2] + 1j * Q * sg / st_
        tdot = [-sp_, cp_, torch.zeros_like(sp_)]
        thp = [cp_ * cot_, sp_ * cot_, -torch.ones_like(sp_)]
        d_th = [-cp_ / st_**2, -sp_ / st_**2, torch.zeros_like(sp_)]
        d_ph = [-sp_ * cot_, cp_ * cot_, torch.zeros_like(sp_)]
        S = S + torch.stack([(1j * Q * sg * (-(d_th[k] * tdot[k] - d_ph[k] * thp[k]))).sum(-1) for k in range(3)], -1)
    LB = LB + Jlb
    # assembly (hamiltonian.py:115-169, rewritten through the channels)
    st, ct, sp, cp = g["st"], g["ct"], g["sp"], g["cp"]
    cot = ct / st
    mag = ((Q * cot) ** 2).sum(-1) + (2j * Q * cot * tg[:, 1::2]).sum(-1)
    KE = (-LB - (tg**2).sum(-1) + mag) / (2 * r * r)
    G = torch.einsum("bkt,bt->bk", alc, tg)
    Mvec = torch.stack([Q * (cp / st).sum(-1), Q * (sp / st).sum(-1), torch.zeros_like(st[:, 0])], -1)
    L2 = -(S + (G + 1j * Mvec) ** 2).sum(-1)
    obs = {
        "angular_momentum_z": G[:, 2].imag,
        "angular_momentum_z_square": -(S[:, 2] + G[:, 2] ** 2).real,
        "angular_momentum_square": L2.real,
    }
    raw = dict(t=tg, LB=LB, S=S, G=G)
    return logpsi, KE, obs, raw
