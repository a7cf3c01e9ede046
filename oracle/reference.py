"""TEST INFRASTRUCTURE ONLY — float64 restatement of the DeepHall reference algorithm.

Follows, line by line in behaviour (not in code), the reference files:

* forward      deephall/networks/psiformer.py:32-91, deephall/networks/blocks.py:23-121
               (Flax Dense / DenseGeneral / MultiHeadAttention / LayerNorm semantics)
* kinetic      deephall/hamiltonian.py:83-172 — gradient by autograd and the FULL
               [N,2,N,2] Hessian of Re and Im log psi (the reference uses
               ``jax.hessian`` = jacfwd(jacrev); here torch.func.hessian), then the
               exact KE / Lz / Lz^2 / L^2 formulas of hamiltonian.py:115-169
* potential    deephall/hamiltonian.py:27-80
* local energy deephall/hamiltonian.py:175-212
* MCMC         deephall/mcmc.py:25-102 (proposal + accept), with the random numbers
               injected as arrays instead of drawn from jax.random
* loss stats   deephall/loss.py:30-38, 66-92
* init_guess   deephall/train.py:40-54

Parameters are a flat dict keyed by the Flax auto-generated paths
(SURVEY.md Appendix B), values are float64 torch tensors.
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch
from scipy import special as ss

DT = torch.float64


@dataclass
class OracleConfig:
    """The System/Network fields the hot path reads (reference config.py:56-104)."""

    nspins: tuple = (3, 0)
    flux: int = 2
    radius: float | None = None
    interaction_strength: float = 1.0
    interaction_type: str = "coulomb"
    num_heads: int = 4
    heads_dim: int = 64
    num_layers: int = 2
    determinants: int = 1
    orbital: str = "full"

    @property
    def nelec(self):
        return int(sum(self.nspins))

    @property
    def Q(self):
        return self.flux / 2

    @property
    def r(self):
        return self.radius if self.radius else math.sqrt(self.Q)


# --------------------------------------------------------------------------
# Parameter tree (Appendix B names) and a Flax-like initialiser
# --------------------------------------------------------------------------


def param_shapes(cfg: OracleConfig) -> dict:
    D = cfg.num_heads * cfg.heads_dim
    H, dh = cfg.num_heads, cfg.heads_dim
    M = int(round(cfg.flux)) + 1
    N, K = cfg.nelec, cfg.determinants
    p = "PsiformerLayers_0/"
    shapes = {p + "Dense_0/kernel": (4, D)}
    for l in range(cfg.num_layers):
        mha = p + f"MultiHeadAttention_{l}/"
        for nm in ("query", "key", "value"):
            shapes[mha + nm + "/kernel"] = (D, H, dh)
            shapes[mha + nm + "/bias"] = (H, dh)
        shapes[mha + "out/kernel"] = (H, dh, D)
        shapes[mha + "out/bias"] = (D,)
        shapes[p + f"Dense_{2 * l + 1}/kernel"] = (D, D)
        shapes[p + f"LayerNorm_{2 * l}/scale"] = (D,)
        shapes[p + f"LayerNorm_{2 * l}/bias"] = (D,)
        shapes[p + f"Dense_{2 * l + 2}/kernel"] = (D, D)
        shapes[p + f"Dense_{2 * l + 2}/bias"] = (D,)
        shapes[p + f"LayerNorm_{2 * l + 1}/scale"] = (D,)
        shapes[p + f"LayerNorm_{2 * l + 1}/bias"] = (D,)
    ob = "Orbitals_0/featured_orbitals/"
    nblocks = 2 if cfg.nspins[1] > 0 and cfg.nspins[0] > 0 else 1
    F = 8 if cfg.orbital == "sparse" else M  # blocks.py:48-57
    for blk in range(nblocks):
        for part in range(2):  # real, imag  (blocks.py:30-31)
            idx = 2 * blk + part
            shapes[ob + f"DenseGeneral_{idx}/kernel"] = (D, F, N, K)
            shapes[ob + f"DenseGeneral_{idx}/bias"] = (F, N, K)
    if cfg.orbital == "sparse":  # lll_weight = DenseGeneral(2Q+1, axis=1) (blocks.py:57)
        shapes["Orbitals_0/lll_weight/kernel"] = (8, M)
        shapes["Orbitals_0/lll_weight/bias"] = (M,)
    shapes["Jastrow_0/ee_par"] = (1,)
    shapes["Jastrow_0/ee_anti"] = (1,)
    return shapes


def init_params(cfg: OracleConfig, seed: int = 42) -> dict:
    """lecun_normal (truncated) kernels, zero biases, LN scale 1, Jastrow alpha 1."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in param_shapes(cfg).items():
        if name.endswith("/kernel"):
            if "out/kernel" in name:
                fan_in = shape[0] * shape[1]
            else:
                fan_in = shape[0]
            std = math.sqrt(1.0 / fan_in) / 0.87962566103423978
            w = rng.standard_normal(size=shape)
            bad = np.abs(w) > 2
            while bad.any():
                w[bad] = rng.standard_normal(size=int(bad.sum()))
                bad = np.abs(w) > 2
            out[name] = torch.tensor(w * std, dtype=DT)
        elif name.endswith("/scale") or name.startswith("Jastrow"):
            out[name] = torch.ones(shape, dtype=DT)
        else:
            out[name] = torch.zeros(shape, dtype=DT)
    return out


# --------------------------------------------------------------------------
# Forward pass (psiformer.py:72-91, blocks.py)
# --------------------------------------------------------------------------


def _layer_norm(x, scale, bias, eps=1e-5):
    # flax LayerNorm, use_fast_variance=True: var = E[x^2] - E[x]^2 clipped at 0
    mean = x.mean(-1, keepdim=True)
    var = torch.clamp((x * x).mean(-1, keepdim=True) - mean * mean, min=0.0)
    return (x - mean) * torch.rsqrt(var + eps) * scale + bias


def _no_tap(name, x_in, y):
    return y


def trunk(params, cfg: OracleConfig, x, tap=_no_tap):
    """PsiformerLayers.__call__ (psiformer.py:37-60).  x: [N,2] -> [N,D].

    ``tap(name, x_in, y) -> y`` sees every dense layer's input and output (oracle/kfac.py
    adds a zero perturbation to read the output tangents, as kfac_jax's layer tags do)."""
    theta, phi = x[..., 0], x[..., 1]
    N = cfg.nelec
    spins = torch.tensor([1.0] * cfg.nspins[0] + [-1.0] * cfg.nspins[1], dtype=x.dtype)
    feat = torch.stack(
        [torch.cos(theta), torch.sin(theta) * torch.cos(phi), torch.sin(theta) * torch.sin(phi), spins], -1
    )
    p = "PsiformerLayers_0/"
    h = tap(p + "Dense_0", feat, feat @ params[p + "Dense_0/kernel"])
    H, dh = cfg.num_heads, cfg.heads_dim
    for l in range(cfg.num_layers):
        mha = p + f"MultiHeadAttention_{l}/"
        q = tap(mha + "query", h, torch.einsum("nd,dhk->nhk", h, params[mha + "query/kernel"]) + params[mha + "query/bias"])
        k = tap(mha + "key", h, torch.einsum("nd,dhk->nhk", h, params[mha + "key/kernel"]) + params[mha + "key/bias"])
        v = tap(mha + "value", h, torch.einsum("nd,dhk->nhk", h, params[mha + "value/kernel"]) + params[mha + "value/bias"])
        q = q / math.sqrt(dh)
        w = torch.einsum("qhd,khd->hqk", q, k)
        w = torch.softmax(w, dim=-1)
        o = torch.einsum("hqk,khd->qhd", w, v)
        attn = tap(mha + "out", o, torch.einsum("qhd,hdD->qD", o, params[mha + "out/kernel"]) + params[mha + "out/bias"])
        h = h + tap(p + f"Dense_{2 * l + 1}", attn, attn @ params[p + f"Dense_{2 * l + 1}/kernel"])
        h = _layer_norm(h, params[p + f"LayerNorm_{2 * l}/scale"], params[p + f"LayerNorm_{2 * l}/bias"])
        z = tap(p + f"Dense_{2 * l + 2}", h, h @ params[p + f"Dense_{2 * l + 2}/kernel"] + params[p + f"Dense_{2 * l + 2}/bias"])
        h = h + torch.tanh(z)
        h = _layer_norm(h, params[p + f"LayerNorm_{2 * l + 1}/scale"], params[p + f"LayerNorm_{2 * l + 1}/bias"])
    return h


def envelope(cfg: OracleConfig, theta, phi):
    """Monopole-harmonic envelope c_m u^(Q+m) v^(Q-m) (blocks.py:44-47, 64-67).  [N,M] complex."""
    Q = cfg.Q
    M = int(round(2 * Q)) + 1
    m = np.arange(-Q, Q + 1)
    norm = torch.tensor(np.sqrt(ss.comb(2 * Q, Q - m)), dtype=theta.dtype)
    ctype = torch.complex128 if theta.dtype == torch.float64 else torch.complex64
    u = (torch.cos(theta / 2) * torch.exp(0.5j * phi.to(ctype)))[..., None]
    v = (torch.sin(theta / 2) * torch.exp(-0.5j * phi.to(ctype)))[..., None]
    a = torch.arange(M, dtype=torch.int64)  # Q + m  (integer)
    b = (M - 1) - a  # Q - m
    # integer powers (the exponents Q +- m are always integers 0..2Q)
    upow = torch.stack([u[..., 0] ** int(e) for e in a.tolist()], -1)
    vpow = torch.stack([v[..., 0] ** int(e) for e in b.tolist()], -1)
    return norm * upow * vpow


def orbitals(params, cfg: OracleConfig, x, tap=_no_tap):
    """Psiformer.orbitals (psiformer.py:78-91): [K,N,N] complex, Jastrow included."""
    theta, phi = x[..., 0], x[..., 1]
    h = trunk(params, cfg, x, tap)
    N, K = cfg.nelec, cfg.determinants
    M = int(round(cfg.flux)) + 1
    ob = "Orbitals_0/featured_orbitals/"
    blocks = []
    n_up = cfg.nspins[0]
    splits = [(0, n_up), (n_up, N)]
    blk = 0
    for lo, hi in splits:
        if hi - lo == 0:
            continue
        hb = h[lo:hi]
        re = tap(ob + f"DenseGeneral_{2 * blk}", hb, torch.einsum(
            "nd,dmjk->nmjk", hb, params[ob + f"DenseGeneral_{2 * blk}/kernel"]) + params[ob + f"DenseGeneral_{2 * blk}/bias"])
        im = tap(ob + f"DenseGeneral_{2 * blk + 1}", hb, torch.einsum(
            "nd,dmjk->nmjk", hb, params[ob + f"DenseGeneral_{2 * blk + 1}/kernel"]) + params[
                ob + f"DenseGeneral_{2 * blk + 1}/bias"])
        blocks.append(torch.complex(re, im))
        blk += 1
    F = torch.cat(blocks, 0)  # [N, M, N, K]  ("sparse": [N, 8, N, K])
    if cfg.orbital == "sparse":
        # lll_weight: DenseGeneral over axis 1 (real kernel [8, M], real bias added to the complex
        # value), output moved to axis 1 (blocks.py:61-62)
        W = params["Orbitals_0/lll_weight/kernel"].to(F.real.dtype)
        b = params["Orbitals_0/lll_weight/bias"].to(F.real.dtype)
        # (tap: the complex input [N, 8, N, K] and the output in this function's [N, M, N, K]
        # layout; oracle/kfac.py regroups them as kfac_jax would)
        F = tap("Orbitals_0/lll_weight", F, torch.einsum("najk,am->nmjk", F, W.to(F.dtype)) + b[None, :, None, None])
    env = envelope(cfg, theta, phi)  # [N, M]
    orb = (F * env[:, :, None, None]).sum(1)  # [N, N, K]
    orb = orb.permute(2, 0, 1)  # [K, N, N]
    J = jastrow(params, cfg, x)
    return torch.exp(J / N) * orb


def _r_ee(x):
    theta, phi = x[..., 0], x[..., 1]
    cart = torch.stack([torch.cos(theta), torch.sin(theta) * torch.cos(phi), torch.sin(theta) * torch.sin(phi)], -1)
    diff = cart[None] - cart[:, None]
    eye = torch.eye(cart.shape[0], dtype=x.dtype)
    return torch.linalg.norm(diff + eye[..., None], dim=-1) * (1.0 - eye)


def jastrow(params, cfg: OracleConfig, x):
    """Jastrow.__call__ (blocks.py:76-121)."""
    r = _r_ee(x)
    n_up, n_dn = cfg.nspins
    J = torch.zeros((), dtype=x.dtype)
    a_par = params["Jastrow_0/ee_par"][0]
    a_anti = params["Jastrow_0/ee_anti"][0]
    for lo, hi in ((0, n_up), (n_up, n_up + n_dn)):
        n = hi - lo
        if n > 1:
            iu = torch.triu_indices(n, n, 1)
            rp = r[lo:hi, lo:hi][iu[0], iu[1]]
            J = J + torch.sum(-(0.25 * a_par**2) / (a_par + rp))
    if n_up > 0 and n_dn > 0:
        ra = r[:n_up, n_up:]
        J = J + torch.sum(-(0.5 * a_anti**2) / (a_anti + ra))
    return J


def logpsi(params, cfg: OracleConfig, x, tap=_no_tap):
    """Psiformer.__call__ (psiformer.py:72-76): complex log psi of one walker x[N,2]."""
    orb = orbitals(params, cfg, x, tap)
    sign, logdet = torch.linalg.slogdet(orb)
    logmax = torch.max(logdet)
    return torch.log(torch.sum(sign * torch.exp(logdet - logmax))) + logmax


# --------------------------------------------------------------------------
# Laughlin wavefunction (networks/laughlin.py:19-100)
# --------------------------------------------------------------------------


@dataclass
class LaughlinConfig:
    """Laughlin(nspins, flux, cf_flux=1, excitation_lz) as networks/__init__.py:25-27 builds
    it; plus the System fields local_energy reads."""

    nspins: tuple = (3, 0)
    flux: int = 6
    excitation_lz: float = 0.0
    cf_flux: int = 1
    radius: float | None = None
    interaction_strength: float = 1.0
    interaction_type: str = "coulomb"

    @property
    def nelec(self):
        return int(sum(self.nspins))

    @property
    def Q(self):
        return self.flux / 2

    @property
    def r(self):
        return self.radius if self.radius else math.sqrt(self.Q)

    @property
    def Q1(self):
        return self.flux / 2 - self.cf_flux * (self.nelec - 1)

    def kind(self):
        """laughlin.py:32-45: ground state (N = 2 Q1 + 1), quasihole (N = 2 Q1),
        quasiparticle (N = 2 Q1 + 2)."""
        n, q1 = self.nelec, self.Q1
        if n == 2 * q1 + 1:
            return "ground"
        if n == 2 * q1:
            return "quasihole"
        if n == 2 * q1 + 2:
            return "quasiparticle"
        raise ValueError("Filling not supported")

    def exponents(self):
        """m of the composite-fermion orbitals u^(Q1+m) v^(Q1-m) (laughlin.py:66-80)."""
        q1, lz = self.Q1, self.excitation_lz
        if self.kind() == "quasihole":
            return np.concatenate([np.arange(-q1, -lz), np.arange(q1, -lz, -1)])
        return np.arange(-q1, q1 + 1)


def laughlin_orbitals(cfg: LaughlinConfig, x):
    """laughlin.py:54-100 (complex [N, N])."""
    theta, phi = x[..., 0], x[..., 1]
    ctype = torch.complex128 if x.dtype == torch.float64 else torch.complex64
    u = (torch.cos(theta / 2) * torch.exp(0.5j * phi.to(ctype)))[..., None]
    v = (torch.sin(theta / 2) * torch.exp(-0.5j * phi.to(ctype)))[..., None]
    N = cfg.nelec
    q1 = cfg.Q1
    element = u * v[:, 0] - u[:, 0] * v + torch.eye(N, dtype=ctype)
    jastrow = torch.prod(element, dim=-1, keepdim=True)
    if cfg.kind() != "quasiparticle":
        m = cfg.exponents()
        a = [int(round(q1 + mm)) for mm in m]
        b = [int(round(q1 - mm)) for mm in m]
        cols = torch.stack([u[:, 0] ** aa * v[:, 0] ** bb for aa, bb in zip(a, b)], -1)
        return cols * jastrow
    m = np.arange(-q1, q1 + 1)
    cols = torch.stack([u[:, 0] ** int(round(q1 + mm)) * v[:, 0] ** int(round(q1 - mm)) for mm in m], -1)
    jastrow_dv = jastrow * (torch.sum(-u[:, 0] / element, dim=-1, keepdim=True) + u)
    jastrow_du = jastrow * (torch.sum(v[:, 0] / element, dim=-1, keepdim=True) - v)
    m1 = cfg.excitation_lz
    excited = (u ** int(round(q1 + m1)) * v ** int(round(q1 - m1))) * (
        (q1 + 1 + m1) * v * jastrow_dv - (q1 + 1 - m1) * u * jastrow_du
    )
    return torch.cat([cols * jastrow, excited], -1)


def laughlin_logpsi(cfg: LaughlinConfig, x):
    """Laughlin.__call__ (laughlin.py:48-52): slogdet + log-sum-exp of one determinant."""
    sign, logdet = torch.linalg.slogdet(laughlin_orbitals(cfg, x))
    return torch.log(sign) + logdet


def laughlin_local_energy(cfg: LaughlinConfig, xs):
    """hamiltonian.local_energy with f = the Laughlin wavefunction (full autograd Hessian)."""
    f = lambda p, y: laughlin_logpsi(cfg, y)  # noqa: E731
    ke = make_local_kinetic_energy(f, cfg.Q, cfg.r)
    els, obs = [], {}
    for b in range(xs.shape[0]):
        kin, o = ke(None, xs[b])
        o = dict(o)
        pot = potential(cfg, xs[b]) * cfg.interaction_strength
        o["potential"], o["kinetic"] = pot, kin
        els.append(kin + pot)
        for k, v in o.items():
            obs.setdefault(k, []).append(v)
    return torch.stack(els), {k: torch.stack(v) for k, v in obs.items()}


# --------------------------------------------------------------------------
# Local energy (hamiltonian.py) — full Hessian, exactly the reference formulas
# --------------------------------------------------------------------------


def coulomb_potential(cos12, r):
    r_ee = torch.sqrt(2 - 2 * cos12)
    return torch.sum(torch.triu(1 / r_ee, diagonal=1)) / r


def harmonic_potential(cos12, Q):
    return torch.sum(torch.triu(1 + (Q + 1) / Q * cos12, diagonal=1))


def potential(cfg: OracleConfig, x):
    """make_potential.potential (hamiltonian.py:63-80)."""
    theta, phi = x[..., 0], x[..., 1]
    xyz = torch.stack([torch.sin(theta) * torch.cos(phi), torch.sin(theta) * torch.sin(phi), torch.cos(theta)], -1)
    cos12 = xyz @ xyz.T
    if cfg.interaction_type == "coulomb":
        return coulomb_potential(cos12, cfg.r)
    return harmonic_potential(cos12, cfg.Q)


def kinetic_from_derivatives(grad_theta, grad_phi, hess, theta, phi, Q, r):
    """hamiltonian.py:115-169 given g and the complex Hessian [N,2,N,2]."""
    sin, cos, tan = torch.sin, torch.cos, torch.tan
    square_grad = torch.sum(grad_theta**2 + grad_phi**2 / sin(theta) ** 2)
    grad_grad = torch.sum(
        grad_theta / tan(theta) + torch.diagonal(hess[:, 0, :, 0]) + torch.diagonal(hess[:, 1, :, 1]) / sin(theta) ** 2
    )
    magnetic = torch.sum((Q / tan(theta)) ** 2 + 2j * Q * cos(theta) / sin(theta) ** 2 * grad_phi)
    kinetic = (-grad_grad - square_grad + magnetic) / 2 / r**2

    r_hat = torch.stack([sin(theta) * cos(phi), sin(theta) * sin(phi), cos(theta)])
    phi_hat = torch.stack([-sin(phi), cos(phi), torch.zeros_like(phi)])
    theta_hat_prime = torch.stack([cos(phi) / tan(theta), sin(phi) / tan(theta), -torch.ones_like(theta)])
    gi = lambda t: t[..., :, None]  # noqa: E731
    gj = lambda t: t[..., None, :]  # noqa: E731
    h_tt = hess[:, 0, :, 0] + gi(grad_theta) * gj(grad_theta)
    h_tp = hess[:, 0, :, 1] + gi(grad_theta) * gj(grad_phi)
    h_pp = hess[:, 1, :, 1] + gi(grad_phi) * gj(grad_phi)
    magnetic_term = Q * (theta_hat_prime * cos(theta) + r_hat)
    l2 = torch.sum(
        2 * gi(phi_hat) * gj(theta_hat_prime) * h_tp
        - gi(phi_hat) * gj(phi_hat) * h_tt
        - gi(theta_hat_prime) * gj(theta_hat_prime) * h_pp
        - (2j * gj(magnetic_term)) * (gi(phi_hat) * gi(grad_theta) - gi(theta_hat_prime) * gi(grad_phi))
        + gi(magnetic_term) * gj(magnetic_term)
    ) - torch.sum(grad_theta / tan(theta))
    obs = {
        "angular_momentum_z": torch.sum(grad_phi).imag,
        "angular_momentum_z_square": -torch.sum(h_pp).real,
        "angular_momentum_square": l2.real,
    }
    return kinetic, obs


def make_local_kinetic_energy(f, Q, r):
    """hamiltonian.py:83-172 with torch.func in place of jax.grad / jax.hessian.

    ``f(params, x[N,2]) -> complex scalar``; returns ``ke(params, x) -> (KE, obs)``.
    """
    from torch.func import grad, hessian

    def _ke(params, data):
        fr = lambda x: f(params, x).real  # noqa: E731
        fi = lambda x: f(params, x).imag  # noqa: E731
        gr = grad(fr)(data)
        gim = grad(fi)(data)
        gt = torch.complex(gr[..., 0], gim[..., 0])
        gp = torch.complex(gr[..., 1], gim[..., 1])
        hr = hessian(fr)(data)
        hi = hessian(fi)(data)
        hess = torch.complex(hr, hi)
        return kinetic_from_derivatives(gt, gp, hess, data[..., 0], data[..., 1], Q, r)

    return _ke


def local_energy_walker(params, cfg: OracleConfig, x, f=None):
    """local_energy._e_l (hamiltonian.py:193-210) for ONE walker."""
    f = f or (lambda p, y: logpsi(p, cfg, y))
    ke = make_local_kinetic_energy(f, cfg.Q, cfg.r)
    pot = potential(cfg, x) * cfg.interaction_strength
    kin, obs = ke(params, x)
    obs = dict(obs)
    obs["potential"] = pot
    obs["kinetic"] = kin
    return kin + pot, obs


def local_energy(params, cfg: OracleConfig, xs):
    """Batched E_L over walkers xs[B,N,2] (loop; the oracle is small-batch only)."""
    els, obs = [], {}
    for b in range(xs.shape[0]):
        e, o = local_energy_walker(params, cfg, xs[b])
        els.append(e)
        for k, v in o.items():
            obs.setdefault(k, []).append(v)
    return torch.stack(els), {k: torch.stack(v) for k, v in obs.items()}


def batch_logpsi(params, cfg, xs):
    return torch.stack([logpsi(params, cfg, xs[b]) for b in range(xs.shape[0])])


def logpsi_param_grad(params, cfg: OracleConfig, xs, ct):
    """sum_b ct[b,0] dRe log psi_b/dp + ct[b,1] dIm log psi_b/dp by torch autograd: the
    reference's jax.value_and_grad of network(params, x).real / .imag (loss.py:53-58)
    contracted with the per-walker weights of loss_prod (loss.py:59-64)."""
    P = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
    total = torch.zeros((), dtype=xs.dtype)
    for b in range(xs.shape[0]):
        lp = logpsi(P, cfg, xs[b])
        total = total + float(ct[b][0]) * lp.real + float(ct[b][1]) * lp.imag
    grads = torch.autograd.grad(total, list(P.values()), allow_unused=True)
    return {k: (g if g is not None else torch.zeros_like(P[k])) for k, g in zip(P, grads)}


def adam_reference(params, grads_seq, lr_fn, b1=0.9, b2=0.999, eps=1e-8):
    """optax.adam (scale_by_adam + scale_by_learning_rate with a schedule), float64: the
    update of optimizers/adam.py:24-43 applied for each gradient in ``grads_seq``."""
    p = {k: v.clone() for k, v in params.items()}
    mu = {k: torch.zeros_like(v) for k, v in p.items()}
    nu = {k: torch.zeros_like(v) for k, v in p.items()}
    for t, g in enumerate(grads_seq):
        for k in p:
            gk = torch.nan_to_num(g[k])
            mu[k] = (1 - b1) * gk + b1 * mu[k]
            nu[k] = (1 - b2) * gk * gk + b2 * nu[k]
            mh = mu[k] / (1 - b1 ** (t + 1))
            vh = nu[k] / (1 - b2 ** (t + 1))
            p[k] = p[k] - lr_fn(t) * mh / (torch.sqrt(vh) + eps)
    return p


# --------------------------------------------------------------------------
# MCMC (mcmc.py) with injected noise
# --------------------------------------------------------------------------


def sph_sampling(x1, normal, uniform, stddev):
    """mcmc.py:67-102. normal/uniform: arrays shaped like theta ([...,N]).

    ``uniform`` in [0,1) is mapped to phi' = 2*pi*uniform (mcmc.py:72).
    Works for numpy or torch float arrays (uses torch internally).
    """
    x1 = torch.as_tensor(x1)
    normal = torch.as_tensor(normal, dtype=x1.dtype)
    uniform = torch.as_tensor(uniform, dtype=x1.dtype)
    theta, phi = x1[..., 0], x1[..., 1]
    theta_p = torch.arctan(normal * stddev)
    phi_p = uniform * 2 * math.pi
    xyz_p = torch.stack(
        [torch.sin(theta_p) * torch.cos(phi_p), torch.sin(theta_p) * torch.sin(phi_p), torch.cos(theta_p)], -1
    )
    one, zero = torch.ones_like(phi), torch.zeros_like(phi)
    rot_z = torch.stack(
        [
            torch.stack([torch.cos(phi), -torch.sin(phi), zero]),
            torch.stack([torch.sin(phi), torch.cos(phi), zero]),
            torch.stack([zero, zero, one]),
        ]
    )
    rot_y = torch.stack(
        [
            torch.stack([torch.cos(theta), zero, torch.sin(theta)]),
            torch.stack([zero, one, zero]),
            torch.stack([-torch.sin(theta), zero, torch.cos(theta)]),
        ]
    )
    x2_xyz = torch.einsum("ij...,jk...,...k->...i", rot_z, rot_y, xyz_p)
    x2, y2, z2 = x2_xyz[..., 0], x2_xyz[..., 1], x2_xyz[..., 2]
    theta_n = torch.arccos(torch.clamp(z2, -1, 1))
    phi_n = torch.sign(y2) * torch.arccos(torch.clamp(x2 / torch.sin(theta_n), -1, 1))
    return torch.stack([theta_n, phi_n], -1)


def mh_accept(x1, x2, lp1, lp2, u_accept):
    """mcmc.py:55-62: accept if lp2 - lp1 > log(u)."""
    cond = (lp2 - lp1) > torch.log(torch.as_tensor(u_accept, dtype=lp1.dtype))
    x = torch.where(cond[..., None, None], x2, x1)
    lp = torch.where(cond, lp2, lp1)
    return x, lp, cond


def mcmc_step(logprob_fn, x, width, normals, uniforms, u_accepts):
    """make_mcmc_step.mcmc_step (mcmc.py:122-148) for one device, injected noise.

    normals/uniforms: [steps,B,N]; u_accepts: [steps,B].  Returns (x, pmove, lp).
    """
    lp = logprob_fn(x)
    steps = normals.shape[0]
    n_acc = 0
    for s in range(steps):
        x2 = sph_sampling(x, normals[s], uniforms[s], width)
        lp2 = logprob_fn(x2)
        x, lp, cond = mh_accept(x, x2, lp, lp2, u_accepts[s])
        n_acc = n_acc + int(cond.sum())
    return x, n_acc / (steps * x.shape[0]), lp


def update_mcmc_width(t, width, adapt_frequency, pmove, pmoves, pmove_max=0.55, pmove_min=0.5):
    """mcmc.py:153-186 (host side)."""
    t_since = t % adapt_frequency
    pmoves[t_since] = float(pmove)
    if t > 0 and t_since == 0:
        if np.mean(pmoves) > pmove_max:
            width *= 1.1
        elif np.mean(pmoves) < pmove_min:
            width /= 1.1
    return width, pmoves


def init_guess_from_uniforms(u1, u2):
    """train.py:40-54 with injected U(0,1) arrays: theta = arccos U(-1,1), phi = U(-pi,pi)."""
    theta = np.arccos(2.0 * np.asarray(u1) - 1.0)
    phi = (2.0 * np.asarray(u2) - 1.0) * np.pi
    return np.stack([theta, phi], -1)


# --------------------------------------------------------------------------
# Loss statistics (loss.py:30-38, 66-92) for one device
# --------------------------------------------------------------------------


def iqr_clip_real(x, scale=100.0):
    x = np.asarray(x, dtype=np.float64)
    q1 = np.nanquantile(x, 0.25)
    q3 = np.nanquantile(x, 0.75)
    iqr = q3 - q1
    return np.clip(x, q1 - scale * iqr, q3 + scale * iqr)


def iqr_clip(x, scale=100.0):
    x = np.asarray(x)
    return iqr_clip_real(x.real, scale) + 1j * iqr_clip_real(x.imag, scale)


def loss_stats(el, obs, ndev_means=None, penalties=False):
    """Device-local part of loss_and_grad stats (loss.py:66-92), single device.

    ``el`` complex [B]; ``obs`` dict of [B] arrays.  Returns dict of scalars.
    ``penalties``: also the clipped Lz^2 / Lz / L^2 means of loss.py:79-80, 87 (needs the
    angular-momentum keys in ``obs``).
    """
    el = np.asarray(el)
    out = {k: np.mean(np.asarray(v)) for k, v in obs.items()}
    energy = np.nanmean(el)
    out["energy"] = energy
    out["clipped_energy"] = np.nanmean(iqr_clip(el))
    out["variance"] = np.nanmean(el.real**2) - energy.real**2
    if penalties:
        out["clipped_lz2"] = np.nanmean(iqr_clip(obs["angular_momentum_z_square"]))
        out["clipped_lz"] = np.nanmean(iqr_clip(obs["angular_momentum_z"]))
        out["clipped_l2"] = np.nanmean(iqr_clip(obs["angular_momentum_square"]))
    return out


def loss_diff(el, obs, stats, lz_penalty=0.0, lz_center=0.0, l2_penalty=0.0):
    """loss.py:75-89: diff = iqr_clip(E_L - <E_L>_clip + penalty terms); ``stats`` holds the
    (device-averaged) clipped means of loss_stats(..., penalties=True)."""
    d = np.asarray(el, dtype=np.complex128) - stats["clipped_energy"]
    if lz_penalty:
        lz2 = np.asarray(obs["angular_momentum_z_square"], dtype=np.float64)
        lz = np.asarray(obs["angular_momentum_z"], dtype=np.float64)
        d = d + lz_penalty * ((lz2 - stats["clipped_lz2"]) - 2 * lz_center * (lz - stats["clipped_lz"]))
    if l2_penalty:
        l2 = np.asarray(obs["angular_momentum_square"], dtype=np.float64)
        d = d + l2_penalty * (l2 - stats["clipped_l2"])
    return iqr_clip(d)
