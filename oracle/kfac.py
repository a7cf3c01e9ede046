"""TEST INFRASTRUCTURE ONLY — float64 restatement of the reference's KFAC step.

The reference optimises with KFAC by default (deephall/config.py:159) through
``make_kfac_training_step`` (deephall/optimizers/kfac.py:195-241), which builds
``kfac_jax.Optimizer`` with

    l2_reg=0, norm_constraint=1e-3, curvature_ema=0.95, inverse_update_period=1,
    estimation_mode="fisher_exact", multi_device=True, learning_rate_schedule =
    Optim.kfac.lr.schedule (rate 0.05, decay 1, delay 2000; config.py:125-161),
    momentum = 0 and damping = 1e-3 passed on every step (kfac.py:217-218, 230-236),

registers the loss with ``register_normal_predictive_distribution(Re log psi[:, None])``
(loss.py:98) and tags the dense layers with its ``repeated_dense`` blocks
(kfac.py:42-102, graph patterns 105-190).

kfac_jax (0.0.6, pyproject.toml:21) is a third-party dependency absent from
/root/reference and not importable here; this module restates its published algorithm
for exactly that configuration.  PARITY UNPINNED beyond the reference's own training pin
(tests/train_test.py:39-48: the energy oscillates around 1.5).  What is restated:

* Blocks.  Every dense layer is a two-Kronecker-factored block (kfac_jax
  DenseTwoKroneckerFactored through RepeatedDenseBlock): Dense_0 (no bias), per layer
  query / key / value / out (with bias) and Dense_{2l+1} (no bias) / Dense_{2l+2} (bias),
  and the orbital DenseGeneral_i (bias).  The parameters no pattern matches — the
  LayerNorm scales and biases (flax computes (x - mean) * (rsqrt(var + eps) * scale) +
  bias with the fast variance, which none of the scale-and-shift patterns describes) and
  the Jastrow alphas — are generic blocks (kfac_jax NaiveDiagonal).
* Statistics ("fisher_exact" with a normal predictive distribution of variance 1/2): the
  output tangent of a layer is dy = sqrt(2) d Re log psi_b / dy (the Fisher factor of the
  loss, 1 / sqrt(variance), times the layer's vjp).  A repeated dense layer's inputs and
  tangents are reshaped to rows (x.size // d_in rows: walker x electron [x head for the
  attention output], kfac.py:87-97); with a bias a column of ones is appended;
  A = x~^T x~ / rows, G = dy^T dy / rows.  A generic parameter's statistic is
  (sum_b sqrt(2) d Re log psi_b / dp)^2 / B (NaiveDiagonal: "(sum_i g_i)^2 / N").
  Across devices the statistics are averaged (multi_device pmean).
* EMA: a weighted moving average, raw <- 0.95 raw + stat, weight <- 0.95 weight + 1,
  value = raw / weight (every step updates with ema_old = curvature_ema, ema_new = 1).
* Scale: a repeated block's curvature is s * (A (x) G) with s = fixed_scale =
  prod(x_shape) // (x_shape[0] * x_shape[-1]) (kfac.py:74-76): N_spin_block for the dense
  layers, N * H for the attention output (x is [B, N, H, dh]).
* Inverse (damping lambda = 1e-3, exact factored Tikhonov with pi adjustment,
  inverse_update_period 1): (s A (x) G + lambda)^-1 ~= (s^1/2 A + pi sqrt(lambda) I)^-1
  (x) (s^1/2 G + sqrt(lambda) / pi I)^-1, pi = sqrt((tr A / dim A) / (tr G / dim G))
  (pi = 1 when a trace is 0).  For a weight V[d_in (+1 bias row), d_out]:
  P V = A_d^-1 V G_d^-1.  Generic: P g = g / (diag + lambda).
* Update: with momentum 0 and a fixed learning rate, delta = -lr * c * P g where
  c = min(1, sqrt(norm_constraint / (lr^2 <P g, g>))) (kfac_jax's norm constraint on the
  preconditioned gradient), lr = schedule(step), step counting from 0.

* Sparse orbitals (blocks.py:52-62).  The featured DenseGeneral_i then have 8 N K outputs
  (dense blocks as above).  lll_weight, DenseGeneral(2Q+1, axis=1) applied to the complex
  featured orbitals x [N, 8, N, K] per walker, is the "repeated_dense_complex_no_bias"
  pattern (kfac.py:127-133, 175-181) — a RepeatedDenseBlock without bias — and its bias,
  which that pattern leaves out, is generic.  The block's statistics follow
  RepeatedDenseBlock.update_curvature_matrix_estimate (kfac.py:78-102) literally:
  rows = x.size // 8, A from x.real.reshape((rows, -1)) — a row-major regrouping of each
  walker's [N, 8, N, K] array into consecutive groups of 8 (the contracted axis is axis 1,
  not the last one, so a group mixes (a, j, k) entries unless N K = 1) — and G from
  dy.real.reshape((rows, -1)) of the output tangent [N, N, K, M] (dy.real = the tangent with
  respect to the real part of the output); fixed_scale = prod(x_shape) // (x_shape[0] *
  x_shape[-1]) = 8 N^2 for x_shape [B, N, 8, N, K].  Whether kfac_jax's graph matcher tags
  an axis-1 dot_general with this pattern cannot be checked here (kfac_jax is absent);
  this restatement assumes it does, as the reference's pattern list intends.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from . import reference as R

DT = torch.float64
CURVATURE_EMA = 0.95
DAMPING = 1e-3
NORM_CONSTRAINT = 1e-3
FISHER_FACTOR = math.sqrt(2.0)  # 1 / sqrt(variance 0.5) of the normal predictive distribution


@dataclass
class Block:
    name: str  # layer path (tap name)
    kernel: str
    bias: str | None
    din: int  # rows of the kernel reshaped [din, dout] (without the bias row)
    dout: int
    scale: float
    lll: bool = False  # the complex lll_weight block (regrouped inputs / tangents, see header)

    @property
    def dA(self):
        return self.din + (1 if self.bias else 0)


def blocks(cfg: R.OracleConfig):
    """Dense blocks in dh_ref_layout order and the generic parameter names."""
    N, H, dh = cfg.nelec, cfg.num_heads, cfg.heads_dim
    D = H * dh
    M, K = int(round(cfg.flux)) + 1, cfg.determinants
    p = "PsiformerLayers_0/"
    out = [Block(p + "Dense_0", p + "Dense_0/kernel", None, 4, D, N)]
    generic = []
    for l in range(cfg.num_layers):
        mha = p + f"MultiHeadAttention_{l}/"
        for nm in ("query", "key", "value"):
            out.append(Block(mha + nm, mha + nm + "/kernel", mha + nm + "/bias", D, D, N))
        out.append(Block(mha + "out", mha + "out/kernel", mha + "out/bias", D, D, N * H))
        out.append(Block(p + f"Dense_{2 * l + 1}", p + f"Dense_{2 * l + 1}/kernel", None, D, D, N))
        out.append(Block(p + f"Dense_{2 * l + 2}", p + f"Dense_{2 * l + 2}/kernel", p + f"Dense_{2 * l + 2}/bias", D, D, N))
        for j in (2 * l, 2 * l + 1):
            generic += [p + f"LayerNorm_{j}/scale", p + f"LayerNorm_{j}/bias"]
    ob = "Orbitals_0/featured_orbitals/"
    sizes = [n for n in cfg.nspins if n > 0]
    F = 8 if cfg.orbital == "sparse" else M  # featured orbitals per (electron, determinant)
    for blk, n in enumerate(sizes):
        for part in range(2):
            nm = ob + f"DenseGeneral_{2 * blk + part}"
            out.append(Block(nm, nm + "/kernel", nm + "/bias", D, F * N * K, n))
    if cfg.orbital == "sparse":
        nm = "Orbitals_0/lll_weight"
        out.append(Block(nm, nm + "/kernel", None, 8, M, 8 * N * N, lll=True))
        generic.append(nm + "/bias")
    generic += ["Jastrow_0/ee_par", "Jastrow_0/ee_anti"]
    return out, generic


def block_rows(blk: Block, x_in, dy):
    """One walker's (inputs, output tangents) of a block as the kfac_jax rows: [rows, din]
    and [rows, dout] (the lll_weight regrouping of the header for the complex block)."""
    if blk.lll:
        x = x_in.real.reshape(-1, blk.din)                       # [N, 8, N, K] row-major, groups of 8
        g = dy.real.permute(0, 2, 3, 1).reshape(-1, blk.dout)    # [N, M, N, K] -> [N, N, K, M]
        return x, g
    return x_in.reshape(x_in.shape[0], -1), dy.reshape(dy.shape[0], -1)


def batch_statistics(params, cfg: R.OracleConfig, xs, shards: int = 1):
    """This step's curvature statistics: {block name: (A, G)}, {generic name: diag}.

    ``shards`` > 1 splits the walkers into equal contiguous device shards and averages the
    per-device statistics (kfac_jax multi_device)."""
    bl, generic = blocks(cfg)
    B = xs.shape[0]
    assert B % shards == 0
    per = B // shards
    acc_A = {b.name: 0.0 for b in bl}
    acc_G = {b.name: 0.0 for b in bl}
    acc_d = {g: 0.0 for g in generic}
    for s in range(shards):
        rec_x = {b.name: [] for b in bl}
        rec_dy = {b.name: [] for b in bl}
        gtan = {g: torch.zeros_like(params[g]) for g in generic}
        for b in range(s * per, (s + 1) * per):
            pr = {k: (v.detach().clone().requires_grad_(k in acc_d)) for k, v in params.items()}
            taps = {}

            def tap(name, x_in, y):
                eps = torch.zeros_like(y, requires_grad=True)
                taps[name] = (x_in.detach(), eps)
                return y + eps

            lp = R.logpsi(pr, cfg, torch.as_tensor(xs[b], dtype=DT), tap)
            names = list(taps)
            grads = torch.autograd.grad(FISHER_FACTOR * lp.real, [taps[n][1] for n in names] + [pr[g] for g in generic],
                                        allow_unused=True)
            byname = {blk.name: blk for blk in bl}
            for n, gy in zip(names, grads[: len(names)]):
                xr, gr = block_rows(byname[n], taps[n][0], gy)
                rec_x[n].append(xr)
                rec_dy[n].append(gr)
            for g, gg in zip(generic, grads[len(names):]):
                if gg is not None:
                    gtan[g] = gtan[g] + gg
        for blk in bl:
            x = torch.cat(rec_x[blk.name])
            dy = torch.cat(rec_dy[blk.name])
            rows = x.shape[0]
            if blk.bias:
                x = torch.cat([x, torch.ones(rows, 1, dtype=DT)], 1)
            acc_A[blk.name] = acc_A[blk.name] + x.T @ x / rows / shards
            acc_G[blk.name] = acc_G[blk.name] + dy.T @ dy / rows / shards
        for g in generic:
            acc_d[g] = acc_d[g] + gtan[g] ** 2 / per / shards
    return {b.name: (acc_A[b.name], acc_G[b.name]) for b in bl}, acc_d


@dataclass
class KfacState:
    raw_A: dict = field(default_factory=dict)
    raw_G: dict = field(default_factory=dict)
    raw_d: dict = field(default_factory=dict)
    weight: float = 0.0
    step: int = 0


def update_curvature(state: KfacState, stats, diag, ema=CURVATURE_EMA, storage=None):
    """``storage=torch.float32`` rounds the EMA sums to float32 (kfac_jax keeps them in
    the parameters' dtype)."""
    rnd = (lambda t: t.to(storage).to(DT)) if storage is not None else (lambda t: t)
    for k, (A, G) in stats.items():
        state.raw_A[k] = rnd(ema * state.raw_A.get(k, 0.0) + A)
        state.raw_G[k] = rnd(ema * state.raw_G.get(k, 0.0) + G)
    for k, d in diag.items():
        state.raw_d[k] = rnd(ema * state.raw_d.get(k, 0.0) + d)
    state.weight = ema * state.weight + 1.0
    if storage is not None:
        state.weight = float(torch.tensor(state.weight, dtype=storage))
    return state


def damped_inverses(A, G, scale, damping=DAMPING):
    """pi-adjusted factored Tikhonov inverses of s A (x) G + damping (see the header)."""
    As, Gs = math.sqrt(scale) * A, math.sqrt(scale) * G
    ta, tg = torch.trace(As) / As.shape[0], torch.trace(Gs) / Gs.shape[0]
    pi = torch.sqrt(ta / tg) if (ta > 0 and tg > 0) else torch.tensor(1.0, dtype=DT)
    sl = math.sqrt(damping)
    Ai = torch.linalg.inv(As + pi * sl * torch.eye(As.shape[0], dtype=DT))
    Gi = torch.linalg.inv(Gs + sl / pi * torch.eye(Gs.shape[0], dtype=DT))
    return Ai, Gi, float(pi)


def precondition(state: KfacState, cfg: R.OracleConfig, grads: dict, damping=DAMPING):
    """P g for every parameter (same keys and shapes as grads)."""
    bl, generic = blocks(cfg)
    out = {}
    for blk in bl:
        A = state.raw_A[blk.name] / state.weight
        G = state.raw_G[blk.name] / state.weight
        Ai, Gi, _ = damped_inverses(A, G, blk.scale, damping)
        V = grads[blk.kernel].reshape(blk.din, blk.dout).to(DT)
        if blk.bias:
            V = torch.cat([V, grads[blk.bias].reshape(1, blk.dout).to(DT)], 0)
        PV = Ai @ V @ Gi
        out[blk.kernel] = PV[: blk.din].reshape(grads[blk.kernel].shape)
        if blk.bias:
            out[blk.bias] = PV[blk.din].reshape(grads[blk.bias].shape)
    for g in generic:
        out[g] = grads[g].to(DT) / (state.raw_d[g] / state.weight + damping)
    return out


def lr_schedule(t, rate=0.05, decay=1.0, delay=2000.0):
    """config.py:134-135 (OptimizerKfac: rate 0.05)."""
    return rate * (1.0 / (1.0 + t / delay)) ** decay


def kfac_step(params, cfg, grads, state: KfacState, stats, diag, lr=None, norm_constraint=NORM_CONSTRAINT,
              storage=None, ema=CURVATURE_EMA):
    """One kfac_jax step given this step's gradient and curvature statistics.  Returns
    (new params, state, info) with info = {"pg": P g, "coef": c, "lr": lr}."""
    update_curvature(state, stats, diag, ema=ema, storage=storage)
    lr = lr_schedule(state.step) if lr is None else lr
    pg = precondition(state, cfg, grads)
    sq = sum(float((pg[k] * grads[k].to(DT)).sum()) for k in pg)
    coef = min(1.0, math.sqrt(norm_constraint / (lr * lr * sq))) if sq > 0 else 1.0
    new = dict(params)
    for k in pg:
        new[k] = params[k] - lr * coef * pg[k]
    state.step += 1
    return new, state, {"pg": pg, "coef": coef, "lr": lr, "sq": sq}
