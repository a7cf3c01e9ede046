"""GPU parity of KFAC (reference optimizers/kfac.py:195-241, the default
optimizer, config.py:159) against the float64 restatement of kfac_jax's algorithm
(oracle/kfac.py — parity unpinned beyond the reference's training pin: kfac_jax is not
importable here).

* statistics: every factor slot of dh_kfac_vjp (the Fisher reverse pass, layer Gram
  matrices, the folded attention output's derived factors, the generic diagonal) against
  oracle.kfac.batch_statistics; tolerance 1.5e-4 x the matrix's largest entry (f32 forward
  and backward — the gradient tests admit 3e-5 per tensor, a Gram matrix of two such
  tangents twice that — sums in double);
* step: the damped inverses, P g, the norm constraint and the update of dh_kfac_step fed
  the SAME float32 statistics and gradient as the oracle, the EMA sums stored in float32 on
  both sides (as kfac_jax keeps them), f64 arithmetic otherwise:
  P g within 1e-5 x its largest entry per tensor, c and <P g, g> within 1e-6;
* training: the reference's train_test.py:23-48 restated with the default optimizer —
  "energy=1.5" and "energy=1.4" both in the log (train_test.py:47-48).
"""

from __future__ import annotations

import logging
import math

import numpy as np
import pytest
import torch

from deephall_amd import Config, train
from deephall_amd.networks.psiformer import ParamTree
from helpers import make_params, make_walkers, oracle_config, to_device_params
from oracle import kfac as KF
from oracle import reference as R
from test_gpu_parity import build

pytestmark = pytest.mark.gpu


def _slots(model, cuda):
    lay = model.kfac_layout(cuda)
    return lay


def _oracle_by_slot(lay, ocfg, stats, diag):
    """The oracle's (A, G) per block, placed into the GPU statistics layout (float64)."""
    blocks, generic = KF.blocks(ocfg)
    assert len(blocks) == len(lay["blocks"])
    out = {}
    for ob, gb in zip(blocks, lay["blocks"]):
        A, G = stats[ob.name]
        assert A.shape[0] == lay["slots"][gb["a_slot"]][0] and G.shape[0] == lay["slots"][gb["g_slot"]][0]
        assert gb["din"] == ob.din and gb["dout"] == ob.dout and abs(gb["scale"] - ob.scale) < 1e-3
        out[gb["a_slot"]] = A
        out[gb["g_slot"]] = G
    gen = torch.cat([diag[g].reshape(-1) for g in generic])
    assert gen.numel() == lay["ngeneric"]
    return out, gen


@pytest.mark.parametrize("name,B,layers,orbital", [("C1", 8, 2, "full"), ("MIX", 8, 1, "full"), ("C2", 6, 2, "full"),
                                                   ("C1", 8, 1, "sparse"), ("MIX", 6, 1, "sparse"),
                                                   ("C2", 4, 1, "sparse")])
def test_kfac_statistics_match_oracle(cuda, name, B, layers, orbital):
    """Every factor slot and the generic diagonal; "sparse" orbitals (blocks.py:52-62) add the
    8 N K-output featured blocks, the complex lll_weight block (kfac.py:127-133, 175-181;
    oracle/kfac.py header) and its generic bias."""
    ocfg = oracle_config(name, num_layers=layers, orbital=orbital)
    p64 = make_params(ocfg)
    system, model = build(ocfg)
    params = to_device_params(p64)
    x = make_walkers(B, ocfg.nelec, seed=31)
    lay = _slots(model, cuda)
    stats = torch.full((lay["nstats"],), float("nan"), device=cuda)
    model.kfac_vjp(params, torch.tensor(x, device=cuda), None, None, stats)
    torch.cuda.synchronize()
    st = stats.double().cpu()
    ref, diag = KF.batch_statistics(p64, ocfg, torch.tensor(x, dtype=torch.float64))
    by_slot, gen = _oracle_by_slot(lay, ocfg, ref, diag)
    assert len(by_slot) == len(lay["slots"])
    errs = {}
    for slot, M in by_slot.items():
        n, off = lay["slots"][slot]
        got = st[off: off + n * n].reshape(n, n)
        errs[slot] = (got - M).abs().max().item() / max(M.abs().max().item(), 1e-30)
    print({k: f"{v:.1e}" for k, v in sorted(errs.items())})
    worst = max(errs.values())
    assert worst < 1.5e-4, errs
    g_got = st[lay["nmat"]: lay["nmat"] + lay["ngeneric"]]
    gerr = (g_got - gen).abs().max().item() / gen.abs().max().item()
    print(f"{name}: worst factor {worst:.1e}, generic {gerr:.1e}")
    assert gerr < 1e-4


def test_kfac_vjp_with_cotangent_and_chunks(cuda):
    """The training path of dh_kfac_vjp: a real cotangent (the gradient's and the
    Fisher pass share one saved forward) and walker chunks (the statistics accumulated across
    chunks, api.cpp's kf.acc).  The statistics equal the ct=None single-chunk result, the
    returned gradient equals model.vjp's, and the chunked run equals the unchunked one."""
    from deephall_amd.networks import psiformer as pf

    ocfg = oracle_config("C1", num_layers=2)
    p64 = make_params(ocfg)
    system, model = build(ocfg)
    params = to_device_params(p64)
    B = 24
    x = torch.tensor(make_walkers(B, ocfg.nelec, seed=33), device=cuda)
    ct = torch.tensor(np.random.default_rng(5).standard_normal((B, 2)), dtype=torch.float32, device=cuda)
    lay = _slots(model, cuda)
    s_ref = torch.zeros(lay["nstats"], device=cuda)  # (the slots' alignment gaps stay 0)
    model.kfac_vjp(params, x, None, None, s_ref)
    g_ref = model.vjp(params, x, ct).flat.clone()
    s_ct = torch.zeros_like(s_ref)
    g_ct = ParamTree.zeros(model.spec, cuda)
    model.kfac_vjp(params, x, ct, g_ct, s_ct)
    h = model.prepare(params, x.device)
    old = pf.VJP_WORKSPACE_BYTES
    try:
        pf.VJP_WORKSPACE_BYTES = h.lib.dh_kfac_workspace_bytes(h.h, 7)  # chunks of <= 7 walkers
        s_ch = torch.zeros_like(s_ref)
        g_ch = ParamTree.zeros(model.spec, cuda)
        model.kfac_vjp(params, x, ct, g_ch, s_ch)
    finally:
        pf.VJP_WORKSPACE_BYTES = old
    torch.cuda.synchronize()
    smax = s_ref.abs().max().item()
    gmax = g_ref.abs().max().item()
    assert torch.isfinite(s_ct).all() and torch.isfinite(s_ch).all()
    assert (s_ct - s_ref).abs().max().item() <= 1e-6 * smax
    assert (g_ct.flat - g_ref).abs().max().item() <= 1e-6 * gmax
    assert (s_ch - s_ref).abs().max().item() <= 2e-6 * smax, (s_ch - s_ref).abs().max().item() / smax
    assert (g_ch.flat - g_ref).abs().max().item() <= 2e-6 * gmax


@pytest.mark.parametrize("name,B,layers,orbital", [("C1", 8, 2, "full"), ("C2", 4, 2, "full"), ("C1", 8, 1, "sparse")])
def test_kfac_step_matches_oracle(cuda, name, B, layers, orbital):
    ocfg = oracle_config(name, num_layers=layers, orbital=orbital)
    p64 = make_params(ocfg)
    system, model = build(ocfg)
    x = torch.tensor(make_walkers(B, ocfg.nelec, seed=32), dtype=torch.float64)
    ref, diag = KF.batch_statistics(p64, ocfg, x)
    ct = np.zeros((B, 2))
    ct[:, 0] = np.random.default_rng(2).standard_normal(B)
    grads = R.logpsi_param_grad(p64, ocfg, x, ct)
    # float32 inputs shared by both sides
    ref = {k: (A.float().double(), G.float().double()) for k, (A, G) in ref.items()}
    diag = {k: v.float().double() for k, v in diag.items()}
    grads = {k: v.float().double() for k, v in grads.items()}
    lay = model.kfac_layout(cuda)
    by_slot, gen = _oracle_by_slot(lay, ocfg, ref, diag)
    stats = torch.zeros(lay["nstats"], dtype=torch.float32)
    for slot, M in by_slot.items():
        n, off = lay["slots"][slot]
        stats[off: off + n * n] = M.reshape(-1).float()
    stats[lay["nmat"]: lay["nmat"] + lay["ngeneric"]] = gen.float()
    stats = stats.to(cuda)
    params = ParamTree.zeros(model.spec, cuda)
    for k, v in p64.items():
        params[k].copy_(v.float().reshape(params[k].shape))
    gtree = ParamTree.zeros(model.spec, cuda)
    for k, v in grads.items():
        gtree[k].copy_(v.float().reshape(gtree[k].shape))
    raw = torch.zeros(lay["nstats"], device=cuda)
    pg = torch.zeros_like(params.flat)
    info = torch.zeros(4, dtype=torch.float64, device=cuda)
    state = KF.KfacState()
    p_ref = dict(p64)
    ema = float(np.float32(0.95))  # the float32 EMA factor and weight the kernels see
    for step in range(2):  # second step: EMA weight 1.95, the same statistics again
        weight = float(np.float32(ema * state.weight + 1.0))
        lr = KF.lr_schedule(step)
        model.kfac_step(raw, stats, ema, weight, gtree, params, lr, KF.DAMPING, KF.NORM_CONSTRAINT, pg, info)
        p_ref, state, inf = KF.kfac_step(p_ref, ocfg, grads, state, ref, diag, storage=torch.float32, ema=ema)
        assert state.weight == pytest.approx(weight)
        torch.cuda.synchronize()
        pgt = ParamTree.view_of(model.spec, pg)
        G = max(v.abs().max().item() for v in inf["pg"].values())
        for k, v in inf["pg"].items():
            got = pgt[k].double().cpu().reshape(v.shape)
            err = (got - v).abs().max().item() / max(v.abs().max().item(), 1e-6 * G)
            assert err < 1e-5, (step, k, err)
        sq, c = info[0].item(), info[1].item()
        assert sq == pytest.approx(inf["sq"], rel=1e-6)
        assert c == pytest.approx(inf["coef"], rel=1e-6)
        for k in p_ref:
            got = params[k].double().cpu().reshape(p_ref[k].shape)
            assert (got - p_ref[k]).abs().max().item() < 1e-6 * max(1.0, p_ref[k].abs().max().item()), k


class _Capture(logging.Handler):
    def __init__(self):
        super().__init__()
        self.lines = []

    def emit(self, record):
        self.lines.append(record.getMessage())


def test_kfac_training_restates_train_test(cuda, tmp_path):
    """tests/train_test.py:23-48 with the reference's default optimizer (KFAC, lr 0.05):
    Psiformer 1 layer, 1 head, heads_dim 4, N=3, 2Q=2, non-interacting, batch 60, seed 42,
    100 iterations; the energy oscillates around the filled-LLL 1.5."""
    cfg = Config.from_dict({
        "batch_size": 60, "seed": 42,
        "system": {"nspins": (3, 0), "flux": 2, "interaction_strength": 0.0},
        "network": {"psiformer": {"num_layers": 1, "num_heads": 1, "heads_dim": 4}},
        "optim": {"iterations": 100},
        "log": {"save_path": str(tmp_path), "initial_energy": False},
    })
    assert str(getattr(cfg.optim.optimizer, "value", cfg.optim.optimizer)) == "kfac"  # the default
    cap = _Capture()
    lg = logging.getLogger("deephall_amd")
    lg.addHandler(cap)
    try:
        state = train(cfg)
    finally:
        lg.removeHandler(cap)
    assert (tmp_path / "train_stats.csv").exists() and (tmp_path / "ckpt_000099.npz").exists()
    text = "\n".join(cap.lines)
    assert "energy=1.5" in text and "energy=1.4" in text  # train_test.py:47-48
    rows = (tmp_path / "train_stats.csv").read_text().splitlines()[1:]
    e = np.array([float(r.split(",")[2]) for r in rows])
    assert abs(np.mean(e[-30:]) - 1.5) < 0.05, e[-30:]
    assert state.opt_state.step == 100 and math.isfinite(state.opt_state.weight)
    with np.load(tmp_path / "ckpt_000099.npz", allow_pickle=False) as f:
        assert "opt_state/raw" in f.files and int(f["opt_state/step"]) == 100
