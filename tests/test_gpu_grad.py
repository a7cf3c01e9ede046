"""GPU parity of the parameter gradient and the Adam step (§8f-2).

The HIP reverse mode (dh_logpsi_vjp, through the C ABI) against torch autograd of the
float64 restatement (oracle.reference.logpsi_param_grad = the reference's
jax.grad of network(params, x).real / .imag contracted with loss_prod's weights,
loss.py:53-64).  Tolerance: per parameter tensor, max |g - g_ref| <= 3e-5 * max |g_ref|
(f32 forward + backward; the weights ct are O(1), the walkers O(10)).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from deephall_amd import config
from deephall_amd.loss import LossMode, make_loss_fn
from deephall_amd.networks.psiformer import ParamTree, flat_params
from deephall_amd.optimizers import AdamState, adam_update, lr_schedule
from helpers import make_params, make_walkers, oracle_config, to_device_params
from oracle import reference as R
from test_gpu_parity import build

pytestmark = pytest.mark.gpu
TOL_G = 3e-5


def grad_errors(g_dev, g_ref, floor=1e-3):
    """max |g - g_ref| / max(max |g_ref|, floor * G) per tensor, G = the largest gradient
    entry of the whole tree: tensors whose exact gradient vanishes (the key biases: softmax
    is invariant to a per-row shift) are compared at the f32 noise level of the tree."""
    G = max(r.abs().max().item() for r in g_ref.values())
    errs = {}
    for k, ref in g_ref.items():
        got = g_dev[k].detach().double().cpu().reshape(ref.shape)
        errs[k] = (got - ref).abs().max().item() / max(ref.abs().max().item(), floor * G)
    print({k.split("/", 1)[-1]: f"{v:.1e}" for k, v in errs.items()})
    return errs


@pytest.mark.parametrize("name,B,orbital", [("C1", 8, "full"), ("C2", 6, "full"), ("MIX", 8, "full"),
                                            ("C1", 6, "sparse"), ("MIX", 6, "sparse")])
def test_vjp_matches_autograd(cuda, name, B, orbital):
    ocfg = oracle_config(name, orbital=orbital)
    p64 = make_params(ocfg)
    system, model = build(ocfg)
    params = to_device_params(p64)
    x = make_walkers(B, ocfg.nelec, seed=21)
    ct = np.random.default_rng(5).standard_normal((B, 2)).astype(np.float32)
    xd = torch.tensor(x, device=cuda)
    lp = torch.empty(B, 2, device=cuda)
    g = model.vjp(params, xd, torch.tensor(ct, device=cuda), logpsi=lp)
    ref = R.logpsi_param_grad(p64, ocfg, torch.tensor(x, dtype=torch.float64), ct.astype(np.float64))
    errs = grad_errors(g, ref)
    worst = max(errs, key=errs.get)
    assert errs[worst] < TOL_G, (worst, errs[worst])
    # the VJP's own forward pass returns log psi too
    lp_ref = R.batch_logpsi(p64, ocfg, torch.tensor(x, dtype=torch.float64))
    assert np.max(np.abs(lp[:, 0].cpu().numpy() - lp_ref.real.numpy()) / np.maximum(1, np.abs(lp_ref.real.numpy()))) < 2e-5


def test_vjp_chunking_and_linearity(cuda):
    """Walker chunks accumulate into the same gradient; the VJP is linear in ct."""
    from deephall_amd.networks import psiformer as pf

    ocfg = oracle_config("C2")
    system, model = build(ocfg)
    params = model.init(3, device=cuda)
    B = 40
    x = torch.tensor(make_walkers(B, ocfg.nelec, seed=8), device=cuda)
    ct = torch.tensor(np.random.default_rng(1).standard_normal((B, 2)), dtype=torch.float32, device=cuda)
    g1 = model.vjp(params, x, ct).flat.clone()
    g2 = model.vjp(params, x, 2 * ct).flat.clone()
    h = model.prepare(params, x.device)
    old = pf.VJP_WORKSPACE_BYTES
    try:
        pf.VJP_WORKSPACE_BYTES = h.lib.dh_vjp_workspace_bytes(h.h, 7)  # chunks of <= 7 walkers
        g3 = model.vjp(params, x, ct).flat.clone()
    finally:
        pf.VJP_WORKSPACE_BYTES = old
    scale = g1.abs().max().item()
    assert (g2 - 2 * g1).abs().max().item() <= 1e-6 * scale
    assert (g3 - g1).abs().max().item() <= 2e-6 * scale
    # zero cotangents give an exactly zero gradient
    g0 = model.vjp(params, x, torch.zeros_like(ct)).flat
    assert g0.abs().max().item() == 0.0


def test_param_tree_upload_paths_agree(cuda):
    """A ParamTree (flat buffer, uploaded as is) and a dict of separate tensors give
    bit-identical log psi; the library's on-device packing (folds Wo Wl, W0 Wqkv) is
    what both go through."""
    ocfg = oracle_config("C2")
    system, model = build(ocfg)
    tree = model.init(11, device=cuda)
    assert isinstance(tree, ParamTree) and tree.is_packed_view(model.spec)
    loose = {k: v.clone() for k, v in tree.items()}
    x = torch.tensor(make_walkers(16, ocfg.nelec, seed=2), device=cuda)
    a = model.apply(tree, x)
    b = model.apply(loose, x)
    assert torch.equal(a, b)
    assert torch.equal(flat_params(model.spec, loose, cuda), tree.flat)
    # in-place update through a view is seen (shared version counter)
    tree["PsiformerLayers_0/Dense_1/kernel"].mul_(0.5)
    c = model.apply(tree, x)
    assert not torch.equal(a, c)


def test_energy_grad_loss_matches_oracle(cuda):
    """make_loss_fn(ENERGY_GRAD) end to end: E_L -> stats -> clipped diff -> weights ->
    reverse mode, against the oracle's loss.py:66-106 on the same walkers."""
    ocfg = oracle_config("C1")
    p64 = make_params(ocfg)
    system, model = build(ocfg)
    params = to_device_params(p64)
    B = 12
    x = make_walkers(B, ocfg.nelec, seed=4)
    loss = make_loss_fn(model, system, LossMode.ENERGY_GRAD)
    stats, grad = loss(params, torch.tensor(x, device=cuda))
    xt = torch.tensor(x, dtype=torch.float64)
    el, obs = R.local_energy(p64, ocfg, xt)
    el = el.detach().numpy()
    o = {k: v.detach().numpy() for k, v in obs.items()}
    st = R.loss_stats(el, o, penalties=True)
    diff = R.loss_diff(el, o, st)
    n = np.sum(~np.isnan(diff))
    ct = np.stack([2 * diff.real / n, 2 * diff.imag / n], -1)
    ref = R.logpsi_param_grad(p64, ocfg, xt, ct)
    errs = grad_errors(grad, ref)
    worst = max(errs, key=errs.get)
    # the diff weights carry the E_L error (f32 Hessian-level), hence the looser bound
    assert errs[worst] < 2e-4, (worst, errs[worst])
    assert float(stats["energy"].real) == pytest.approx(float(np.mean(el.real)), rel=1e-5)


def test_adam_matches_optax_semantics(cuda):
    ocfg = oracle_config("C1")
    system, model = build(ocfg)
    params = model.init(1, device=cuda)
    p0 = {k: v.detach().double().cpu().clone() for k, v in params.items()}
    st = AdamState(params)
    lr = config.LearningRate(rate=0.05, decay=1.0, delay=3.0)
    rng = np.random.default_rng(0)
    seq = []
    for t in range(4):
        g = ParamTree.zeros(model.spec, cuda)
        g.flat.copy_(torch.tensor(rng.standard_normal(g.flat.numel()), dtype=torch.float32))
        if t == 2:
            g.flat[5] = float("nan")  # nan_to_num (loss.py:64)
        seq.append({k: v.detach().double().cpu() for k, v in g.items()})
        adam_update(params, g, st, lr_schedule(lr, st.count))
    ref = R.adam_reference(p0, seq, lambda t: lr_schedule(lr, t))
    for k in ref:
        got = params[k].detach().double().cpu()
        assert torch.allclose(got, ref[k], rtol=1e-5, atol=1e-6), k


def test_singular_walker_does_not_poison_gradient(cuda):
    """a walker with two coincident electrons has psi = 0 (two equal orbital
    rows), a NaN E_L and therefore a zero cotangent (nanmean / nan_to_num drop it,
    loss.py:59-64).  The reverse pass must skip it — its inverse is inf and 0 * inf would
    put NaN into every weight gradient — so the gradient equals the one without it."""
    ocfg = oracle_config("C1")
    p64 = make_params(ocfg)
    system, model = build(ocfg)
    params = to_device_params(p64)
    x = make_walkers(6, ocfg.nelec, seed=8)
    x[2, 1] = x[2, 0]  # coincident electrons
    ct = np.random.default_rng(9).standard_normal((6, 2)).astype(np.float32)
    ct[2] = 0.0
    lp = torch.empty(6, 2, device=cuda)
    g_all = model.vjp(params, torch.tensor(x, device=cuda), torch.tensor(ct, device=cuda), logpsi=lp)
    assert not np.isfinite(lp[2, 0].item())  # psi = 0 for the coincident walker
    keep = [0, 1, 3, 4, 5]
    g_ref = model.vjp(params, torch.tensor(x[keep], device=cuda), torch.tensor(ct[keep], device=cuda))
    assert torch.isfinite(g_all.flat).all()
    scale = g_ref.flat.abs().max().item()
    assert (g_all.flat - g_ref.flat).abs().max().item() <= 1e-6 * scale
    # through the loss: E_L of that walker is NaN, the gradient stays finite
    _, grad = make_loss_fn(model, system, LossMode.ENERGY_GRAD)(params, torch.tensor(x, device=cuda))
    assert torch.isfinite(grad.flat).all()
