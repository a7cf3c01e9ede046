"""Rank process of tests/test_gpu_0_multirank.py (not a test module).

``worker.py OUT [MODE]``, every rank on device 0 with the gloo backend (a one-GPU box;
the 8-GPU runs use RCCL), writing argv[1]_<rank>.npz:

* ``vmc`` (default): one VMC iteration's device work on this rank's contiguous walker
  shard — mcmc_step with its pmove pmean, the local energy, dh_energy_stats and the
  packed statistics all-reduce; the rank's walkers, accept counts and reduced statistics.
* ``grad``: make_loss_fn(ENERGY_GRAD) on fixed walkers (loss.py:66-108): the statistics
  all-reduce, the clipped difference, reverse mode and the gradient all-reduce.
* ``train``: train() (train.py:80-167) with Adam for 2 iterations, checkpoint every
  step (save_time_interval 0, save_step_interval 1: the collective save decision),
  the run directory in argv[3]; the final parameters and this rank's walkers.
* ``nccl``: a world-size-1 "nccl" (RCCL) process group and one all-reduce on the GPU.
* ``kfac``: the default optimizer across ranks (optimizers/kfac.py:195-241, multi_device):
  make_loss_fn(ENERGY_GRAD, curvature=True) on fixed walkers (the ONE [gradient | curvature
  statistics] all-reduce), then two KFAC steps of make_optimizer_step on them; the averaged
  gradient and statistics, the parameters after each step and the preconditioned gradient.
"""

from __future__ import annotations

import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main_grad(out, world, rank):
    from deephall_amd import config, make_network
    from deephall_amd.loss import LossMode, make_loss_fn
    from helpers import make_walkers

    system = config.System(nspins=(6, 0), flux=15)
    model = make_network(system, config.Network())
    params = model.init(3, device="cuda")
    B = 64
    per = B // world
    x = torch.tensor(make_walkers(B, 6, seed=5)[rank * per : (rank + 1) * per], device="cuda")
    stats, grad = make_loss_fn(model, system, LossMode.ENERGY_GRAD)(params, x)
    torch.cuda.synchronize()
    np.savez(f"{out}_{rank}.npz", grad=grad.flat.cpu().numpy(), energy=complex(stats["energy"].item()))


def main_train(out, world, rank, run_dir):
    from deephall_amd import Config, train

    cfg = Config.from_dict({
        "batch_size": 60, "seed": 42,
        "system": {"nspins": (3, 0), "flux": 2, "interaction_strength": 0.0},
        "network": {"psiformer": {"num_layers": 1, "num_heads": 1, "heads_dim": 4}},
        "mcmc": {"burn_in": 4},
        "optim": {"iterations": 2, "optimizer": "adam", "adam": {"lr": {"rate": 0.02}}},
        "log": {"save_path": run_dir, "save_time_interval": 0, "save_step_interval": 1},
    })
    state = train(cfg)
    torch.cuda.synchronize()
    np.savez(f"{out}_{rank}.npz", params=state.params.flat.cpu().numpy(), data=state.data.cpu().numpy(),
             width=float(state.mcmc_width))


def main_kfac(out, world, rank):
    from deephall_amd import Config, make_network
    from deephall_amd.loss import _kfac_buffer
    from deephall_amd.mcmc import resolve_network
    from deephall_amd.loss import LossMode, make_loss_fn
    from deephall_amd.optimizers import make_optimizer_step
    from deephall_amd.types import CheckpointState
    from helpers import make_walkers

    cfg = Config.from_dict({
        "batch_size": 64, "seed": 42,
        "system": {"nspins": (3, 0), "flux": 2},
        "network": {"psiformer": {"num_layers": 2, "num_heads": 2, "heads_dim": 16}},
        "optim": {"optimizer": "kfac"},
    })
    model = make_network(cfg.system, cfg.network)
    params = model.init(11, device="cuda")
    B = 64
    per = B // world
    x = torch.tensor(make_walkers(B, 3, seed=21)[rank * per : (rank + 1) * per], device="cuda")
    loss_grad = make_loss_fn(model, cfg.system, LossMode.ENERGY_GRAD, curvature=True)
    stats, grad = loss_grad(params, x)
    g0 = grad.flat.clone()
    curv = loss_grad.curvature.clone()
    extra = {}
    if world == 1:  # the per-shard statistics two ranks would average (kfac_jax multi_device)
        for hh, hx in enumerate((x[: B // 2], x[B // 2:])):
            loss_grad(params, hx.contiguous())
            extra[f"curv_h{hh}"] = loss_grad.curvature.cpu().numpy().copy()
    # generic (NaiveDiagonal) parameters: their statistic is not additive over shards
    gmask = torch.zeros_like(params.flat, dtype=torch.bool)
    for k in params:
        if "LayerNorm" in k or "Jastrow" in k or "lll_weight/bias" in k:
            off = params[k].data_ptr() - params.flat.data_ptr()
            gmask[off // 4: off // 4 + params[k].numel()] = True
    init, step = make_optimizer_step(cfg, model)
    state = CheckpointState(params, x, init(params), 0.1)
    p0 = params.flat.clone()
    snaps, pgs, inputs = [], [], []
    for _ in range(2):
        state, _ = step(state)
        snaps.append(state.params.flat.clone())
        pgs.append(state.opt_state.pgrad.clone())
        # the step's all-reduced [gradient | curvature statistics] (the loss fn's cached buffer)
        buf, nref = _kfac_buffer(resolve_network(model), x.device)
        inputs.append(buf.clone())
    torch.cuda.synchronize()
    if world > 1 and rank == 0:
        extra.update(_kfac_oracle_two_steps(model, cfg, p0, snaps[0], inputs, nref, world, B))
    np.savez(f"{out}_{rank}.npz", grad=g0.cpu().numpy(), curv=curv.cpu().numpy(), p0=p0.cpu().numpy(),
             p1=snaps[0].cpu().numpy(), p2=snaps[1].cpu().numpy(), pg1=pgs[0].cpu().numpy(),
             pg2=pgs[1].cpu().numpy(), info=state.opt_state.info.cpu().numpy(), gmask=gmask.cpu().numpy(),
             energy=complex(stats["energy"].item()), **extra)


def _kfac_oracle_two_steps(model, cfg, p0, p1, inputs, nref, world, B):
    """the two-rank run's two KFAC steps against oracle/kfac.py fed the
    SAME per-step inputs — each step's all-reduced gradient and curvature statistics, as the
    ranks hold them — with float32 EMA storage (as tests/test_gpu_kfac.py).  Also the oracle's
    own two-shard statistics (kfac_jax multi_device: per-device statistics, averaged) at the
    step-2 parameters, against the statistics the ranks all-reduced there.  Returns the
    oracle's P g / parameters per step and the statistics' relative errors."""
    from deephall_amd.networks.psiformer import ParamTree
    from helpers import make_walkers
    from oracle import kfac as KF
    from oracle import reference as R

    ocfg = R.OracleConfig(nspins=tuple(cfg.system.nspins), flux=cfg.system.flux,
                          num_heads=cfg.network.psiformer.num_heads, heads_dim=cfg.network.psiformer.heads_dim,
                          num_layers=cfg.network.psiformer.num_layers)
    lay = model.kfac_layout(p0.device)
    blocks, generic = KF.blocks(ocfg)
    assert len(blocks) == len(lay["blocks"])

    def tree(flat):
        t = ParamTree.view_of(model.spec, flat.to(p0.device))
        return {k: t[k].double().cpu() for k in t}

    def unpack(curv):
        curv = curv.double().cpu()
        stats = {}
        for ob, gb in zip(blocks, lay["blocks"]):
            (na, oa), (ng, og) = lay["slots"][gb["a_slot"]], lay["slots"][gb["g_slot"]]
            stats[ob.name] = (curv[oa: oa + na * na].reshape(na, na), curv[og: og + ng * ng].reshape(ng, ng))
        diag, o = {}, lay["nmat"]
        shapes = tree(p0)
        for g in generic:
            n = shapes[g].numel()
            diag[g] = curv[o: o + n].reshape(shapes[g].shape)
            o += n
        return stats, diag

    ema = float(np.float32(0.95))  # the float32 EMA factor the kernels see
    state = KF.KfacState()
    p_ref = tree(p0)
    res = {}
    for s, buf in enumerate(inputs, start=1):
        grads = tree(buf[:nref])
        stats, diag = unpack(buf[nref:])
        p_ref, state, inf = KF.kfac_step(p_ref, ocfg, grads, state, stats, diag, storage=torch.float32, ema=ema)
        flat = ParamTree.zeros(model.spec, p0.device)
        pgt = ParamTree.zeros(model.spec, p0.device)
        for k in p_ref:
            flat[k].copy_(p_ref[k].float().reshape(flat[k].shape))
            pgt[k].copy_(inf["pg"][k].float().reshape(pgt[k].shape))
        res[f"oracle_p{s}"] = flat.flat.cpu().numpy()
        res[f"oracle_pg{s}"] = pgt.flat.cpu().numpy()
        res[f"oracle_coef{s}"] = inf["coef"]
    # the oracle's two-shard statistics at the parameters of step 2 (the ranks' step-1 result)
    xs = torch.tensor(make_walkers(B, ocfg.nelec, seed=21), dtype=torch.float64)
    ref, rdiag = KF.batch_statistics(tree(p1), ocfg, xs, shards=world)
    got, gdiag = unpack(inputs[1][nref:])
    errs = []
    for k, (A, G) in ref.items():
        errs.append(float((got[k][0] - A).abs().max() / A.abs().max()))
        errs.append(float((got[k][1] - G).abs().max() / G.abs().max()))
    gen_ref = torch.cat([rdiag[g].reshape(-1) for g in generic])
    gen_got = torch.cat([gdiag[g].reshape(-1) for g in generic])
    res["stat2_err_dense"] = max(errs)
    res["stat2_err_generic"] = float((gen_got - gen_ref).abs().max() / gen_ref.abs().max())
    return res


def main_nccl(out):
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    from deephall_amd import constants

    t = torch.arange(16, dtype=torch.float32, device="cuda")
    dist.all_reduce(t)
    m = constants.pmean(torch.ones(3, device="cuda") * 2.5)
    torch.cuda.synchronize()
    np.savez(f"{out}_0.npz", t=t.cpu().numpy(), m=m.cpu().numpy(), backend=dist.get_backend())
    dist.destroy_process_group()


def main():
    out = sys.argv[1]
    mode = sys.argv[2] if len(sys.argv) > 2 else "vmc"
    if mode == "nccl":
        torch.cuda.set_device(0)
        return main_nccl(out)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(0)
    if world > 1:
        dist.init_process_group("gloo")
    if mode == "grad":
        main_grad(out, world, rank)
    elif mode == "train":
        main_train(out, world, rank, sys.argv[3])
    elif mode == "kfac":
        main_kfac(out, world, rank)
    else:
        main_vmc(out, world, rank)
    if world > 1:
        dist.destroy_process_group()


def main_vmc(out, world, rank):
    from deephall_amd import config, make_network
    from deephall_amd.hamiltonian import _run_local_energy
    from deephall_amd.loss import device_stats, reduce_stats
    from deephall_amd.mcmc import make_mcmc_step
    from deephall_amd.random import Key
    from helpers import make_params, make_walkers, oracle_config, to_device_params

    ocfg = oracle_config("C2")
    system = config.System(nspins=ocfg.nspins, flux=ocfg.flux)
    model = make_network(system, config.Network())
    params = to_device_params(make_params(ocfg))
    B = 64
    per = B // world
    xs = make_walkers(B, ocfg.nelec, seed=3)[rank * per : (rank + 1) * per]
    x = torch.tensor(xs, device="cuda")
    step = make_mcmc_step(model, batch_per_device=per, steps=4)
    x, pmove = step(params, x, Key(77, 5), 0.15)  # walker_offset = rank * per, pmean of pmove
    nacc = step.last_n_accept
    e_l, obs = _run_local_energy(model, params, x)
    stats = reduce_stats(device_stats(model, e_l, obs, nacc, 4))
    torch.cuda.synchronize()
    np.savez(f"{out}_{rank}.npz", x=x.cpu().numpy(), n_acc=nacc.cpu().numpy(), mcmc_pmove=float(pmove),
             e_l=e_l.cpu().numpy(), **{k: complex(v.item()) for k, v in stats.items()})


if __name__ == "__main__":
    main()
