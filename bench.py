"""Benchmark: the DeepHall VMC inner loop on MI355X (BASELINE.json metric).

One "step" = one VMC iteration of the reference's loop body (train.py:126-140)
without the optimizer: ``mcmc_step`` (10 all-electron Metropolis moves = 11
log-psi evaluations per walker, mcmc.py:122-148) + the local energy of every
walker (hamiltonian.py:175-212) + the device statistics and ONE packed
all-reduce (loss.py:66-92).  Workload: BASELINE.json configs[1] — nspins=[6,0],
flux=15, default Psiformer (4 heads x 64, 2 layers, 1 determinant), 4096
walkers per GPU, random-init weights, walkers from init_guess + burn-in.

value = local energies per second over all GPUs (= walkers x GPUs / step time), each
timed step ending in the host sync of the reference loop (the width adaptation reads
pmove, mcmc.py:180).  walker_steps_per_sec = B x steps / t(mcmc_step call) from a
separate region of >= 20 mcmc_step calls (each with its pmove all-reduce and host sync,
SURVEY.md §8d).  Multi-GPU: weak scaling, walkers sharded, one all-reduce of 16 floats
per step.  ``--gpus N`` without a torchrun environment starts N rank processes itself
(one GPU each, RCCL) before anything touches the GPU; rank 0 prints the line.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "local-energies/sec + MCMC walker-steps/sec, N={N} 2Q={flux}, 1/2/4/8 GPUs"  # BASELINE.json metric
PEAK_F32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: Peak FP32 (matrix), dense
PEAK_BF16_MFMA_TFLOPS = 16 * PEAK_F32_MFMA_TFLOPS  # same guide: f32 MFMA = 1/16 of BF16 (~2.5 PF dense)
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096, help="walkers per GPU")
    ap.add_argument("--nspins", type=int, nargs=2, default=[6, 0])
    ap.add_argument("--flux", type=int, default=15)
    ap.add_argument("--mcmc-steps", type=int, default=10)
    ap.add_argument("--burn-in", type=int, default=5)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-components", action="store_true",
                    help="skip the MCMC-only / E_L-only timings (used under rocprofv3 so that every "
                    "profiled GEMM launch belongs to a warmup or timed VMC step)")
    ap.add_argument("--groups", type=int, default=1,
                    help="walker groups run on parallel HIP streams within one VMC iteration")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="do not record per-kernel HIP events in the timed region (no roofline)")
    ap.add_argument("--mcmc-calls", type=int, default=20, help="timed mcmc_step calls for walker_steps_per_sec")
    ap.add_argument("--extra-configs", default="C4,C5",
                    help="comma list of EXTRA_CONFIGS also timed (one-GPU lines in configs_1gpu; '' = none)")
    ap.add_argument("--extra-steps", type=int, default=3)
    ap.add_argument("--extra-mcmc-calls", type=int, default=5,
                    help="timed mcmc_step calls for the C4 / C5 lines' walker_steps_per_sec")
    ap.add_argument("--extra-warmup", type=int, default=2)
    ap.add_argument("--cpu-c1-seconds", type=float, default=6.0,
                    help="CPU-baseline budget for BASELINE.json configs[0] (N=3 2Q=2, B=100)")
    return ap.parse_args()


def spawn_ranks(n: int) -> int:
    """torchrun-style launch of n rank processes of this script (one GPU each).  The parent
    makes no GPU call; rank 0's stdout (the JSON line) is passed through."""
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = procs[0].stdout.read().decode()
    rcs = [p.wait() for p in procs]
    sys.stdout.write(out)
    sys.stdout.flush()
    return max(abs(rc) for rc in rcs)


EXTRA_CONFIGS = {"C4": ((10, 0), 23), "C5": ((20, 0), 57)}  # BASELINE.json configs[3], [4]


def run_workload(args, dev, rank, world, nspins, flux, B, n_steps, n_warmup, burn_in, instrument, components,
                 mcmc_calls=None):
    """One workload: burn-in, W warmup VMC steps, exactly K timed steps (barrier + sync on both
    sides, max over ranks), then the instrumented region and the component timings."""
    from deephall_amd import _lib, config
    from deephall_amd.hamiltonian import _run_local_energy
    from deephall_amd.loss import device_stats, reduce_stats
    from deephall_amd.mcmc import make_mcmc_step, update_mcmc_width
    from deephall_amd.networks import make_network
    from deephall_amd.networks.psiformer import get_handle
    from deephall_amd.random import Key, PRNGKey
    from deephall_amd.train import init_guess, make_vmc_iteration

    lib = _lib.load()
    system = config.System(nspins=tuple(nspins), flux=flux)
    model = make_network(system, config.Network())
    N = sum(nspins)
    params = model.init(PRNGKey(42), device=dev)
    data = init_guess(Key(4242), B, N, dev, walker_offset=rank * B, network=model)
    steps = args.mcmc_steps
    mcmc_step = make_mcmc_step(model, batch_per_device=B, steps=steps)
    key = PRNGKey(7)
    width = 0.1

    iteration = make_vmc_iteration(model, B, steps, args.groups)
    iteration1 = make_vmc_iteration(model, B, steps, 1)  # instrumented region: one stream

    import numpy as np

    pmoves = np.zeros(100)
    t_iter = [0]

    def vmc_step(data, key, it=iteration):
        nonlocal width, pmoves
        data, e_l, obs, n_accept = it(params, data, key, width)
        local_stats = device_stats(model, e_l, obs, n_accept, steps)
        stats = reduce_stats(local_stats)  # the one all-reduce of the step
        # host side of the reference loop: width adaptation reads pmove (a device sync,
        # mcmc.py:180 / train.py:131-137)
        width, pmoves = update_mcmc_width(t_iter[0], width, 100, stats["pmove"], pmoves)
        t_iter[0] += 1
        return data, stats

    for _ in range(burn_in):
        data, _ = mcmc_step(params, data, key, width, reduce=False)
        key = key.advance(steps)
    for _ in range(n_warmup):
        data, stats = vmc_step(data, key)
        key = key.advance(steps)
    h = get_handle(model.spec, dev)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    # ---------------- timed region: exactly K steps, no instrumentation
    barrier()
    t0 = time.perf_counter()
    for _ in range(n_steps):
        data, stats = vmc_step(data, key)
        key = key.advance(steps)
    barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    energy = complex(stats["energy"].item())
    pmove = float(stats["pmove"].item())

    # ---------------- instrumented region: the same K steps again with a HIP event pair
    # around every kernel launch (on the launch stream), for the per-kernel breakdown and
    # the roofline.  The events themselves cost ~10 % of a step, so `value` comes from the
    # un-instrumented region above; the walker groups run one after the other here so
    # that each launch's duration is its own.
    import ctypes as C

    prof = (C.c_double * (4 * len(_lib.PROF_KINDS)))()
    dt_prof = float("nan")
    if instrument:
        lib.dh_profile_enable(h.h, 1)
        barrier()
        a = time.perf_counter()
        for _ in range(n_steps):
            data, _ = vmc_step(data, key, iteration1)  # kernels one at a time: clean durations
            key = key.advance(steps)
        barrier()
        dt_prof = time.perf_counter() - a
        lib.dh_profile_read(h.h, prof, 1)
        lib.dh_profile_enable(h.h, 0)

    # ---------------- MCMC walker-steps/s: >= 20 mcmc_step calls, each with
    # its pmove all-reduce and the host read of pmove; then the E_L-only rate
    t_mcmc = t_el = float("nan")
    mcmc_calls = mcmc_calls or args.mcmc_calls
    if components:
        barrier()
        a = time.perf_counter()
        for _ in range(mcmc_calls):
            data, pm = mcmc_step(params, data, key, width)
            float(pm)  # device sync, as pmove.item() in update_mcmc_width
            key = key.advance(steps)
        barrier()
        t_mcmc = time.perf_counter() - a
        tm = torch.tensor([t_mcmc], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        t_mcmc = float(tm.item()) / mcmc_calls
        a = time.perf_counter()
        for _ in range(3):
            _run_local_energy(model, params, data)
        barrier()
        t_el = (time.perf_counter() - a) / 3

    return dict(dt=dt, dt_prof=dt_prof, prof=list(prof), t_mcmc=t_mcmc, t_el=t_el, energy=energy, pmove=pmove)


def kernels_of(prof, n_steps):
    from deephall_amd import _lib

    kern = {}
    for i, k in enumerate(_lib.PROF_KINDS):
        cnt, ms, fl, by = prof[4 * i : 4 * i + 4]
        if cnt:
            kern[k] = {"launches_per_step": cnt / n_steps, "ms_per_step": ms / n_steps, "avg_us": 1e3 * ms / cnt}
    return kern


def roofline_of(prof, n_steps, dt_prof, x6, traffic=None, traffic_src=None):
    """Dominant kernel class: the local-energy channel GEMMs (class gemm_ch of dh_profile_read; in
    the split-bf16 modes gemm_x6m_kernel for the wide maps and gemm_lnch_kernel, GEMM + channel
    LayerNorm, for the 256-column ones at N <= 6).  Its arithmetic runs as 6 bf16 MFMA products per
    f32 product, so the ceiling of its algorithmic f32 flop rate is the dense bf16 MFMA peak / 6.
    The log-psi GEMMs (class gemm) are reported beside it."""
    from deephall_amd import _lib

    kinds = _lib.PROF_KINDS

    def _cls(name):
        i = kinds.index(name)
        return prof[4 * i], prof[4 * i + 1], prof[4 * i + 2], prof[4 * i + 3]

    g_cnt, g_ms, g_fl, g_by = _cls("gemm_ch")
    l_cnt, l_ms, l_fl, l_by = _cls("gemm")
    f_cnt, f_ms, f_fl, f_by = _cls("layer1_ch")
    achieved = (g_fl / (g_ms * 1e-3)) / 1e12 if g_ms > 0 else 0.0
    peak = PEAK_BF16_MFMA_TFLOPS / 6 if x6 else PEAK_F32_MFMA_TFLOPS
    return {
        "kernel": ("local-energy channel GEMMs (the 256-deep ones), split-bf16 f32 GEMM "
                   "(v_mfma_f32_16x16x32_bf16): gemm_x6m_kernel (layer 2's q|k|v and the orbital map) + "
                   "gemm_lnch_kernel (layer 2's two 256-column maps with the channel LayerNorm fused in; "
                   f"its LN work counted in the launch time, not in the flops), averaged over the "
                   f"{g_cnt / n_steps:g} launches per step"
                   if x6 else "gemm_ntp_kernel (exact-f32 channel GEMMs)"),
        "bound": "mfma",
        "achieved": round(achieved, 2),
        "peak": round(peak, 1),
        "unit": "TFLOP/s",
        "frac": round(achieved / peak, 4),
        "traffic": traffic,
        "peak_basis": ("dense bf16 MFMA 2516.8 TF/s / 6 bf16 products per f32 product "
                       "(algorithmic f32 flops)" if x6 else "dense f32 MFMA 157.3 TF/s"),
        "achieved_over_f32_mfma_peak": round(achieved / PEAK_F32_MFMA_TFLOPS, 4),
        "flops_per_launch": g_fl / g_cnt if g_cnt else 0,
        "avg_launch_us": 1e3 * g_ms / g_cnt if g_cnt else 0,
        "share_of_step": round(g_ms / (dt_prof * 1e3), 4) if g_ms else None,
        "measured_over": f"{n_steps} instrumented VMC steps (HIP event pair per launch)",
        "traffic_source": traffic_src,
        "bytes_per_launch_algorithmic": g_by / g_cnt if g_cnt else 0,
        "layer1_ch": {  # gemm_lnch MODE 2: layer 1 whole (LayerNorms, tanh, three 32-deep products)
            "launches_per_step": f_cnt / n_steps,
            "avg_launch_us": 1e3 * f_ms / f_cnt if f_cnt else 0,
            "share_of_step": round(f_ms / (dt_prof * 1e3), 4) if f_ms else None,
        } if f_cnt else None,
        "logpsi_gemms": {
            "launches_per_step": l_cnt / n_steps,
            "avg_launch_us": 1e3 * l_ms / l_cnt if l_cnt else 0,
            "achieved_tflops": round((l_fl / (l_ms * 1e-3)) / 1e12, 2) if l_ms > 0 else 0.0,
            "share_of_step": round(l_ms / (dt_prof * 1e3), 4) if l_ms else None,
        },
    }


def f_fwd(N, flux):
    """Forward flops per walker, default Psiformer (D = 256, 2 layers, 1 det)."""
    return 2 * N * 4 * 256 + 2 * (12 * N * 256**2 + 4 * N * N * 256) + 4 * N * 256 * (flux + 1) * N

def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for the multi-rank path on a one-GPU box (never set by the driver):
    # DH_BENCH_BACKEND=gloo, DH_BENCH_ONE_GPU=1 puts every rank on device 0
    if os.environ.get("DH_BENCH_ONE_GPU"):
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group(os.environ.get("DH_BENCH_BACKEND", "nccl"))
    dev = torch.device("cuda", local if world > 1 else torch.cuda.current_device())


    B = args.batch
    N = sum(args.nspins)
    r = run_workload(args, dev, rank, world, tuple(args.nspins), args.flux, B, args.steps, args.warmup,
                     args.burn_in, not args.no_kernel_events, not args.no_components)
    dt, dt_prof, prof, t_mcmc, t_el = r["dt"], r["dt_prof"], r["prof"], r["t_mcmc"], r["t_el"]
    energy, pmove = r["energy"], r["pmove"]
    steps = args.mcmc_steps
    # the other BASELINE.json configs with a larger N (configs[3] N=10 2Q=23, configs[4] N=20 2Q=57),
    # one-GPU weak-scaling lines of the same VMC iteration (4096 walkers per GPU), a few steps each
    extra = {}
    if args.extra_configs and world == 1:  # one-GPU lines: not repeated by the multi-rank runs
        for tag in args.extra_configs.split(","):
            nsp, fx = EXTRA_CONFIGS[tag]
            rx = run_workload(args, dev, rank, world, nsp, fx, B, args.extra_steps, args.extra_warmup, 2,
                              not args.no_kernel_events, not args.no_components, args.extra_mcmc_calls)
            extra[tag] = (nsp, fx, rx)

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    kern = kernels_of(prof, args.steps)
    from deephall_amd.networks import psiformer as _pf

    gemm_mode = _pf._GEMM_MODE
    x6 = gemm_mode in ("x6", "x6all")
    # HBM traffic per channel-GEMM launch: rocprofv3 PMC (FETCH_SIZE x2 + WRITE_SIZE, separate
    # passes) of this same workload, committed by tools/profile_round.sh; default config only
    traffic = traffic_src = None
    tf = ROOT / "profiles" / "gemm_traffic.json"
    if tf.exists() and (B, tuple(args.nspins), args.flux, steps) == (4096, (6, 0), 15, 10):
        tj = json.loads(tf.read_text())
        traffic = tj.get("channel_gemm_bytes_per_launch") if x6 else None
        traffic_src = f"profiles/gemm_traffic.json ({tj.get('tag', '?')})" if traffic else None
    roofline = roofline_of(prof, args.steps, dt_prof, x6, traffic, traffic_src) if not args.no_kernel_events else None
    # MFMA utilisation of the same kernels: rocprofv3 PMC SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8
    # x 1024 SIMDs) of this workload (tools/pmc_mfma.py, committed by tools/profile_round.sh)
    mf = ROOT / "profiles" / "mfma_pmc.json"
    if roofline and mf.exists() and (B, tuple(args.nspins), args.flux, steps) == (4096, (6, 0), 15, 10):
        mj = json.loads(mf.read_text())
        ks = mj.get("kernels", {})

        def busy_of(pat):
            import re as _re
            sel = {k: v for k, v in ks.items() if _re.search(pat, k)}
            w = sum(v["avg_us"] * v["dispatches"] for v in sel.values())
            return (round(sum(v["mfma_busy"] * v["avg_us"] * v["dispatches"] for v in sel.values()) / w, 4) if w else None,
                    {k: v["mfma_busy"] for k, v in sel.items()})
        ch, ch_k = busy_of(r"gemm_x6m_kernel|gemm_lnch_kernel<\d+, [01]")
        lp, lp_k = busy_of(r"chain_x6s_kernel")
        roofline["mfma_busy"] = {"channel_gemms": ch, "logpsi_chain": lp, "per_kernel": {**ch_k, **lp_k},
                                 "source": f"profiles/mfma_pmc.json ({mj.get('tag', '?')})",
                                 "definition": "MFMA cycles / (dispatch cycles x 1024 SIMDs), time-weighted"}
    B_total = B * world
    value = B_total * args.steps / dt
    F_fwd = f_fwd(N, args.flux)
    metric = METRIC.format(N=N, flux=args.flux)
    out = {
        "metric": metric,
        "value": round(value, 1),
        "unit": "local-energies/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * dt / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (init_guess walkers + burn-in, random-init Psiformer weights)",
        "config": {
            "workload": f"VMC iteration (mcmc_step {steps} MH moves + local energy + stats all-reduce), "
            f"nspins={list(args.nspins)} flux={args.flux}, Psiformer 4x64 heads, 2 layers, 1 det",
            "walkers_per_gpu": B,
            "global_batch": B_total,
            "parallelism": f"walker-dp{world}",
            "walker_groups_per_gpu": args.groups,
            "gemm_arithmetic": gemm_mode,
        },
        "walker_steps_per_sec": round(B_total * steps / t_mcmc, 1) if t_mcmc == t_mcmc else None,
        "walker_steps_per_sec_def": (f"B_total x steps / t(mcmc_step call), mean of {args.mcmc_calls} calls incl. "
                                     "the initial log-psi pass, the pmove all-reduce and the host sync"),
        "components": {
            "mcmc_step_ms": round(1e3 * t_mcmc, 3),
            "local_energy_ms": round(1e3 * t_el, 3),
            "local_energies_per_sec_el_only": round(B_total / t_el, 1),
            "model_tflops_el_only": round(B_total * (2 * N + 5) * F_fwd / t_el / 1e12, 2),
            "model_tflops_mcmc_only": round(B_total * (steps + 1) * F_fwd / t_mcmc / 1e12, 2),
        } if not args.no_components else None,
        "ms_per_step_instrumented": round(1e3 * dt_prof / args.steps, 3) if dt_prof == dt_prof else None,
        "kernels": kern,
        "roofline": roofline,
        "energy": [round(energy.real, 5), round(energy.imag, 5)],
        "pmove": round(pmove, 3),
    }
    if extra:
        out["configs_1gpu"] = {}
        for tag, (nsp, fx, rx) in extra.items():
            n = sum(nsp)
            rl = roofline_of(rx["prof"], args.extra_steps, rx["dt_prof"], x6) if not args.no_kernel_events else None
            out["configs_1gpu"][tag] = {
                "config": f"nspins={list(nsp)} flux={fx} (BASELINE.json configs[{3 if tag == 'C4' else 4}], "
                          f"{B} walkers per GPU, weak scaling)",
                # a one-GPU line: this rank's walkers over the max-over-ranks time (B, not
                # B_total: with --gpus > 1 the ranks run these configs side by side)
                "value": round(B * args.extra_steps / rx["dt"], 1),
                "unit": "local-energies/s",
                "steps": args.extra_steps,
                "warmup": args.extra_warmup,
                "ms_per_step": round(1e3 * rx["dt"] / args.extra_steps, 3),
                "roofline": {k: rl[k] for k in ("bound", "achieved", "peak", "unit", "frac", "avg_launch_us",
                                                "flops_per_launch", "share_of_step")} if rl else None,
                "kernels_ms_per_step": {k: round(v["ms_per_step"], 3)
                                        for k, v in kernels_of(rx["prof"], args.extra_steps).items()},
                "energy": [round(rx["energy"].real, 5), round(rx["energy"].imag, 5)],
                "walker_steps_per_sec": round(B * args.mcmc_steps / rx["t_mcmc"], 1) if rx["t_mcmc"] == rx["t_mcmc"] else None,
                "walker_steps_per_sec_def": f"B x steps / t(mcmc_step call), mean of {args.extra_mcmc_calls} calls",
                "mcmc_step_ms": round(1e3 * rx["t_mcmc"], 3) if rx["t_mcmc"] == rx["t_mcmc"] else None,
                "local_energies_per_sec_el_only": round(B / rx["t_el"], 1) if rx["t_el"] == rx["t_el"] else None,
                "model_tflops_step": round(B * (2 * n + 5 + args.mcmc_steps + 1) * f_fwd(n, fx)
                                           / rx["dt"] * args.extra_steps / 1e12, 2),
            }
    if world == 1 and not args.no_cpu_baseline:
        from oracle import cpu_baseline
        from oracle.reference import OracleConfig

        # the GPU box gives one GPU's job a 16-CPU share (os.cpu_count() reports the whole host)
        threads = min(16, os.cpu_count() or 1)
        cb = cpu_baseline.measure(
            OracleConfig(nspins=tuple(args.nspins), flux=args.flux), steps=steps,
            budget_s=args.cpu_baseline_seconds, threads=threads,
        )
        c1 = cpu_baseline.measure(OracleConfig(nspins=(3, 0), flux=2), steps=steps, budget_s=args.cpu_c1_seconds,
                                  threads=threads, el_batch=20, fwd_batch=100)
        out["cpu_baseline"] = {
            "value": round(cb["local_energies_per_sec"], 3),
            "unit": "local-energies/s",
            "cores": cb["threads"],
            "kind": "port",
            "sample": cb["sample"],
            "cpu_model": cb["cpu_model"],
            "host_cpus": cb["host_cpus"],
            "cores_note": "16 threads = the CPU share gpurun gives a one-GPU job (the host has more cores)",
            "walker_steps_per_sec": round(cb["walker_steps_per_sec"] * steps / (steps + 1), 1),
            "el_only_per_sec": round(cb["el_only_per_sec"], 3),
            "c1": {"config": "nspins=[3,0] flux=2 (BASELINE.json configs[0]), vmap batches of the B=100 walkers",
                   "local_energies_per_sec": round(c1["local_energies_per_sec"], 3),
                   "walker_steps_per_sec": round(c1["walker_steps_per_sec"] * steps / (steps + 1), 1),
                   "sample": c1["sample"]},
        }
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
