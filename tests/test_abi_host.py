"""C ABI + host logic without a GPU: the library loads, exports every symbol the
header declares, validates configs, reports the packed layout; the Python mirror's
host-side pieces (config, width adaptation, parameter packing) behave like the
reference's."""

from __future__ import annotations

import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest
import torch

from deephall_amd import _lib
from deephall_amd.config import Config, System
from deephall_amd.mcmc import update_mcmc_width
from deephall_amd.networks.psiformer import NetworkSpec, flat_params, init_params, param_shapes, ref_offsets
from oracle import reference as R

ROOT = Path(__file__).resolve().parents[1]


def header_symbols():
    txt = (ROOT / "include" / "deephall_amd.h").read_text()
    return sorted(set(re.findall(r"^(?:int|void|size_t|const char\*)\s+(dh_\w+)\(", txt, re.M)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) <= set(_lib.EXPORTS)
    assert b"gfx950" in lib.dh_version()


def make_handle(**kw):
    spec = NetworkSpec(**{**dict(nspins=(6, 0), flux=15, ndets=1, num_heads=4, heads_dim=64, num_layers=2), **kw})
    lib = _lib.load()
    h = C.c_void_p()
    rc = lib.dh_create(C.byref(spec.to_c()), C.byref(h))
    return lib, spec, h, rc


def test_create_layout_workspace():
    lib, spec, h, rc = make_handle()
    assert rc == 0
    nseg = lib.dh_param_layout(h, None, 0)
    assert nseg == 5 + 8 * spec.num_layers
    offs = (C.c_size_t * (nseg + 1))()
    lib.dh_param_layout(h, offs, nseg + 1)
    offs = list(offs)
    assert all(o % 64 == 0 for o in offs) and offs == sorted(offs)
    # layout covers the reference's parameter count (841,410 at C2)
    n_ref = sum(int(np.prod(s)) for s in param_shapes(spec).values())
    assert n_ref == 841410
    assert offs[-1] >= n_ref - 2 * 256 * 256  # Wo/Wl folded into one matrix
    ws_el = lib.dh_workspace_bytes(h, 4096, 1)
    ws_lp = lib.dh_workspace_bytes(h, 4096, 0)
    assert ws_el > 10 * ws_lp > 0
    lib.dh_destroy(h)


@pytest.mark.parametrize(
    "bad",
    [dict(nspins=(0, 0)), dict(nspins=(40, 0)), dict(ndets=0), dict(ndets=17), dict(orbital_type="bogus"),
     dict(num_heads=1, heads_dim=3)],
)
def test_create_rejects_bad_configs(bad):
    lib, spec, h, rc = make_handle(**bad)
    assert rc == -1
    assert len(lib.dh_last_error()) > 0


def test_calls_without_params_fail_cleanly():
    lib, spec, h, rc = make_handle()
    out = (C.c_float * 8)()
    rc = lib.dh_logpsi(h, C.cast(out, C.c_void_p), 1, C.cast(out, C.c_void_p), None, 0, None)
    assert rc == -4  # DH_ESTATE: parameters not set
    lib.dh_destroy(h)


@pytest.mark.parametrize("kw", [dict(), dict(nspins=(2, 1), flux=3, num_heads=2, heads_dim=8, ndets=2),
                                dict(nspins=(20, 0), flux=57), dict(orbital_type="sparse"),
                                dict(nspins=(2, 2), flux=5, orbital_type="sparse")])
def test_ref_layout_matches_reference_tree(kw):
    """dh_ref_layout (the flat reference tree the library packs on the device and the
    gradient layout) == the Python ParamTree layout, in SURVEY.md Appendix B order."""
    lib, spec, h, rc = make_handle(**kw)
    assert rc == 0
    nseg = lib.dh_ref_layout(h, None, 0)
    nblk = 2 if spec.nspins[0] > 0 and spec.nspins[1] > 0 else 1
    lll = 2 if spec.orbital_type == "sparse" else 0
    assert nseg == 1 + 15 * spec.num_layers + 4 * nblk + lll + 2 == len(param_shapes(spec))
    offs = (C.c_size_t * (nseg + 1))()
    lib.dh_ref_layout(h, offs, nseg + 1)
    assert list(offs) == ref_offsets(spec)
    for (name, shape), a, b in zip(param_shapes(spec).items(), list(offs), list(offs)[1:]):
        assert a % 64 == 0 and b - a >= int(np.prod(shape)), name
    t = init_params(spec, seed=3)  # a ParamTree: views into one flat buffer
    assert t.is_packed_view(spec) and t.flat.numel() == offs[nseg]
    assert torch.equal(flat_params(spec, {k: v.clone() for k, v in t.items()}, "cpu"), t.flat)
    lib.dh_destroy(h)


@pytest.mark.parametrize("orbital", ["full", "sparse"])
@pytest.mark.parametrize("nspins", [(3, 0), (2, 2)])
def test_param_tree_matches_oracle_names(orbital, nspins):
    spec = NetworkSpec(nspins=nspins, flux=2, ndets=1, num_heads=4, heads_dim=64, num_layers=2, orbital_type=orbital)
    ocfg = R.OracleConfig(nspins=nspins, flux=2, orbital=orbital)
    assert list(param_shapes(spec)) == list(R.param_shapes(ocfg))  # same names, same order
    for k, v in R.param_shapes(ocfg).items():
        assert tuple(param_shapes(spec)[k]) == tuple(v)


def test_update_mcmc_width_matches_reference():
    pm1, pm2 = np.zeros(4), np.zeros(4)
    w1 = w2 = 0.1
    seq = [0.9, 0.8, 0.7, 0.9, 0.2, 0.1, 0.3, 0.2, 0.52, 0.53, 0.51, 0.5]
    for t, p in enumerate(seq):
        w1, pm1 = update_mcmc_width(t, w1, 4, torch.tensor(p), pm1)
        w2, pm2 = R.update_mcmc_width(t, w2, 4, p, pm2)
        assert w1 == pytest.approx(w2)


def test_config_from_dict():
    cfg = Config.from_dict({"batch_size": 64, "system": {"flux": 15, "nspins": (6, 0)}, "extra": 1})
    assert cfg.batch_size == 64 and cfg.system.flux == 15 and cfg.system.nspins == (6, 0)
    assert isinstance(cfg.system, System) and cfg.mcmc.steps == 10 and cfg.mcmc.width == 0.1


def test_callable_boundary_routing_and_no_cpu_path():
    """Arbitrary callables (hamiltonian.py:83, mcmc.py:105) route to generic.py; native
    networks keep the native path; CPU tensors are refused (no CPU fallback)."""
    from deephall_amd import generic, hamiltonian, mcmc
    from deephall_amd.networks.psiformer import Psiformer

    def f(params, x):
        return torch.zeros((), dtype=torch.complex64)

    step = mcmc.make_mcmc_step(lambda p, d: d.sum((1, 2)), batch_per_device=4, steps=2)
    assert step.__module__ == generic.__name__
    with pytest.raises(RuntimeError, match="GPU only"):
        step(None, torch.zeros(4, 3, 2), None, 0.1)
    ke = hamiltonian.make_local_kinetic_energy(f, 1.0, 1.0)
    with pytest.raises(RuntimeError, match="GPU only"):
        ke(None, torch.zeros(2, 3, 2))
    with pytest.raises(TypeError):
        mcmc.make_mcmc_step(42, batch_per_device=4)
    net = Psiformer((3, 0), 1.0, 1, 1, 4, 1)
    assert mcmc.native_network(net.apply) is net
    assert mcmc.native_network(f) is None
    # the Hessian layout the C ABI expects: [B][N][2][N][2] complex, double
    g, H = generic.derivatives(lambda p, x: (x[:, 0] * x[:, 1]).sum().to(torch.complex128), None,
                               torch.rand(2, 3, 2, dtype=torch.float64))
    assert g.shape == (2, 3, 2) and H.shape == (2, 3, 2, 3, 2)
    assert torch.allclose(H[:, 1, 0, 1, 1].real, torch.ones(2, dtype=torch.float64))


def test_param_tree_view_check_tracks_mutations():
    """ParamTree.is_packed_view caches its leaf walk per tree mutation (the check sits between
    a step's host sync and its first launch): replacing a leaf through any dict mutator makes
    the tree a non-packed view again; in-place leaf updates keep it packed."""
    spec = NetworkSpec(nspins=(3, 0), flux=2, ndets=1, num_heads=4, heads_dim=64, num_layers=2)
    t = init_params(spec, 0, "cpu")
    assert t.is_packed_view(spec) and t.is_packed_view(spec)
    name = next(iter(t))
    t[name].add_(1.0)  # in place: still a view into flat
    assert t.is_packed_view(spec)
    t[name] = t[name].clone()
    assert not t.is_packed_view(spec)
    t2 = init_params(spec, 0, "cpu")
    t2.update({name: t2[name].clone()})
    assert not t2.is_packed_view(spec)
    t3 = init_params(spec, 0, "cpu")
    assert t3.is_packed_view(spec)
    t3.pop(name)
    assert not t3.is_packed_view(spec)


def test_dh_config_rejects_foreign_layouts():
    """dh_create checks dh_config.struct_size: the 11-field binding the
    round-2 INTEGRATION.md showed, and the 14-field layout without struct_size, both fail
    with DH_EINVAL before any field past the caller's struct is read."""
    lib = _lib.load()
    DH_EINVAL = -1
    assert C.sizeof(_lib.DhConfig) == 60

    class Old11(C.Structure):
        _fields_ = [(n, C.c_int) for n in ("n_up", "n_dn", "flux")] + [
            ("radius", C.c_float), ("interaction_strength", C.c_float)] + [
            (n, C.c_int) for n in ("interaction_type", "num_heads", "heads_dim", "num_layers", "ndets", "orbital_type")]

    class Old14(C.Structure):
        _fields_ = Old11._fields_ + [("network_type", C.c_int), ("excitation_lz", C.c_float), ("cf_flux", C.c_int)]

    for cls in (Old11, Old14):
        old = cls(n_up=6, n_dn=0, flux=15, num_heads=4, heads_dim=64, num_layers=2, ndets=1)
        h = C.c_void_p()
        assert lib.dh_create(C.cast(C.pointer(old), C.POINTER(_lib.DhConfig)), C.byref(h)) == DH_EINVAL
        assert b"struct_size" in lib.dh_last_error()
    cfg = NetworkSpec(nspins=(6, 0), flux=15, ndets=1, num_heads=4, heads_dim=64, num_layers=2).to_c()
    cfg.struct_size = 56
    h = C.c_void_p()
    assert lib.dh_create(C.byref(cfg), C.byref(h)) == DH_EINVAL
    cfg.struct_size = C.sizeof(_lib.DhConfig)
    assert lib.dh_create(C.byref(cfg), C.byref(h)) == 0
    lib.dh_destroy(h)


def test_restore_keeps_params_when_optimizer_changed(tmp_path):
    """An Adam checkpoint (opt_state/mu, nu, count) restored into a run whose optimizer state
    has other keys (KFAC: raw, weight, step): params, walkers and step come back, the optimizer
    state is re-initialised with a warning instead of the whole checkpoint being skipped
    (log.py restore_checkpoint) — only when the saved key set differs from the
    current optimizer's; a same-optimizer state of the wrong size raises."""
    from deephall_amd import config
    from deephall_amd.log import LogManager
    from deephall_amd.networks import make_network

    model = make_network(config.System(nspins=(3, 0), flux=2), config.Network())
    p = model.init(3, device="cpu")
    arrays = {"step": np.asarray(4), "mcmc_width": np.asarray(0.25), "data": np.zeros((6, 3, 2), np.float32)}
    for k, v in p.items():
        arrays[f"params/{k}"] = v.numpy()
    n = p.flat.numel()
    arrays.update({"opt_state/mu": np.zeros(n, np.float32), "opt_state/nu": np.zeros(n, np.float32),
                   "opt_state/count": np.asarray(5)})
    path = tmp_path / "ckpt_000004.npz"
    np.savez_compressed(path, **arrays)

    class KfacLike:
        inits = 0

        def __init__(self):
            KfacLike.inits += 1
            self.raw = torch.zeros(3)

        def state_dict(self):
            return {"raw": self.raw, "weight": 0.0, "step": 0}

        def load_state_dict(self, d):
            self.raw.copy_(torch.as_tensor(d["raw"]))

    step, st = LogManager.restore_checkpoint(path, model, torch.device("cpu"), lambda params: KfacLike())
    assert step == 5 and st.mcmc_width == 0.25 and st.data.shape == (6, 3, 2)
    for k in p:
        assert torch.equal(st.params[k], p[k])
    assert isinstance(st.opt_state, KfacLike) and KfacLike.inits == 1  # the fresh state, never loaded
    # the SAME optimizer's state with a wrong size is an error, not a silent reset
    bad = dict(arrays)
    for k in ("opt_state/mu", "opt_state/nu", "opt_state/count"):
        bad.pop(k)
    bad.update({"opt_state/raw": np.zeros(5, np.float32), "opt_state/weight": np.asarray(1.0),
                "opt_state/step": np.asarray(1)})
    path2 = tmp_path / "ckpt_000005.npz"
    np.savez_compressed(path2, **bad)
    with pytest.raises(RuntimeError):
        LogManager.restore_checkpoint(path2, model, torch.device("cpu"), lambda params: KfacLike())
