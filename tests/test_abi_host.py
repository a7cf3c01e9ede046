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
from deephall_amd.networks.psiformer import NetworkSpec, init_params, pack_params, param_shapes
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
    [dict(nspins=(0, 0)), dict(nspins=(40, 0)), dict(ndets=0), dict(ndets=17), dict(orbital_type="sparse"),
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


def test_pack_params_layout_matches_reference_tree():
    lib, spec, h, rc = make_handle(nspins=(2, 1), flux=3, num_heads=2, heads_dim=8, ndets=2)
    nseg = lib.dh_param_layout(h, None, 0)
    offs = (C.c_size_t * (nseg + 1))()
    lib.dh_param_layout(h, offs, nseg + 1)
    offs = list(offs)
    p = init_params(spec, seed=3)
    buf = pack_params(spec, p, offs, "cpu").double()
    D = spec.D
    seg = lambda s, n: buf[offs[s] : offs[s] + n]  # noqa: E731
    assert torch.allclose(seg(0, 4 * D), p["PsiformerLayers_0/Dense_0/kernel"].double().reshape(-1))
    mha = "PsiformerLayers_0/MultiHeadAttention_0/"
    wq = seg(1, D * 3 * D).reshape(D, 3 * D)
    assert torch.allclose(wq[:, D : 2 * D], p[mha + "key/kernel"].double().reshape(D, D))
    wol = seg(3, D * D).reshape(D, D)
    ref = p[mha + "out/kernel"].double().reshape(D, D) @ p["PsiformerLayers_0/Dense_1/kernel"].double()
    assert torch.allclose(wol, ref, atol=1e-6)
    # orbital block order: (blk, part) = DenseGeneral_{2 blk + part}
    L = spec.num_layers
    MNK = spec.M * spec.nelec * spec.ndets
    worb = buf[offs[1 + 8 * L] : offs[2 + 8 * L]][: D * ((4 * MNK + 127) // 128 * 128)].reshape(D, -1)
    ob = "Orbitals_0/featured_orbitals/"
    assert torch.allclose(worb[:, 3 * MNK : 4 * MNK], p[ob + "DenseGeneral_3/kernel"].double().reshape(D, MNK))
    jas = buf[offs[3 + 8 * L] : offs[3 + 8 * L] + 2]
    assert jas.tolist() == [1.0, 1.0]
    w0qkv = buf[offs[4 + 8 * L] : offs[4 + 8 * L] + 4 * 3 * D].reshape(4, 3 * D)
    wq0 = torch.cat([p[mha + n + "/kernel"].double().reshape(D, D) for n in ("query", "key", "value")], 1)
    assert torch.allclose(w0qkv, p["PsiformerLayers_0/Dense_0/kernel"].double() @ wq0, atol=1e-6)
    lib.dh_destroy(h)


def test_param_tree_matches_oracle_names():
    spec = NetworkSpec(nspins=(3, 0), flux=2, ndets=1, num_heads=4, heads_dim=64, num_layers=2)
    ocfg = R.OracleConfig(nspins=(3, 0), flux=2)
    assert set(param_shapes(spec)) == set(R.param_shapes(ocfg))
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
