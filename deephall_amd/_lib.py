"""ctypes binding of the C ABI declared in include/deephall_amd.h.

The HIP library is the only compute path: if it is missing this module raises —
there is no CPU / PyTorch fallback.
"""

from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "_lib" / "libdeephall_amd.so"

DH_NSTATS = 16
STAT_NAMES = [
    "energy_re",
    "energy_im",
    "clipped_re",
    "clipped_im",
    "ere2",
    "kinetic_re",
    "kinetic_im",
    "potential",
    "angular_momentum_z",
    "angular_momentum_z_square",
    "angular_momentum_square",
    "pmove",
    "nvalid",
    "clipped_lz2",
    "clipped_lz",
    "clipped_l2",
]

EXPORTS = [
    "dh_create",
    "dh_destroy",
    "dh_last_error",
    "dh_version",
    "dh_param_layout",
    "dh_set_params",
    "dh_workspace_bytes",
    "dh_set_gemm_mode",
    "dh_logpsi",
    "dh_mcmc_step",
    "dh_local_energy",
    "dh_energy_stats",
    "dh_loss_diff",
    "dh_init_walkers",
    "dh_potential",
    "dh_histograms",
    "dh_monopole_orbitals",
    "dh_mh_init",
    "dh_mh_propose",
    "dh_mh_accept",
    "dh_kinetic_from_derivatives",
    "dh_debug_trunk",
    "dh_debug_gemm",
    "dh_debug_gemm_ln",
    "dh_debug_gemm_x6_ln",
    "dh_debug_chain_x6",
    "dh_debug_gemm_lnch",
    "dh_debug_set_lnch_form",
    "dh_debug_x6_plane_rows",
    "dh_debug_split_planes",
    "dh_debug_gemm_x6",
    "dh_ref_layout",
    "dh_set_params_ref",
    "dh_vjp_workspace_bytes",
    "dh_logpsi_vjp",
    "dh_grad_cotangent",
    "dh_adam_update",
    "dh_profile_enable",
    "dh_profile_read",
    "dh_debug_f_offset",
    "dh_debug_env_leaf",
    "dh_kfac_layout",
    "dh_kfac_workspace_bytes",
    "dh_kfac_vjp",
    "dh_kfac_step",
]


PROF_KINDS = ["gemm", "attention", "layernorm", "input", "det_value", "det_energy", "mcmc",
              "gemm_ch", "attention_ch", "layernorm_ch", "input_ch", "layer1_ch"]


class DhConfig(C.Structure):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("n_up", C.c_int),
        ("n_dn", C.c_int),
        ("flux", C.c_int),
        ("radius", C.c_float),
        ("interaction_strength", C.c_float),
        ("interaction_type", C.c_int),
        ("num_heads", C.c_int),
        ("heads_dim", C.c_int),
        ("num_layers", C.c_int),
        ("ndets", C.c_int),
        ("orbital_type", C.c_int),
        ("network_type", C.c_int),
        ("excitation_lz", C.c_float),
        ("cf_flux", C.c_int),
    ]

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        self.struct_size = C.sizeof(DhConfig)


_lib = None


def load(path: Path | str | None = None):
    """Load (once) and return the HIP library; raise if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    # DH_LIB_PATH: an alternative build of the same library (A/B timing tools only)
    p = Path(path) if path else Path(os.environ.get("DH_LIB_PATH") or LIB_PATH)
    if not p.exists():
        raise RuntimeError(
            f"deephall_amd HIP library not found at {p}. Build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)."
        )
    lib = C.CDLL(str(p))
    vp, sz, i32, u64, i64 = C.c_void_p, C.c_size_t, C.c_int, C.c_uint64, C.c_int64
    lib.dh_create.argtypes = [C.POINTER(DhConfig), C.POINTER(vp)]
    lib.dh_create.restype = i32
    lib.dh_destroy.argtypes = [vp]
    lib.dh_destroy.restype = None
    lib.dh_last_error.restype = C.c_char_p
    lib.dh_version.restype = C.c_char_p
    lib.dh_param_layout.argtypes = [vp, C.POINTER(sz), i32]
    lib.dh_param_layout.restype = i32
    lib.dh_set_params.argtypes = [vp, vp, sz, vp]
    lib.dh_set_params.restype = i32
    lib.dh_workspace_bytes.argtypes = [vp, i32, i32]
    lib.dh_workspace_bytes.restype = sz
    lib.dh_set_gemm_mode.argtypes = [vp, i32]
    lib.dh_set_gemm_mode.restype = i32
    lib.dh_logpsi.argtypes = [vp, vp, i32, vp, vp, sz, vp]
    lib.dh_logpsi.restype = i32
    lib.dh_mcmc_step.argtypes = [vp, vp, vp, vp, i32, i32, C.c_float, u64, u64, i64, vp, vp, sz, vp]
    lib.dh_mcmc_step.restype = i32
    lib.dh_local_energy.argtypes = [vp, vp, i32, vp, vp, vp, sz, vp]
    lib.dh_local_energy.restype = i32
    lib.dh_energy_stats.argtypes = [vp, vp, vp, vp, i32, i32, i32, vp, vp]
    lib.dh_energy_stats.restype = i32
    f32 = C.c_float
    lib.dh_loss_diff.argtypes = [vp, vp, vp, i32, vp, f32, f32, f32, vp, vp, vp]
    lib.dh_loss_diff.restype = i32
    lib.dh_init_walkers.argtypes = [vp, vp, i32, u64, i64, vp]
    lib.dh_init_walkers.restype = i32
    lib.dh_potential.argtypes = [vp, vp, i32, vp, vp]
    lib.dh_potential.restype = i32
    lib.dh_histograms.argtypes = [vp, i32, i32, i32, i32, vp, vp, vp]
    lib.dh_histograms.restype = i32
    lib.dh_monopole_orbitals.argtypes = [vp, i32, i32, vp, vp]
    lib.dh_monopole_orbitals.restype = i32
    lib.dh_debug_trunk.argtypes = [vp, vp, i32, i32, vp, sz, vp]
    lib.dh_debug_trunk.restype = i32
    lib.dh_debug_f_offset.argtypes = [vp, i32, i32]
    lib.dh_debug_f_offset.restype = sz
    lib.dh_debug_env_leaf.argtypes = [vp, i32, i32, i32, vp, vp]
    lib.dh_debug_env_leaf.restype = i32
    lib.dh_debug_gemm.argtypes = [i32, vp, i32, vp, i32, vp, vp, i32, vp, i32, i32, i32, i32, i32, vp]
    lib.dh_debug_gemm.restype = i32
    lib.dh_debug_gemm_ln.argtypes = [i32, i32, vp, i32, vp, i32, vp, vp, vp, i32, i32, vp]
    lib.dh_debug_gemm_ln.restype = i32
    lib.dh_debug_gemm_x6_ln.argtypes = [i32, i32, vp, i32, vp, i32, vp, vp, vp, i32, i32, vp]
    lib.dh_debug_gemm_x6_ln.restype = i32
    lib.dh_debug_chain_x6.argtypes = [vp, vp, i32, vp, vp, vp, i32, vp, vp, vp, i32, vp, i32, vp, i32, vp, i32, vp]
    lib.dh_debug_chain_x6.restype = i32
    lib.dh_debug_gemm_lnch.argtypes = [i32, i32, vp, vp, i32, vp, vp, vp, vp, i32, vp]
    lib.dh_debug_gemm_lnch.restype = i32
    lib.dh_debug_set_lnch_form.argtypes = [i32]
    lib.dh_debug_set_lnch_form.restype = i32
    lib.dh_debug_x6_plane_rows.argtypes = [i32]
    lib.dh_debug_x6_plane_rows.restype = i32
    lib.dh_debug_split_planes.argtypes = [vp, i32, i32, i32, vp, vp]
    lib.dh_debug_split_planes.restype = i32
    lib.dh_debug_gemm_x6.argtypes = [i32, vp, i32, vp, i32, vp, vp, i32, vp, i32, i32, i32, i32, i32, vp]
    lib.dh_debug_gemm_x6.restype = i32
    lib.dh_ref_layout.argtypes = [vp, C.POINTER(sz), i32]
    lib.dh_ref_layout.restype = i32
    lib.dh_set_params_ref.argtypes = [vp, vp, sz, vp]
    lib.dh_set_params_ref.restype = i32
    lib.dh_vjp_workspace_bytes.argtypes = [vp, i32]
    lib.dh_vjp_workspace_bytes.restype = sz
    lib.dh_logpsi_vjp.argtypes = [vp, vp, i32, vp, vp, vp, vp, sz, vp]
    lib.dh_logpsi_vjp.restype = i32
    lib.dh_kfac_layout.argtypes = [vp, C.POINTER(sz), i32]
    lib.dh_kfac_layout.restype = i32
    lib.dh_kfac_workspace_bytes.argtypes = [vp, i32]
    lib.dh_kfac_workspace_bytes.restype = sz
    lib.dh_kfac_vjp.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, sz, vp]
    lib.dh_kfac_vjp.restype = i32
    lib.dh_kfac_step.argtypes = [vp, vp, vp, f32, f32, vp, vp, f32, f32, f32, vp, vp, vp, sz, vp]
    lib.dh_kfac_step.restype = i32
    lib.dh_grad_cotangent.argtypes = [vp, vp, i32, i32, vp, vp]
    lib.dh_grad_cotangent.restype = i32
    lib.dh_adam_update.argtypes = [vp, vp, vp, vp, sz, f32, f32, f32, f32, i32, vp]
    lib.dh_adam_update.restype = i32
    lib.dh_mh_init.argtypes = [vp, vp, vp, i32, vp]
    lib.dh_mh_init.restype = i32
    lib.dh_mh_propose.argtypes = [vp, vp, i32, i32, f32, u64, u64, i64, vp, vp]
    lib.dh_mh_propose.restype = i32
    lib.dh_mh_accept.argtypes = [vp, vp, vp, vp, vp, i32, i32, u64, u64, i64, vp, vp]
    lib.dh_mh_accept.restype = i32
    lib.dh_kinetic_from_derivatives.argtypes = [vp, vp, vp, i32, i32, C.c_double, C.c_double, vp, vp, vp]
    lib.dh_kinetic_from_derivatives.restype = i32
    lib.dh_profile_enable.argtypes = [vp, i32]
    lib.dh_profile_enable.restype = i32
    lib.dh_profile_read.argtypes = [vp, C.POINTER(C.c_double), i32]
    lib.dh_profile_read.restype = i32
    _lib = lib
    return lib


def check(rc: int):
    if rc != 0:
        msg = load().dh_last_error().decode(errors="replace")
        raise RuntimeError(f"deephall_amd error {rc}: {msg}")
