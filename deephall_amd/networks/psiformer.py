"""Psiformer wavefunction on MI355X — mirror of deephall/networks/psiformer.py + blocks.py.

``Psiformer`` keeps the reference module's constructor fields
(psiformer.py:63-70: nspins, Q, ndets, num_heads, heads_dim, num_layers,
orbital_type) and its two entry points:

* ``init(key, data)`` -> parameter dict with the Flax auto-generated names
  (SURVEY.md Appendix B), lecun-normal kernels, zero biases, LayerNorm scale 1,
  Jastrow alphas 1 (the Flax defaults the reference relies on);
* ``apply(params, data[B, N, 2])`` -> complex64 log psi [B].  The reference's
  ``model.apply`` is per walker and vmapped by its callers (train.py:69); the
  native kernels are batched, so the batch axis is explicit here.

All arithmetic runs in the HIP library (include/deephall_amd.h); this module only
flattens the parameter tree into the ``dh_ref_layout`` buffer (the library packs
it on the device) and manages the per-device handle and workspace.
"""

from __future__ import annotations

import ctypes as C
import functools
import os
import math
from dataclasses import dataclass

import numpy as np
import torch

from .. import _lib

_HANDLES: dict = {}
VJP_WORKSPACE_BYTES = 16 << 30  # walkers beyond this go through in chunks


def _ptr(t: torch.Tensor | None):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def _stream(device: torch.device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


@dataclass(frozen=True)
class NetworkSpec:
    """Everything the native handle needs (dh_config)."""

    nspins: tuple
    flux: int
    ndets: int
    num_heads: int
    heads_dim: int
    num_layers: int
    orbital_type: str = "full"
    radius: float | None = None
    interaction_strength: float = 1.0
    interaction_type: str = "coulomb"
    network_type: str = "psiformer"
    excitation_lz: float = 0.0
    cf_flux: int = 1

    @property
    def nelec(self) -> int:
        return int(sum(self.nspins))

    @property
    def D(self) -> int:
        return self.num_heads * self.heads_dim

    @property
    def M(self) -> int:
        return int(self.flux) + 1

    def to_c(self) -> _lib.DhConfig:
        c = _lib.DhConfig()
        c.n_up, c.n_dn = int(self.nspins[0]), int(self.nspins[1])
        c.flux = int(self.flux)
        c.radius = float(self.radius) if self.radius else 0.0
        c.interaction_strength = float(self.interaction_strength)
        c.interaction_type = 0 if str(getattr(self.interaction_type, "value", self.interaction_type)) == "coulomb" else 1
        c.num_heads, c.heads_dim, c.num_layers = self.num_heads, self.heads_dim, self.num_layers
        c.ndets = self.ndets
        c.orbital_type = {"full": 0, "sparse": 1}.get(str(getattr(self.orbital_type, "value", self.orbital_type)), -1)
        c.network_type = {"psiformer": 0, "laughlin": 1}.get(str(getattr(self.network_type, "value", self.network_type)), -1)
        c.excitation_lz = float(self.excitation_lz)
        c.cf_flux = int(self.cf_flux)
        return c


class NativeHandle:
    """One dh_handle per (spec, device); owns the workspace tensor."""

    def __init__(self, spec: NetworkSpec, device: torch.device):
        self.lib = _lib.load()
        self.spec = spec
        self.device = device
        self.h = C.c_void_p()
        cfg = spec.to_c()
        _lib.check(self.lib.dh_create(C.byref(cfg), C.byref(self.h)))
        nseg = self.lib.dh_ref_layout(self.h, None, 0)
        offs = (C.c_size_t * (nseg + 1))()
        self.lib.dh_ref_layout(self.h, offs, nseg + 1)
        self.ref_offsets = [int(o) for o in offs]
        if self.ref_offsets != ref_offsets(spec):
            raise RuntimeError("dh_ref_layout disagrees with the Python parameter tree")
        self.nref = self.ref_offsets[-1]
        self.ws = {}  # one workspace per HIP stream (walker groups may run on parallel streams)
        self._params_key = None
        self.set_gemm_mode(_GEMM_MODE)

    def set_gemm_mode(self, mode: str):
        """GEMM arithmetic: "x6all" (split-bf16, f32-accurate, every GEMM; default), "x6"
        (split-bf16 for the local-energy channel rows only), "f32" (exact-f32 MFMA) or
        "x6all_unfused" (as x6all with the channel LayerNorms as separate passes; test hook)."""
        _lib.check(self.lib.dh_set_gemm_mode(self.h, _GEMM_MODES[mode]))

    def __del__(self):
        try:
            if self.h:
                self.lib.dh_destroy(self.h)
        except Exception:  # noqa: BLE001
            pass

    def workspace(self, nbytes: int) -> torch.Tensor:
        sid = torch.cuda.current_stream(self.device).cuda_stream
        ws = self.ws.get(sid)
        if ws is None or ws.numel() < nbytes:
            self.ws.pop(sid, None)
            ws = None
            torch.cuda.empty_cache()
            ws = torch.empty(int(nbytes), dtype=torch.uint8, device=self.device)
            self.ws[sid] = ws
        return ws

    def set_params_ref(self, flat: torch.Tensor, key):
        """Upload the flat reference tree; the library packs it on the device (folds,
        transposes, split-bf16 planes: dh_set_params_ref)."""
        if self._params_key == key:
            return
        assert flat.numel() == self.nref and flat.dtype == torch.float32 and flat.is_cuda
        _lib.check(self.lib.dh_set_params_ref(self.h, _ptr(flat), self.nref, _stream(self.device)))
        self._flat = flat  # keep alive while the copy is in flight
        self._params_key = key


_GEMM_MODES = {"f32": 0, "x6": 1, "x6all": 2, "x6all_unfused": 3}
_GEMM_MODE = os.environ.get("DH_GEMM", "x6all")
if _GEMM_MODE not in _GEMM_MODES:
    raise ValueError(f"DH_GEMM must be one of {sorted(_GEMM_MODES)}, got {_GEMM_MODE!r}")


def set_gemm_mode(mode: str):
    """Select the local-energy GEMM arithmetic for every handle (existing and future)."""
    global _GEMM_MODE
    if mode not in _GEMM_MODES:
        raise ValueError(f"GEMM mode must be one of {sorted(_GEMM_MODES)}")
    _GEMM_MODE = mode
    for h in _HANDLES.values():
        h.set_gemm_mode(mode)


def get_handle(spec: NetworkSpec, device) -> NativeHandle:
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError("deephall_amd runs on the GPU only (no CPU fallback): pass CUDA/HIP tensors")
    key = (spec, device.index if device.index is not None else torch.cuda.current_device())
    if key not in _HANDLES:
        _HANDLES[key] = NativeHandle(spec, torch.device("cuda", key[1]))
    return _HANDLES[key]


def flatten_params(params) -> dict:
    """Accept a flat {'A/B/kernel': t} dict or a nested Flax-like dict (optionally under 'params')."""
    if "params" in params and isinstance(params["params"], dict):
        params = params["params"]
    flat = {}

    def rec(prefix, d):
        for k, v in d.items():
            name = f"{prefix}/{k}" if prefix else k
            if isinstance(v, dict):
                rec(name, v)
            else:
                flat[name] = v
    rec("", params)
    return flat


def param_shapes(spec: NetworkSpec) -> dict:
    """Shapes of the reference's parameter tree (Flax auto-naming)."""
    if spec.network_type == "laughlin":
        return {}  # laughlin.py has no parameters
    D, H, dh = spec.D, spec.num_heads, spec.heads_dim
    M, N, K = spec.M, spec.nelec, spec.ndets
    p = "PsiformerLayers_0/"
    s = {p + "Dense_0/kernel": (4, D)}
    for l in range(spec.num_layers):
        mha = p + f"MultiHeadAttention_{l}/"
        for nm in ("query", "key", "value"):
            s[mha + nm + "/kernel"] = (D, H, dh)
            s[mha + nm + "/bias"] = (H, dh)
        s[mha + "out/kernel"] = (H, dh, D)
        s[mha + "out/bias"] = (D,)
        s[p + f"Dense_{2 * l + 1}/kernel"] = (D, D)
        s[p + f"LayerNorm_{2 * l}/scale"] = (D,)
        s[p + f"LayerNorm_{2 * l}/bias"] = (D,)
        s[p + f"Dense_{2 * l + 2}/kernel"] = (D, D)
        s[p + f"Dense_{2 * l + 2}/bias"] = (D,)
        s[p + f"LayerNorm_{2 * l + 1}/scale"] = (D,)
        s[p + f"LayerNorm_{2 * l + 1}/bias"] = (D,)
    ob = "Orbitals_0/featured_orbitals/"
    nblk = sum(1 for n in spec.nspins if n > 0)
    sparse = str(getattr(spec.orbital_type, "value", spec.orbital_type)) == "sparse"
    F = 8 if sparse else M  # blocks.py:48-57
    for i in range(2 * nblk):
        s[ob + f"DenseGeneral_{i}/kernel"] = (D, F, N, K)
        s[ob + f"DenseGeneral_{i}/bias"] = (F, N, K)
    if sparse:  # lll_weight = DenseGeneral(2Q+1, axis=1), blocks.py:57
        s["Orbitals_0/lll_weight/kernel"] = (8, M)
        s["Orbitals_0/lll_weight/bias"] = (M,)
    s["Jastrow_0/ee_par"] = (1,)
    s["Jastrow_0/ee_anti"] = (1,)
    return s


def ref_offsets(spec: NetworkSpec) -> list:
    """Float offsets of the flat reference tree (dh_ref_layout): param_shapes order,
    64-float aligned segments; the last entry is the total."""
    offs, o = [], 0
    for shape in param_shapes(spec).values():
        offs.append(o)
        o += (int(np.prod(shape)) + 63) // 64 * 64
    offs.append(o)
    return offs


@functools.lru_cache(maxsize=None)
def _leaf_offsets(spec: NetworkSpec) -> tuple:
    """((name, byte offset into the flat tree), ...) in dh_ref_layout order."""
    return tuple((name, 4 * o) for name, o in zip(param_shapes(spec), ref_offsets(spec)))


class ParamTree(dict):
    """{Flax path: tensor} whose tensors are views into ONE flat float32 buffer in the
    dh_ref_layout order (``.flat``).  Optimizers update ``.flat`` in place; the kernels
    upload it as is.  Replacing a leaf goes through item assignment (``tree[name] = t``),
    which the tree counts, so the view check runs once per mutation, not once per call
    (it sits between a step's host sync and its first launch)."""

    flat: torch.Tensor
    _mut = 0
    _checked = None

    def _touch(self):
        self._mut += 1
        self._checked = None

    def __setitem__(self, k, v):
        super().__setitem__(k, v)
        self._touch()

    def __delitem__(self, k):
        super().__delitem__(k)
        self._touch()

    def update(self, *a, **kw):
        super().update(*a, **kw)
        self._touch()

    def pop(self, *a):
        self._touch()
        return super().pop(*a)

    def popitem(self):
        self._touch()
        return super().popitem()

    def setdefault(self, *a):
        self._touch()
        return super().setdefault(*a)

    def clear(self):
        super().clear()
        self._touch()

    @classmethod
    def zeros(cls, spec: NetworkSpec, device) -> "ParamTree":
        offs = ref_offsets(spec)
        return cls.view_of(spec, torch.zeros(offs[-1], dtype=torch.float32, device=device))

    @classmethod
    def view_of(cls, spec: NetworkSpec, flat: torch.Tensor) -> "ParamTree":
        """A tree of views into an existing flat buffer (dh_ref_layout order)."""
        offs = ref_offsets(spec)
        if flat.dim() != 1 or flat.numel() != offs[-1] or flat.dtype != torch.float32:
            raise ValueError(f"flat buffer must be float32 [{offs[-1]}]")
        t = cls()
        for (name, shape), o in zip(param_shapes(spec).items(), offs):
            t[name] = flat[o : o + int(np.prod(shape))].view(shape)
        t.flat = flat
        return t

    def is_packed_view(self, spec: NetworkSpec) -> bool:
        """True while every leaf is still the original view into ``flat``."""
        flat = getattr(self, "flat", None)
        if flat is None:
            return False
        base = flat.data_ptr()
        sig = (spec, base, self._mut)
        if self._checked == sig:
            return True
        for name, off in _leaf_offsets(spec):
            v = self.get(name)
            if v is None or v.data_ptr() != base + off or not v.is_contiguous():
                return False
        self._checked = sig
        return True


def init_params(spec: NetworkSpec, seed: int, device="cpu") -> ParamTree:
    """Flax-default initialisation: lecun_normal (truncated to 2 sigma) kernels
    (fan_in = input features; H*dh for the attention output), zero biases,
    LayerNorm scale 1, Jastrow alphas 1 (blocks.py:92,100)."""
    rng = np.random.default_rng(seed)
    out = ParamTree.zeros(spec, device)
    for name, shape in param_shapes(spec).items():
        if name.endswith("/kernel"):
            fan_in = shape[0] * shape[1] if "out/kernel" in name else shape[0]
            std = math.sqrt(1.0 / fan_in) / 0.87962566103423978
            w = rng.standard_normal(size=shape)
            bad = np.abs(w) > 2
            while bad.any():
                w[bad] = rng.standard_normal(size=int(bad.sum()))
                bad = np.abs(w) > 2
            arr = w * std
        elif name.endswith("/scale") or name.startswith("Jastrow"):
            arr = np.ones(shape)
        else:
            arr = np.zeros(shape)
        out[name].copy_(torch.tensor(arr, dtype=torch.float32))
    return out


def flat_params(spec: NetworkSpec, params, device) -> torch.Tensor:
    """The flat reference-layout buffer of a parameter dict: ``params.flat`` when the dict
    is an intact ParamTree on ``device``, else a float32 copy assembled segment by segment."""
    if isinstance(params, ParamTree) and params.is_packed_view(spec) and params.flat.device == torch.device(device):
        return params.flat
    P = flatten_params(params)
    offs = ref_offsets(spec)
    flat = torch.zeros(offs[-1], dtype=torch.float32, device=device)
    for (name, shape), o in zip(param_shapes(spec).items(), offs):
        n = int(np.prod(shape))
        if name not in P:
            if name.startswith("Jastrow"):  # optional leaves (blocks.py:92,100): alpha = 1
                flat[o] = 1.0
                continue
            raise KeyError(f"parameter {name} missing")
        t = P[name]
        if tuple(t.shape) != tuple(shape):
            raise ValueError(f"parameter {name}: shape {tuple(t.shape)} != {tuple(shape)}")
        flat[o : o + n] = t.detach().reshape(-1).to(device=device, dtype=torch.float32)
    return flat


class Psiformer:
    """Psiformer(nspins, Q, ndets, num_heads, heads_dim, num_layers, orbital_type)
    (psiformer.py:63-91) backed by the HIP kernels."""

    def __init__(self, nspins, Q, ndets, num_heads, heads_dim, num_layers, orbital_type="full", system=None):
        self.nspins = tuple(int(n) for n in nspins)
        self.Q = float(Q)
        self.ndets = int(ndets)
        self.num_heads, self.heads_dim, self.num_layers = int(num_heads), int(heads_dim), int(num_layers)
        self.orbital_type = str(getattr(orbital_type, "value", orbital_type))
        if self.orbital_type not in ("full", "sparse"):
            raise ValueError(f"unknown orbital type {self.orbital_type!r}")
        radius = getattr(system, "radius", None) if system is not None else None
        lam = getattr(system, "interaction_strength", 1.0) if system is not None else 1.0
        itype = getattr(system, "interaction_type", "coulomb") if system is not None else "coulomb"
        self.spec = NetworkSpec(
            nspins=self.nspins,
            flux=int(round(2 * self.Q)),
            ndets=self.ndets,
            num_heads=self.num_heads,
            heads_dim=self.heads_dim,
            num_layers=self.num_layers,
            orbital_type=self.orbital_type,
            radius=radius,
            interaction_strength=float(lam),
            interaction_type=str(getattr(itype, "value", itype)),
        )
        self._flat_cache = {}
        self._epoch = 0

    # ---- reference-compatible entry points
    def init(self, key, data=None, device=None) -> ParamTree:
        seed = int(getattr(key, "seed", key))
        if device is None:
            device = data.device if isinstance(data, torch.Tensor) else ("cuda" if torch.cuda.is_available() else "cpu")
        return init_params(self.spec, seed, device)

    def apply(self, params, data: torch.Tensor) -> torch.Tensor:
        """Batched log psi: data [B, N, 2] float32 (cuda) -> complex64 [B]."""
        h = self.prepare(params, data.device)
        x = self._check_walkers(data)
        B = x.shape[0]
        out = torch.empty(B, 2, dtype=torch.float32, device=x.device)
        nbytes = h.lib.dh_workspace_bytes(h.h, B, 0)
        ws = h.workspace(nbytes)
        _lib.check(h.lib.dh_logpsi(h.h, _ptr(x), B, _ptr(out), _ptr(ws), ws.numel(), _stream(x.device)))
        return torch.complex(out[:, 0], out[:, 1])

    __call__ = apply

    def vjp(self, params, data: torch.Tensor, ct: torch.Tensor, out: "ParamTree | None" = None,
            logpsi: torch.Tensor | None = None) -> "ParamTree":
        """Parameter gradient sum_b ct[b,0] dRe log psi_b/dp + ct[b,1] dIm log psi_b/dp by
        reverse mode in the HIP library (dh_logpsi_vjp), as a ParamTree of float32 views
        (the reference's jax.grad of network(params, x).real / .imag, loss.py:53-58)."""
        h = self.prepare(params, data.device)
        x = self._check_walkers(data)
        B = x.shape[0]
        ct = ct.to(device=x.device, dtype=torch.float32).contiguous()
        if tuple(ct.shape) != (B, 2):
            raise ValueError(f"cotangents must be [{B}, 2]")
        if out is None:
            out = ParamTree.zeros(self.spec, x.device)
        need = h.lib.dh_vjp_workspace_bytes(h.h, B)
        one = h.lib.dh_vjp_workspace_bytes(h.h, 1)
        ws = h.workspace(max(min(need, VJP_WORKSPACE_BYTES), one))
        _lib.check(h.lib.dh_logpsi_vjp(h.h, _ptr(x), B, _ptr(ct), _ptr(out.flat), _ptr(logpsi), _ptr(ws), ws.numel(),
                                       _stream(x.device)))
        return out

    # ---- KFAC (optimizers/kfac.py:195-241; dh_kfac_*)
    def kfac_layout(self, device) -> dict:
        """dh_kfac_layout: statistics size, factor slots and dense blocks."""
        h = get_handle(self.spec, device)
        n = h.lib.dh_kfac_layout(h.h, None, 0)
        if n < 0:
            _lib.check(n)
        buf = (C.c_size_t * n)()
        h.lib.dh_kfac_layout(h.h, buf, n)
        v = [int(t) for t in buf]
        nb, ns = v[3], v[2]
        blocks = [dict(zip(("kernel_seg", "bias_seg", "din", "dout", "a_slot", "g_slot", "scale"), v[6 + 7 * i: 13 + 7 * i]))
                  for i in range(nb)]
        for b in blocks:
            b["scale"] = b["scale"] / 1000.0
            if b["bias_seg"] >= 2**63:
                b["bias_seg"] = None
        o = 6 + 7 * nb
        slots = [(v[o + 2 * i], v[o + 2 * i + 1]) for i in range(ns)]
        return {"nstats": v[0], "nmat": v[1], "ngeneric": v[4], "step_ws": v[5], "blocks": blocks, "slots": slots}

    def kfac_vjp(self, params, data: torch.Tensor, ct: torch.Tensor | None, grad: "ParamTree | None",
                 stats: torch.Tensor, logpsi: torch.Tensor | None = None):
        """dh_kfac_vjp: one forward pass, the gradient for ``ct`` into ``grad`` (as vjp) and the
        Fisher curvature statistics of this batch into ``stats`` (float32 [nstats])."""
        h = self.prepare(params, data.device)
        x = self._check_walkers(data)
        B = x.shape[0]
        if ct is not None:
            ct = ct.to(device=x.device, dtype=torch.float32).contiguous()
            if tuple(ct.shape) != (B, 2):
                raise ValueError(f"cotangents must be [{B}, 2]")
        need = h.lib.dh_kfac_workspace_bytes(h.h, B)
        one = h.lib.dh_kfac_workspace_bytes(h.h, 1)
        ws = h.workspace(max(min(need, VJP_WORKSPACE_BYTES), one))
        _lib.check(h.lib.dh_kfac_vjp(h.h, _ptr(x), B, _ptr(ct), _ptr(grad.flat) if grad is not None else None,
                                     _ptr(stats), _ptr(logpsi), _ptr(ws), ws.numel(), _stream(x.device)))

    def kfac_step(self, raw: torch.Tensor, stats: torch.Tensor | None, ema: float, weight: float, grad: "ParamTree",
                  params: "ParamTree | None", lr: float, damping: float, norm_constraint: float,
                  pgrad: torch.Tensor, info: torch.Tensor):
        """dh_kfac_step: EMA of the statistics, damped inverses, P g and (params given) the
        norm-constrained update in place on ``params.flat``."""
        dev = grad.flat.device
        h = get_handle(self.spec, dev)
        ws = h.kfac_ws if getattr(h, "kfac_ws", None) is not None else None
        need = self.kfac_layout(dev)["step_ws"] if ws is None else ws.numel()
        if ws is None:
            ws = h.kfac_ws = torch.empty(need, dtype=torch.uint8, device=dev)
        _lib.check(h.lib.dh_kfac_step(h.h, _ptr(raw), _ptr(stats), float(ema), float(weight), _ptr(grad.flat),
                                      _ptr(params.flat) if params is not None else None, float(lr), float(damping),
                                      float(norm_constraint), _ptr(pgrad), _ptr(info), _ptr(ws), ws.numel(),
                                      _stream(dev)))

    # ---- plumbing
    def _check_walkers(self, data: torch.Tensor) -> torch.Tensor:
        if data.dim() != 3 or data.shape[1] != self.spec.nelec or data.shape[2] != 2:
            raise ValueError(f"walkers must be [B, {self.spec.nelec}, 2], got {tuple(data.shape)}")
        if not data.is_cuda:
            raise RuntimeError("deephall_amd runs on the GPU only (no CPU fallback)")
        return data.to(torch.float32).contiguous()

    def prepare(self, params, device) -> NativeHandle:
        h = get_handle(self.spec, device)
        if isinstance(params, ParamTree) and params.is_packed_view(self.spec) and params.flat.device == h.device:
            flat = params.flat
            # in-place updates through any view bump the shared version counter; updates
            # written by the optimizer kernels call invalidate()
            key = ("flat", flat.data_ptr(), flat._version, self._epoch)
        else:
            P = flatten_params(params) if isinstance(params, dict) else params
            key = (id(params), tuple((id(v), v.data_ptr(), v._version) for v in P.values()), self._epoch)
            if key not in self._flat_cache:
                self._flat_cache.clear()
                self._flat_cache[key] = flat_params(self.spec, P, h.device)
            flat = self._flat_cache[key]
        h.set_params_ref(flat, key)
        return h

    def with_system(self, radius=None, interaction_strength=None):
        """The same network with another sphere radius / interaction strength (what
        make_local_kinetic_energy(f, Q, r) evaluates, hamiltonian.py:83)."""
        import dataclasses as _dc

        other = object.__new__(type(self))
        other.__dict__.update(self.__dict__)
        kw = {}
        if radius is not None:
            kw["radius"] = float(radius)
        if interaction_strength is not None:
            kw["interaction_strength"] = float(interaction_strength)
        other.spec = _dc.replace(self.spec, **kw)
        other._flat_cache = {}
        return other

    def invalidate(self):
        """Force the next call to re-upload the parameters (after updates that bypass the
        tensors' version counters: optimizer kernels, ``p.data.copy_``)."""
        self._flat_cache.clear()
        self._epoch += 1
