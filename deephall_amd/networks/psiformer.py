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

All arithmetic runs in the HIP library (include/deephall_amd.h); this module
only packs parameters into the layout of ``dh_param_layout`` and manages the
per-device handle and workspace.
"""

from __future__ import annotations

import ctypes as C
import os
import math
from dataclasses import dataclass

import numpy as np
import torch

from .. import _lib

_HANDLES: dict = {}


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
        c.orbital_type = 0 if str(getattr(self.orbital_type, "value", self.orbital_type)) == "full" else 1
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
        nseg = self.lib.dh_param_layout(self.h, None, 0)
        offs = (C.c_size_t * (nseg + 1))()
        self.lib.dh_param_layout(self.h, offs, nseg + 1)
        self.offsets = [int(o) for o in offs]
        self.nparams = self.offsets[-1]
        self.ws = {}  # one workspace per HIP stream (walker groups may run on parallel streams)
        self._params_key = None
        self.set_gemm_mode(_GEMM_MODE)

    def set_gemm_mode(self, mode: str):
        """GEMM arithmetic: "x6all" (split-bf16, f32-accurate, every GEMM; default), "x6"
        (split-bf16 for the local-energy channel rows only) or "f32" (exact-f32 MFMA)."""
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

    def set_params(self, packed: torch.Tensor, key):
        if self._params_key == key:
            return
        assert packed.numel() == self.nparams and packed.dtype == torch.float32 and packed.is_cuda
        _lib.check(self.lib.dh_set_params(self.h, _ptr(packed), self.nparams, _stream(self.device)))
        self._packed = packed  # keep alive while the copy is in flight
        self._params_key = key


_GEMM_MODES = {"f32": 0, "x6": 1, "x6all": 2}
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
    for i in range(2 * nblk):
        s[ob + f"DenseGeneral_{i}/kernel"] = (D, M, N, K)
        s[ob + f"DenseGeneral_{i}/bias"] = (M, N, K)
    s["Jastrow_0/ee_par"] = (1,)
    s["Jastrow_0/ee_anti"] = (1,)
    return s


def init_params(spec: NetworkSpec, seed: int, device="cpu") -> dict:
    """Flax-default initialisation: lecun_normal (truncated to 2 sigma) kernels
    (fan_in = input features; H*dh for the attention output), zero biases,
    LayerNorm scale 1, Jastrow alphas 1 (blocks.py:92,100)."""
    rng = np.random.default_rng(seed)
    out = {}
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
        out[name] = torch.tensor(arr, dtype=torch.float32, device=device)
    return out


def pack_params(spec: NetworkSpec, params: dict, offsets: list, device) -> torch.Tensor:
    """Packed float32 device buffer in the dh_param_layout order (include/deephall_amd.h).

    The attention output projection and the following bias-free Dense
    (psiformer.py:44-45) are folded into one matrix Wol = Wo @ Wl (computed in
    float64), bol = bo @ Wl.
    """
    P = flatten_params(params)
    D, M, N, K = spec.D, spec.M, spec.nelec, spec.ndets
    dev = torch.device(device)
    buf = torch.zeros(offsets[-1], dtype=torch.float32, device=dev)
    f64 = lambda name: P[name].detach().to(dev, torch.float64)  # noqa: E731
    seg = 0

    def put(t):
        nonlocal seg
        flat = t.reshape(-1).to(torch.float32)
        size = offsets[seg + 1] - offsets[seg]
        assert flat.numel() <= size, (seg, flat.numel(), size)
        buf[offsets[seg] : offsets[seg] + flat.numel()] = flat
        seg += 1

    p = "PsiformerLayers_0/"
    put(f64(p + "Dense_0/kernel"))
    for l in range(spec.num_layers):
        mha = p + f"MultiHeadAttention_{l}/"
        wq = torch.cat([f64(mha + n + "/kernel").reshape(D, D) for n in ("query", "key", "value")], 1)
        bq = torch.cat([f64(mha + n + "/bias").reshape(D) for n in ("query", "key", "value")])
        wl = f64(p + f"Dense_{2 * l + 1}/kernel")
        put(wq)
        put(bq)
        put(f64(mha + "out/kernel").reshape(D, D) @ wl)
        put(f64(mha + "out/bias") @ wl)
        put(torch.stack([f64(p + f"LayerNorm_{2 * l}/scale"), f64(p + f"LayerNorm_{2 * l}/bias")]))
        put(f64(p + f"Dense_{2 * l + 2}/kernel"))
        put(f64(p + f"Dense_{2 * l + 2}/bias"))
        put(torch.stack([f64(p + f"LayerNorm_{2 * l + 1}/scale"), f64(p + f"LayerNorm_{2 * l + 1}/bias")]))
    ob = "Orbitals_0/featured_orbitals/"
    nblk = sum(1 for n in spec.nspins if n > 0)
    MNK = M * N * K
    cols = nblk * 2 * MNK
    ld = ((cols + 127) // 128) * 128
    W = torch.zeros(D, ld, dtype=torch.float64, device=dev)
    bvec = torch.zeros(ld, dtype=torch.float64, device=dev)
    for i in range(2 * nblk):  # (blk, part) order: DenseGeneral_{2 blk + part}
        W[:, i * MNK : (i + 1) * MNK] = f64(ob + f"DenseGeneral_{i}/kernel").reshape(D, MNK)
        bvec[i * MNK : (i + 1) * MNK] = f64(ob + f"DenseGeneral_{i}/bias").reshape(MNK)
    put(W)
    put(bvec)
    jp = P.get("Jastrow_0/ee_par")
    ja = P.get("Jastrow_0/ee_anti")
    put(
        torch.tensor(
            [float(jp.reshape(-1)[0]) if jp is not None else 1.0, float(ja.reshape(-1)[0]) if ja is not None else 1.0],
            dtype=torch.float64,
            device=dev,
        )
    )
    # layer-1 q|k|v projection folded into the input map: W0 @ Wqkv (float64), [4][3D]
    if spec.num_layers > 0:
        mha = p + "MultiHeadAttention_0/"
        wq0 = torch.cat([f64(mha + n + "/kernel").reshape(D, D) for n in ("query", "key", "value")], 1)
        put(f64(p + "Dense_0/kernel") @ wq0)
    else:
        seg += 1
    assert seg == len(offsets) - 1
    return buf


class Psiformer:
    """Psiformer(nspins, Q, ndets, num_heads, heads_dim, num_layers, orbital_type)
    (psiformer.py:63-91) backed by the HIP kernels."""

    def __init__(self, nspins, Q, ndets, num_heads, heads_dim, num_layers, orbital_type="full", system=None):
        self.nspins = tuple(int(n) for n in nspins)
        self.Q = float(Q)
        self.ndets = int(ndets)
        self.num_heads, self.heads_dim, self.num_layers = int(num_heads), int(heads_dim), int(num_layers)
        self.orbital_type = str(getattr(orbital_type, "value", orbital_type))
        if self.orbital_type != "full":
            raise NotImplementedError("orbital type 'sparse' (blocks.py:52-62) is not implemented on MI355X yet")
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
        self._pack_cache = {}

    # ---- reference-compatible entry points
    def init(self, key, data=None, device=None) -> dict:
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

    # ---- plumbing
    def _check_walkers(self, data: torch.Tensor) -> torch.Tensor:
        if data.dim() != 3 or data.shape[1] != self.spec.nelec or data.shape[2] != 2:
            raise ValueError(f"walkers must be [B, {self.spec.nelec}, 2], got {tuple(data.shape)}")
        if not data.is_cuda:
            raise RuntimeError("deephall_amd runs on the GPU only (no CPU fallback)")
        return data.to(torch.float32).contiguous()

    def prepare(self, params, device) -> NativeHandle:
        h = get_handle(self.spec, device)
        flat = flatten_params(params) if isinstance(params, dict) else params
        key = (id(params), tuple((id(v), v._version) for v in flat.values()) if isinstance(flat, dict) else None)
        if key not in self._pack_cache:
            self._pack_cache.clear()
            self._pack_cache[key] = pack_params(self.spec, flat, h.offsets, h.device)
        h.set_params(self._pack_cache[key], key)
        return h
