"""Layer 1's attention inside the chain kernel's prologue (gemm_x6.hip chain_x6s_kernel<0, N>,
attn_val.h) computes exactly what the separate attention_val_kernel<N, true> launch does:
log psi, the walkers after two MCMC moves and the accept counts are BIT-identical with the
fusion on and off (DH_CHAIN_ATTN=0), including a partial last 96-row tile (B = 1000 at N = 6)
and the other walker-aligned electron counts (N = 3 and the two-spin N = 4)."""

from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _run(tmp_path, tag, env_extra, nspins, flux, B):
    out = tmp_path / f"{tag}.npz"
    env = dict(os.environ, **env_extra)
    cmd = [sys.executable, str(ROOT / "tests" / "chain_attn_worker.py"), str(out), str(nspins[0]), str(nspins[1]),
           str(flux), str(B)]
    subprocess.run(cmd, env=env, check=True, timeout=100)
    return np.load(out)


@pytest.mark.parametrize("nspins,flux,B", [((6, 0), 15, 1000), ((3, 0), 2, 700), ((2, 2), 3, 512)])
def test_chain_attention_bitwise(tmp_path, nspins, flux, B):
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    fused = _run(tmp_path, "fused", {}, nspins, flux, B)
    sep = _run(tmp_path, "separate", {"DH_CHAIN_ATTN": "0"}, nspins, flux, B)
    for k in ("lp_re", "lp_im", "data", "nacc"):
        assert np.array_equal(fused[k], sep[k]), k
