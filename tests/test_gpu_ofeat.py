"""Layer 1's attention output in feature space (round 6, dh_internal.h ofeat_k).

The layer-1 values are v_j = f~_j Wv~ (f~ = the four input features and 1), so the attention
output o_i = sum_j A_ij v_j equals o~_i Wv~ with o~_i = sum_j A_ij f~_j, and the next map
o Wol = o~ (Wv~ Wol) = o~ U contracts over 8 H = 32 instead of 256 (psiformer.py:42-45).  The
chain kernel's prologue (log psi, rows < 65536) and attention_feat2_kernel + gemm_lnch (the
local energy) take that form; the log-psi path for larger batches still forms o (256 wide,
attention_val_kernel) and contracts it with Wol.  Both routes must agree to f32 rounding on the
same walkers (distribution of the relative difference: median, p99, max): the first 1000
walkers of a batch past 65536 rows (the o route) against the same 1000 walkers alone (the o~
route, with a partial last tile), for N = 6 (C2), N = 3, the two-spin N = 4 and N = 10 (C4:
90-row tiles of 9 whole walkers); at N = 20 (C5) every batch size runs the chain (80-row layer-1
tiles of 4 walkers, 96-row layer-2 tiles with the orbital map), so the big batch must reproduce
the small one; and the local energy of the o~ route against the float64 oracle lives in
test_gpu_parity.py / test_gpu_floor.py."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from deephall_amd import config, make_network
from deephall_amd.random import Key, PRNGKey
from deephall_amd.train import init_guess

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nspins,flux", [((6, 0), 15), ((3, 0), 2), ((2, 2), 3), ((10, 0), 23), ((20, 0), 57)])
def test_chain_ofeat_matches_o_route(cuda, nspins, flux):
    N = sum(nspins)
    model = make_network(config.System(nspins=nspins, flux=flux), config.Network())
    params = model.init(PRNGKey(11), device=cuda)
    # rows = big * N >= 65536: the non-chain log-psi path (at N = 20 the chain at any size)
    big = 65536 // N + 64
    x = init_guess(Key(5), big, N, cuda, network=model)
    lp_big = model.apply(params, x)[:1000].cpu().numpy()
    lp_small = model.apply(params, x[:1000].contiguous()).cpu().numpy()
    assert np.isfinite(lp_small).all()
    d = np.abs(lp_small.real - lp_big.real) / np.maximum(np.abs(lp_big.real), 1.0)
    q = np.percentile(d, [50, 99, 100])
    print(f"N={N}: relative |d log psi| median {q[0]:.2e} p99 {q[1]:.2e} max {q[2]:.2e}")
    # two f32 routes: a walker with an ill-conditioned orbital matrix amplifies the rounding of
    # either (test_gpu_floor.py's gates measure the same spread against the float32 reference run);
    # the N x N determinant's amplification grows with N, so the gates scale with N / 10 past N = 10
    # (N = 20 measured: median 9.6e-7, p99 2.3e-5, max 1.1e-4; the phase's worst walker 2.6e-4)
    sc = max(1.0, N / 10)
    assert q[0] < 1e-6 * sc and q[1] < 2e-5 * sc and q[2] < 1e-3, q
    ph = np.abs(np.angle(np.exp(1j * (lp_small.imag - lp_big.imag))))
    assert ph.max() < 1e-4 * sc**2  # N = 20 measured 2.6e-4 on the worst of 1000 walkers
