"""Worker of tests/test_gpu_chain_attn.py (not a test module).

Log psi of B walkers and two MCMC moves through the production path, with layer 1's
attention either inside the chain kernel (default) or as its own attention_val_kernel
launch (DH_CHAIN_ATTN=0, set by the parent: the switch is read once per process).
Writes log psi, the moved walkers and the accept counts to argv[1] (.npz).
argv: out nspins_up nspins_down flux B
"""

from __future__ import annotations

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    out, nu, nd, flux, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    from deephall_amd import config, make_network
    from deephall_amd.mcmc import make_mcmc_step
    from deephall_amd.random import Key, PRNGKey
    from deephall_amd.train import init_guess

    dev = torch.device("cuda", 0)
    model = make_network(config.System(nspins=(nu, nd), flux=flux), config.Network())
    params = model.init(PRNGKey(11), device=dev)
    data = init_guess(Key(5), B, nu + nd, dev, network=model)
    lp = model.apply(params, data)
    step = make_mcmc_step(model, batch_per_device=B, steps=2)
    data, _ = step(params, data, PRNGKey(3), 0.3, reduce=False)
    torch.cuda.synchronize()
    np.savez(out, lp_re=lp.real.cpu().numpy(), lp_im=lp.imag.cpu().numpy(), data=data.cpu().numpy(),
             nacc=step.last_n_accept.cpu().numpy())


if __name__ == "__main__":
    main()
