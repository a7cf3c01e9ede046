"""Phase stamps of the log-psi chain kernel (chain_x6s) inside the model's forward pass at
the bench batch: build with  FILE=gemm_x6.hip bash tools/build_variant.sh chain_stamp -DCHAIN_STAMP=1
and run  DH_LIB_PATH=ab/chain_stamp.so python tools/chain_stamp.py [N] [B]  on the GPU box.

Per launch form (layer 1 with its attention prologue / layer 2 with the orbital map), the
mean over tiles of each phase in shader-clock cycles (s_memtime) and as a share of the tile."""

import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from deephall_amd import _lib, config, make_network  # noqa: E402
from helpers import make_walkers  # noqa: E402

NAMES = ["prologue (o / X1 -> planes)", "P1 GEMM", "P1 bias + residual", "P1 LayerNorm", "P1 planes + barrier",
         "P2 GEMM", "P2 h1 + tanh", "P2 LayerNorm", "P2 planes + h + barrier",
         "P3 pass 0 GEMM", "P3 pass 0 stores", "P3 pass 1 GEMM", "P3 pass 1 stores", "P3 pass 2 GEMM",
         "P3 pass 2 stores"]
# layer 1 (round 6): o~ prologue, 32-deep P1, LN1 statistics + coefficient rows, P2 = r V, tanh, r B
NAMES1 = ["prologue (o~ -> planes)", "P1 GEMM (o~ U, 32 deep)", "P1 bias + f W0", "LN1 stats + r rows",
          "(none)", "P2: r V, tanh, += r B", "(none)", "P2 LayerNorm", "P2 planes + h + barrier",
          "P3 pass 0 GEMM", "P3 pass 0 stores", "P3 pass 1 GEMM", "P3 pass 1 stores", "P3 pass 2 GEMM",
          "P3 pass 2 stores"]


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    lib = _lib.load()
    fn = lib.dh_debug_chain_stamps
    fn.argtypes = [C.c_void_p, C.c_int]
    system = config.System(nspins=(N, 0), flux={6: 15, 3: 2, 10: 23, 20: 57}[N])
    model = make_network(system, config.Network())
    params = model.init(1, device="cuda")
    x = torch.tensor(make_walkers(B, N, seed=3), device="cuda")
    for _ in range(3):
        model.apply(params, x)
    torch.cuda.synchronize()
    WG, NS = 512, 16
    buf = np.zeros(2 * WG * NS, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0
    st = buf.reshape(2, WG, NS).astype(np.int64)
    for slot, name in ((1, "layer 1 + attention (chain_x6s<0, N>)"), (0, "layer 2 + orbitals (chain_x6s<0, 0>)")):
        t = st[slot]
        used = t[:, 0] > 0
        t = t[used]
        if not len(t):
            continue
        last = max(i for i in range(NS) if (t[:, i] > 0).all())
        tot = (t[:, last] - t[:, 0]).mean()
        print(f"== {name}: {len(t)} tiles, tile span {tot:.0f} cycles (stamps 0..{last})")
        names = NAMES1 if slot == 1 else NAMES
        for i in range(last):
            d = (t[:, i + 1] - t[:, i]).mean()
            print(f"   {names[i]:30s} {d:9.0f} cycles  {100 * d / tot:5.1f} %")
        spread = (t[:, 0] - t[:, 0].min()) 
        print(f"   tile start spread: median {np.median(spread):.0f}, max {spread.max():.0f} cycles")


if __name__ == "__main__":
    main()
