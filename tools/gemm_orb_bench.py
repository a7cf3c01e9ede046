"""Orbital-map GEMM shapes of C4 / C5 (ncols = 2 M N = 480 / 2320): persistent kernel widths."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parent))
from gemm_bench import run  # noqa: E402

for name, rows, n in (("c4_orb", 4096 * 10 * 25, 480), ("c5_orb", 2048 * 20 * 45, 2320), ("c5_orb_val", 4096 * 20, 2320)):
    line = [f"{name:10s}"]
    for v in (250, 251, 252, 255):
        ms, tf = run(v, rows, n, 256, 25 if name == "c4_orb" else 45, reps=5, check=True)
        line.append(f"v{v}: {ms * 1e3:8.1f}us {tf:6.1f}TF")
    print("  ".join(line), flush=True)
