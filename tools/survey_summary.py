"""Tabulate an f32-floor margin survey (DH_FLOOR_LOG jsonl written by tests/helpers.within_f32_floor)
into the text committed under profiles/: per gate (fixture/observable) the HIP / float32-run ratios
of median, 90th percentile and maximum, each as a fraction of its limit, the worst first.

    python tools/survey_summary.py gpurun_out/r04_survey_x6all.jsonl > profiles/r04_floor_survey.txt
"""

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
from helpers import FLOOR_X, FLOOR_X_MAX, FLOOR_X_P90  # noqa: E402


def main(path):
    rows = [json.loads(line) for line in open(path)]
    gates = [r for r in rows if r.get("label")]
    print(f"# {path}: {len(gates)} gate evaluations (limits: median {FLOOR_X}x, p90 {FLOOR_X_P90}x, "
          f"max {FLOOR_X_MAX}x of the float32 run's error, every fixture)")
    print(f"# 'use' = the largest ratio / limit of the three; 1.0 = at the gate; 'abs' = passed on the "
          f"absolute floor (every error <= floor_abs)")
    print(f"{'gate':34s} {'med':>6s} {'p90':>6s} {'max':>6s} {'use':>6s} {'emax':>9s} {'fmax':>9s}")
    out = []
    for r in gates:
        use = max(r["med"] / FLOOR_X, r["p90"] / FLOOR_X_P90, r["max"] / FLOOR_X_MAX)
        absok = r["emax"] <= r["floor_abs"]
        out.append((0.0 if absok else use, r, absok))
    for use, r, absok in sorted(out, key=lambda t: -t[0]):
        tag = "abs" if absok else f"{use:6.2f}"
        print(f"{r['label']:34s} {r['med']:6.2f} {r['p90']:6.2f} {r['max']:6.2f} {tag:>6s} {r['emax']:9.2e} {r['fmax']:9.2e}")
    worst = max(u for u, _, _ in out)
    print(f"# worst use {worst:.2f}: margin {100 * (1 - worst):.0f}% to the gate")


if __name__ == "__main__":
    main(sys.argv[1])
