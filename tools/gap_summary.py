"""GPU idle time between kernels from a rocprofv3 kernel trace (``*_kernel_trace.csv``).

Sorts the dispatches of the busiest queue by start time, reports the idle gap before each
kernel aggregated by the kernel that FOLLOWS the gap (the launch the GPU was waiting
for), and the total busy / idle split over the last ``--window`` ms of the trace (the
bench's timed steps).  Usage: python tools/gap_summary.py trace.csv [window_ms]
"""

import csv
import sys
from collections import defaultdict

from prof_summary import short


def main(path, window_ms=None):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    if window_ms is not None:
        t_end = ev[-1][1]
        ev = [e for e in ev if e[0] >= t_end - window_ms * 1e6]
    gaps = defaultdict(lambda: [0, 0.0, 0.0])  # count, total us, max us
    busy = idle = 0.0
    prev_end = ev[0][0]
    for s, e, name in ev:
        g = max(0.0, (s - prev_end) / 1e3)
        idle += g
        busy += max(0.0, (e - max(s, prev_end)) / 1e3)
        c = gaps[name]
        c[0] += 1
        c[1] += g
        c[2] = max(c[2], g)
        prev_end = max(prev_end, e)
    span = (ev[-1][1] - ev[0][0]) / 1e3
    print(f"span {span / 1e3:.3f} ms, busy {busy / 1e3:.3f} ms, idle {idle / 1e3:.3f} ms ({100 * idle / span:.1f} %)")
    print("| next kernel | gaps | idle us total | max gap us |")
    print("|---|---|---|---|")
    for name, (n, tot, mx) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"| {name} | {n} | {tot:.1f} | {mx:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else None)
