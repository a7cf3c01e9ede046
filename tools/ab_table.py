"""Summarise gpurun_out/ab/*.json (tools/ab_bench.sh): value and per-kernel ms per step."""
import glob
import json
import sys

rows = {}
for f in sorted(glob.glob("gpurun_out/ab/*.json")):
    txt = open(f).read().strip().splitlines()
    if not txt:
        continue
    d = json.loads(txt[-1])
    tag = f.split("/")[-1][:-5]
    rows[tag] = d
keys = sorted({k for d in rows.values() for k in d.get("kernels", {})})
print(f"{'run':8s} {'value':>10s} {'ms':>7s} " + " ".join(f"{k[:12]:>12s}" for k in keys))
for tag, d in rows.items():
    ks = d.get("kernels", {})
    print(f"{tag:8s} {d['value']:10.0f} {d['ms_per_step']:7.3f} " +
          " ".join(f"{ks[k]['ms_per_step']:12.3f}" if k in ks else " " * 12 for k in keys))
