"""Summarise bench JSON lines (tools/ab_bench.sh, tools/runs/*.sh A/B runs): value, walker-steps/s,
C4 / C5 lines and per-kernel ms per step.  usage: ab_table.py [files...] (default gpurun_out/ab/*.json)"""
import glob
import json
import sys

rows = {}
for f in sys.argv[1:] or sorted(glob.glob("gpurun_out/ab/*.json")):
    txt = open(f).read().strip().splitlines()
    if not txt:
        continue
    d = json.loads(txt[-1])
    tag = f.split("/")[-1][:-5]
    rows[tag] = d
keys = sorted({k for d in rows.values() for k in d.get("kernels", {})})
print(f"{'run':10s} {'value':>9s} {'ms':>6s} {'wsteps/s':>9s} {'C4':>8s} {'C5':>7s} " + " ".join(f"{k[:11]:>11s}" for k in keys))
for tag, d in rows.items():
    ks = d.get("kernels", {})
    c = d.get("configs_1gpu", {})
    c4 = c.get("C4", {}).get("value", float("nan"))
    c5 = c.get("C5", {}).get("value", float("nan"))
    print(f"{tag:10s} {d['value']:9.0f} {d['ms_per_step']:6.3f} {d.get('walker_steps_per_sec', 0) / 1e6:9.2f} {c4:8.0f} {c5:7.0f} " +
          " ".join(f"{ks[k]['ms_per_step']:11.3f}" if k in ks else " " * 11 for k in keys))
