#!/bin/bash
# round 6 v37: the driver's default bench invocation on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v37
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
tail -1 $O/bench.json | cut -c1-300
python - <<'PY'
import json
d=json.loads(open("gpurun_out/r06_v37/bench.json").read().strip().splitlines()[-1])
print("value",d["value"],"ms",d["ms_per_step"],"wsteps",d.get("walker_steps_per_sec"),"frac",d["roofline"]["frac"],"cpu",d["cpu_baseline"]["value"])
for t,c in d.get("configs_1gpu",{}).items(): print(t,c["value"],c.get("walker_steps_per_sec"),c["ms_per_step"])
PY
