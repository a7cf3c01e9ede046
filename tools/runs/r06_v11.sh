#!/bin/bash
# round 6 v11: envelope first at C4 / C5 (Weff = E2 W2, six special F rows, env_phi_kernel):
# parity / floor / bitwise tests, then the C4 / C5 lines A/B (pre_env = before, new = this tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v11
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_floor.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1; do
  for v in pre_env new; do
    DH_LIB_PATH=ab/$v.so timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || exit 1
  done
done
python tools/ab_table.py $O/ab_pre_env_*.json $O/ab_new_*.json
python - <<'PY'
import json
for v in ("pre_env", "new"):
    d = json.loads(open(f"gpurun_out/r06_v11/ab_{v}_1.json").read().strip().splitlines()[-1])
    for t, c in d["configs_1gpu"].items():
        print(v, t, c["value"], c["ms_per_step"], c.get("walker_steps_per_sec"), c["kernels_ms_per_step"])
PY
