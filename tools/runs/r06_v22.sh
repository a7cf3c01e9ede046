#!/bin/bash
# round 6 v22: layer 1 of log psi in the chain kernel at N = 20 past 64K rows (80-row tiles of
# 4 walkers, attention in the prologue): parity / floor / o~ tests, then C5 / C4 / C2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v22
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ofeat.py tests/test_gpu_parity.py tests/test_gpu_floor.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in base new; do
  DH_LIB_PATH=ab/$v.so timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 > $O/ab_${v}.json 2> $O/ab_${v}.err || exit 1
done
python tools/ab_table.py $O/ab_base.json $O/ab_new.json
python - <<'PY'
import json
for v in ("base","new"):
    d=json.loads(open(f"gpurun_out/r06_v22/ab_{v}.json").read().strip().splitlines()[-1])
    for t,c in d["configs_1gpu"].items():
        print(v,t,c["value"],c["ms_per_step"],c.get("walker_steps_per_sec"),c.get("mcmc_step_ms"))
PY
