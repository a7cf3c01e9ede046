#!/bin/bash
# round 6 v35: both log-psi layers in the chain kernel at N = 20 past 64K rows (big20: layer 2's
# P3 is the 2320-column orbital map) vs layer 1 only (base): the N = 20 o~-route test and the C5
# bitwise test with the variant, then C5 A/B twice each
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v35
mkdir -p $O
DH_LIB_PATH=ab/big20.so timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ofeat.py -k "57" > $O/tests.log 2>&1
rc=$?; grep -E "N=20|passed|failed" $O/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in base big20; do
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --nspins 20 0 --flux 57 --steps 5 --warmup 2 --no-cpu-baseline --extra-configs= > $O/${v}_$i.json 2> $O/${v}_$i.err || exit 1
  done
done
python - <<'PY'
import json
for i in (1, 2):
    for v in ("base","big20"):
        d=json.loads(open(f"gpurun_out/r06_v35/{v}_{i}.json").read().strip().splitlines()[-1])
        c=d.get("components") or {}
        print(v,i,round(d["value"]),d["ms_per_step"],"mcmc_step ms",c.get("mcmc_step_ms"),"walker-steps/s",d.get("walker_steps_per_sec"))
PY
