#!/bin/bash
# round 6 v25: layer1_ch_kernel with r V on the matrix cores (base = HEAD, valu = this tree with
# the VALU form, new = MFMA form): floor / parity tests, C4 / C5 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v25
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_floor.py > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in base valu new; do
  for cfg in "10 0 23 c4" "20 0 57 c5"; do
    set -- $cfg
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --nspins $1 $2 --flux $3 --steps 5 --warmup 2 --no-cpu-baseline --no-components --extra-configs= > $O/${v}_$4.json 2> $O/${v}_$4.err || exit 1
  done
done
python - <<'PY'
import json
for v in ("base","valu","new"):
    for c in ("c4","c5"):
        d=json.loads(open(f"gpurun_out/r06_v25/{v}_{c}.json").read().strip().splitlines()[-1])
        k=d.get("kernels",{}).get("layer1_ch",{})
        print(v,c,round(d["value"]),d["ms_per_step"],"layer1_ch us",round(k.get("avg_us",0),1))
PY
