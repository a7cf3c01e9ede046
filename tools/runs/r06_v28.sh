#!/bin/bash
# round 6 v28: layer1_ch's LN_ch1 statistics from the Gram of E (no per-feature sums): floor /
# parity / fused-vs-two-pass tests, then C4 / C5 A/B (nogram = the per-feature sums)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v28
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -s --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_floor.py tests/test_gpu_lnch.py -k "not C2_bench" > $O/tests.log 2>&1
rc=$?; grep -E "^C4|^C5|passed|failed" $O/tests.log | tail -26; [ $rc -eq 0 ] || exit $rc
for v in nogram new; do
  for cfg in "10 0 23 c4" "20 0 57 c5"; do
    set -- $cfg
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --nspins $1 $2 --flux $3 --steps 5 --warmup 2 --no-cpu-baseline --no-components --extra-configs= > $O/${v}_$4.json 2> $O/${v}_$4.err || exit 1
  done
done
python - <<'PY'
import json
for v in ("nogram","new"):
    for c in ("c4","c5"):
        d=json.loads(open(f"gpurun_out/r06_v28/{v}_{c}.json").read().strip().splitlines()[-1])
        k=d.get("kernels",{}).get("layer1_ch",{})
        print(v,c,round(d["value"]),d["ms_per_step"],"layer1_ch us",round(k.get("avg_us",0),1))
PY
