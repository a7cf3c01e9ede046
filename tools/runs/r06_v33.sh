#!/bin/bash
# round 6 v33: attention_mfma with two q|k|v prefetch register sets at N = 10 (new, 3 waves per
# SIMD) vs one set at 4 waves per SIMD (head): parity / floor tests, C4 / C5 A/B twice each
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v33
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_floor.py tests/test_gpu_lnch.py -k "not C2_bench" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in head new; do
    for cfg in "10 0 23 c4" "20 0 57 c5"; do
      set -- $cfg
      DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --nspins $1 $2 --flux $3 --steps 5 --warmup 2 --no-cpu-baseline --no-components --extra-configs= > $O/${v}_$4_$i.json 2> $O/${v}_$4_$i.err || exit 1
    done
  done
done
python - <<'PY'
import json
for i in (1, 2):
    for v in ("head","new"):
        for c in ("c4","c5"):
            d=json.loads(open(f"gpurun_out/r06_v33/{v}_{c}_{i}.json").read().strip().splitlines()[-1])
            k=d.get("kernels",{}).get("attention_ch",{})
            print(v,c,i,round(d["value"]),d["ms_per_step"],"attention_ch avg us",round(k.get("avg_us",0),1))
PY
