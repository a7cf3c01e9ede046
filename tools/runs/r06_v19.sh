#!/bin/bash
# round 6 v19: layer1_ch_kernel variants (rows of LDS reads in flight, waves per SIMD) at C4 / C5
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v19
mkdir -p $O
for v in new y2 x3y2 w3 w3y2; do
  for cfg in "10 0 23 c4" "20 0 57 c5"; do
    set -- $cfg
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --nspins $1 $2 --flux $3 --steps 5 --warmup 2 --no-cpu-baseline --no-components --extra-configs= > $O/${v}_$4.json 2> $O/${v}_$4.err || exit 1
  done
done
python - <<'PY'
import json
for v in ("new","y2","x3y2","w3","w3y2"):
    for c in ("c4","c5"):
        d=json.loads(open(f"gpurun_out/r06_v19/{v}_{c}.json").read().strip().splitlines()[-1])
        k=d.get("kernels_ms_per_step",{})
        print(v,c,round(d["value"]),d["ms_per_step"],k.get("layer1_ch"))
PY
