#!/bin/bash
# round 6 v23: layer1_ch_kernel ablations at C4 / C5 (bit 0 no x, 1 no LN_ch1, 2 no r rows / y,
# 3 no LN_ch2; wrong results, timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v23
mkdir -p $O
for v in new abl1 abl2 abl4 abl8; do
  for cfg in "10 0 23 c4" "20 0 57 c5"; do
    set -- $cfg
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --nspins $1 $2 --flux $3 --steps 3 --warmup 1 --burn-in 0 --no-cpu-baseline --extra-configs= > $O/${v}_$4.json 2> $O/${v}_$4.err || exit 1
  done
done
python - <<'PY'
import json
for v in ("new","abl1","abl2","abl4","abl8"):
    for c in ("c4","c5"):
        d=json.loads(open(f"gpurun_out/r06_v23/{v}_{c}.json").read().strip().splitlines()[-1])
        k=d.get("kernels",{}).get("layer1_ch")
        print(v,c,round(d["value"]),d["ms_per_step"],"layer1_ch",k)
PY
