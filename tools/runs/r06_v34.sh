#!/bin/bash
# round 6 v34: four waves per SIMD for env_phi_kernel<10> (epw4) and layer1_ch_kernel<10> (l1w4)
# against the current occupancy (base): C4 A/B twice each
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v34
mkdir -p $O
for i in 1 2; do
  for v in base epw4 l1w4; do
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --nspins 10 0 --flux 23 --steps 5 --warmup 2 --no-cpu-baseline --no-components --extra-configs= > $O/${v}_$i.json 2> $O/${v}_$i.err || exit 1
  done
done
python - <<'PY'
import json
for i in (1, 2):
    for v in ("base","epw4","l1w4"):
        d=json.loads(open(f"gpurun_out/r06_v34/{v}_{i}.json").read().strip().splitlines()[-1])
        k=d.get("kernels",{})
        print(v,i,round(d["value"]),d["ms_per_step"],{n: round(x["avg_us"],1) for n,x in k.items() if n in ("layer1_ch","det_energy","gemm_ch")})
PY
