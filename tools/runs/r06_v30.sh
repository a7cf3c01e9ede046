#!/bin/bash
# round 6 v30: attention_mfma_kernel<10> at 4 waves per SIMD (w10) vs the compiler's 3 (new):
# C4 A/B twice each
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v30
mkdir -p $O
for i in 1 2; do
  for v in new w10; do
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --nspins 10 0 --flux 23 --steps 5 --warmup 2 --no-cpu-baseline --no-components --extra-configs= > $O/${v}_$i.json 2> $O/${v}_$i.err || exit 1
  done
done
python - <<'PY'
import json
for i in (1, 2):
    for v in ("new","w10"):
        d=json.loads(open(f"gpurun_out/r06_v30/{v}_{i}.json").read().strip().splitlines()[-1])
        k=d.get("kernels",{})
        a=[(n, round(x["avg_us"],1)) for n,x in k.items() if "attention" in n]
        print(v,i,round(d["value"]),d["ms_per_step"],a)
PY
