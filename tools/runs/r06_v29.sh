#!/bin/bash
# round 6 v29: gemm_x6m output tiles by nontemporal stores (nt) vs plain (new): C2 A/B twice
# each, then FETCH_SIZE of the nt build's x6m launches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v29
mkdir -p $O
for i in 1 2; do
  for v in new nt; do
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --extra-configs= > $O/${v}_$i.json 2> $O/${v}_$i.err || exit 1
  done
done
python tools/ab_table.py $O/new_*.json $O/nt_*.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
DH_LIB_PATH=ab/nt.so timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gemm_x6m" --output-format csv -d $O/fetch -o f -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-components --no-kernel-events --extra-configs= > /dev/null || exit 1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r06_v29/fetch/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    acc[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(k, "launches", len(v), "FETCH_SIZE x2 bytes per launch", 2 * 1024 * sum(v) / len(v))
PY
