#!/bin/bash
# round 6 v10b: A/B of the workgroup-wide layer-1 prologue (c1 = HEAD's gemm_x6.hip, new = this tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v10
mkdir -p $O
for i in 1 2; do
  for v in c1 new; do
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --extra-configs= > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || exit 1
  done
done
python tools/ab_table.py $O/ab_c1_*.json $O/ab_new_*.json
