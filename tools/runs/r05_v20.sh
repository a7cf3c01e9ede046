#!/bin/bash
# round 5 v20: dh_energy_stats alone at B = 4096 / 32768: production vs the quantiles-only ablation
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
for B in 4096 32768; do
  timeout -k 10 120 python tools/stats_bench.py $B 200 || exit 1
  DH_LIB_PATH=ab/stats_abl2.so timeout -k 10 120 python tools/stats_bench.py $B 200 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05/v20_stats.txt
