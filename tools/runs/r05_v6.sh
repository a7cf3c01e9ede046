#!/bin/bash
# round 5 v6: GPU suite with the restructured layer-1 feature-space attention
# (attention_feat2_kernel, O(N) tangent channels), same-box A/B DH_ATTN_FEAT2=0 / 1 on the
# C2 line and the C4 / C5 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v6_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v6_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --steps 10 --mcmc-calls 5 --extra-configs=C4,C5 --extra-steps 3"
for i in 1 2; do
  DH_ATTN_FEAT2=0 timeout -k 10 300 $B > gpurun_out/r05/v6_ab_feat1_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B > gpurun_out/r05/v6_ab_feat2_$i.json 2>/dev/null || exit 1
  echo "ab round $i done"
done
