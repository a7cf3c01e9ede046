#!/bin/bash
# round 5 v7: GPU suite with layer 1's channel residual formed in gemm_lnch's MODE-0 epilogue
# (the input kernel writes geometry only); same-box A/B DH_LNCH_FEAT=0 / 1 on the C2 line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v7_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v7_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --steps 20 --mcmc-calls 5 --extra-configs="
for i in 1 2 3; do
  DH_LNCH_FEAT=0 timeout -k 10 300 $B > gpurun_out/r05/v7_ab_h0_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B > gpurun_out/r05/v7_ab_feat_$i.json 2>/dev/null || exit 1
  echo "ab round $i done"
done
