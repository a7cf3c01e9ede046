#!/bin/bash
# round 5 v8: GPU suite with (a) the radix-select keys held in registers in stats_kernel and
# (b) layer 1's channel residual formed by layernorm_ch_quad at N = 10, 20 (the input kernel
# writes geometry only there too); same-box A/B DH_LNCH_FEAT=0 / 1 on the C4 / C5 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v8_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v8_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --steps 10 --mcmc-calls 5 --extra-configs=C4,C5 --extra-steps 3"
for i in 1 2; do
  DH_LNCH_FEAT=0 timeout -k 10 300 $B > gpurun_out/r05/v8_ab_h0_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B > gpurun_out/r05/v8_ab_feat_$i.json 2>/dev/null || exit 1
  echo "ab round $i done"
done
