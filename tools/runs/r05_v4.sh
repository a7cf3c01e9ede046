#!/bin/bash
# round 5 v4: GPU suite with the split-bf16 layer-2 channel attention at N = 20
# (attention_x6_kernel), same-box A/B of the C5 line DH_ATTN_X6=0 / 1, then a C5 rocprofv3
# kernel-stats pass (where the C5 step goes, per kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v4_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v4_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --steps 10 --mcmc-calls 5 --extra-configs=C5 --extra-steps 3"
for i in 1 2; do
  DH_ATTN_X6=0 timeout -k 10 300 $B > gpurun_out/r05/v4_ab_f32_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B > gpurun_out/r05/v4_ab_x6_$i.json 2>/dev/null || exit 1
  echo "ab round $i done"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r05/v4_c5prof -o c5 -- \
  python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --nspins 20 0 --flux 57 --steps 3 --warmup 2 --mcmc-calls 2 \
  --extra-configs= > $GRAFT_REPO_ROOT/gpurun_out/r05/v4_c5prof.log 2>&1 || exit 1
echo prof-done
