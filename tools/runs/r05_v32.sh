#!/bin/bash
# round 5 v32: envelope leaves by powers by squaring in env_stream / det_energy_kernel (N = 10, 20;
# ab/leaf_sq.so, DET_LEAF_SQ=1) vs the in-tree build: full GPU suite through the variant (C4 / C5
# floor gates), same-box C4 / C5 bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
DH_LIB_PATH=ab/leaf_sq.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v32_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v32_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --steps 3 --mcmc-calls 2 --extra-configs=C4,C5 --extra-steps 3"
for i in 1 2; do
  timeout -k 10 400 $B > gpurun_out/r05/v32_ab_head_$i.json 2>/dev/null || exit 1
  DH_LIB_PATH=ab/leaf_sq.so timeout -k 10 400 $B > gpurun_out/r05/v32_ab_sq_$i.json 2>/dev/null || exit 1
  echo "round $i done"
done
