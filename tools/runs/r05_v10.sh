#!/bin/bash
# round 5 v10: GPU suite with the chain kernel's P1 residual loads batched ahead of P2's weight
# prefetch; same-box A/B against ab/head_x6.so (the previous gemm_x6.hip), chain stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v10_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v10_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --steps 20 --mcmc-calls 20 --extra-configs="
for i in 1 2 3; do
  DH_LIB_PATH=ab/head_x6.so timeout -k 10 300 $B > gpurun_out/r05/v10_ab_head_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B > gpurun_out/r05/v10_ab_new_$i.json 2>/dev/null || exit 1
  echo "ab round $i done"
done
DH_LIB_PATH=ab/chain_stamp.so timeout -k 10 200 python tools/chain_stamp.py 6 4096 > gpurun_out/r05/v10_chain_stamps.txt 2>&1 || exit 1
echo stamps-done
