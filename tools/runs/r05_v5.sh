#!/bin/bash
# round 5 v5: GPU suite with (a) attention_x6_kernel reloading every prefetch slot right after
# its commit (a whole channel of cover) and (b) the chain kernel's P3 passes on swapped MFMA
# operands with full-rate dword row stores (CHAIN_P3T); same-box A/Bs: DH_ATTN_X6=0/1 on the
# C5 line, ab/nop3t.so (CHAIN_P3T=0) on the C2 line / mcmc_step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v5_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v5_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --steps 10 --mcmc-calls 10"
for i in 1 2; do
  DH_LIB_PATH=ab/nop3t.so timeout -k 10 300 $B --extra-configs= > gpurun_out/r05/v5_ab_nop3t_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B --extra-configs= > gpurun_out/r05/v5_ab_p3t_$i.json 2>/dev/null || exit 1
  DH_ATTN_X6=0 timeout -k 10 300 $B --extra-configs=C5 --extra-steps 3 --mcmc-calls 3 > gpurun_out/r05/v5_ab_attf32_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B --extra-configs=C5 --extra-steps 3 --mcmc-calls 3 > gpurun_out/r05/v5_ab_attx6_$i.json 2>/dev/null || exit 1
  echo "ab round $i done"
done
