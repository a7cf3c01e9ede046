#!/bin/bash
# round 5 v3: GPU suite with the register-streamed C5 envelope contraction (env_stream_kernel),
# then a same-box A/B of the C5 line: DH_ENV_STREAM=0 (round-4 LDS-DMA ring) vs the new kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v3_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v3_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --steps 10 --mcmc-calls 5 --extra-configs=C5 --extra-steps 3"
for i in 1 2; do
  DH_ENV_STREAM=0 timeout -k 10 300 $B > gpurun_out/r05/v3_ab_ring_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B > gpurun_out/r05/v3_ab_stream_$i.json 2>/dev/null || exit 1
  echo "ab round $i done"
done
