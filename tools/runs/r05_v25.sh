#!/bin/bash
# round 5 v25: closing candidate — GPU suite, smoke, round profile (kernel stats, GEMM PMC traffic,
# full default bench line with C4 / C5 and the CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05_v25
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05_v25/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05_v25/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_v25/smoke.log 2>&1 || exit 1
tail -3 gpurun_out/r05_v25/smoke.log
TAG=r05_v25 bash tools/profile_round.sh
