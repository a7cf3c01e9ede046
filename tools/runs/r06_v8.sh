#!/bin/bash
# round 6 v8: GPU suite (env_leaf powers test, partial-tile P3 stores), smoke, then the round
# profile: kernel stats, GEMM PMC traffic, MFMA-busy PMC, full default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v8
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q -s --maxfail=8 --timeout 300 --timeout-method thread -m gpu tests/ \
  > $O/tests.log 2>&1
rc=$?; grep "^M=" $O/tests.log; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
TAG=r06_v8 bash tools/profile_round.sh || exit 1
tail -c 600 gpurun_out/r06_v8/bench.json
