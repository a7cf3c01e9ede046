#!/bin/bash
# round 6 v20: the full GPU suite and smoke() on the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v20
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -4 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -3 $O/smoke.log; exit $rc
