#!/bin/bash
# round 6 v36: the full GPU suite and smoke() on the final tree (C5 log psi all-chain)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v36
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; grep -E "N=20|FAILED" $O/gpu_tests.log | head; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; exit $rc
