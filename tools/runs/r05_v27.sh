#!/bin/bash
# round 5 v27: the final tree (gemm_lnch without the SLP vectorizer): GPU suite, smoke, default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05_v27
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05_v27/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05_v27/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_v27/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r05_v27/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r05_v27/bench.json 2> gpurun_out/r05_v27/bench.err || exit 1
tail -c 400 gpurun_out/r05_v27/bench.json
