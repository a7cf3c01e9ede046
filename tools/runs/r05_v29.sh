#!/bin/bash
# round 5 v29: the final tree (det_energy_wave leaves by powers by squaring): GPU suite, smoke, default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05_v29
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05_v29/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05_v29/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_v29/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r05_v29/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r05_v29/bench.json 2> gpurun_out/r05_v29/bench.err || exit 1
tail -c 400 gpurun_out/r05_v29/bench.json
