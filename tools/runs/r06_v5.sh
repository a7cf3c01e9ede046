#!/bin/bash
# round 6 v5: MODE 2 with the r rows formed by thread (electron, column): parity / floor / lnch
# tests, then rocprofv3 kernel stats of the bench (C2)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_floor.py tests/test_gpu_lnch.py tests/test_gpu_ofeat.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 5 --warmup 1 --burn-in 0 --no-cpu-baseline --no-components --extra-configs= > $O/bench_under_rocprof.json || exit 1
python3 tools/prof_summary.py $(find $O/trace -name "*kernel_stats.csv") "r06_v5" > $O/kernel_stats.md
head -16 $O/kernel_stats.md
