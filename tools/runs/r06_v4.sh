#!/bin/bash
# round 6 v4: rocprofv3 kernel stats of the bench (C2) for the MODE 2 tree
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v4
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 5 --warmup 1 --burn-in 0 --no-cpu-baseline --no-components --extra-configs= > $O/bench_under_rocprof.json || exit 1
python3 tools/prof_summary.py $(find $O/trace -name "*kernel_stats.csv") "r06_v4" > $O/kernel_stats.md
cat $O/kernel_stats.md | head -30
