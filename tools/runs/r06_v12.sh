#!/bin/bash
# round 6 v12: kernel stats of the C4 / C5 steps with the envelope-first path
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v12
mkdir -p $O
for cfg in "10 0 23 c4" "20 0 57 c5"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$4 -o run -- python3 bench.py --nspins $1 $2 --flux $3 --steps 2 --warmup 1 --burn-in 0 --no-cpu-baseline --no-components --extra-configs= > $O/bench_$4.json || exit 1
  python3 tools/prof_summary.py $(find $O/trace_$4 -name "*kernel_stats.csv") "r06_v12 $4" > $O/kernel_stats_$4.md
  head -22 $O/kernel_stats_$4.md
done
