#!/bin/bash
# round 6 v31: final round profile of the round-6 tree (C2 kernel stats, PMC traffic and MFMA busy,
# bench line) and the C4 / C5 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r06_v31 bash tools/profile_round.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v31
for cfg in "10 0 23 c4" "20 0 57 c5"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$4 -o run -- python3 bench.py --nspins $1 $2 --flux $3 --steps 2 --warmup 1 --burn-in 0 --no-cpu-baseline --no-components --extra-configs= > $O/bench_$4.json || exit 1
  python3 tools/prof_summary.py $(find $O/trace_$4 -name "*kernel_stats.csv") "r06_v31 $4: rocprofv3 --kernel-trace --stats -- python bench.py --nspins $1 $2 --flux $3 --steps 2 --warmup 1 --burn-in 0" > $O/kernel_stats_$4.md
done
tail -1 $O/bench.json | cut -c1-400
