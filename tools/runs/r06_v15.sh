#!/bin/bash
# round 6 v15: envelope leaves in env_coef (leaf table by LDS-DMA into env_phi), C5's special-row
# orbital map on gemm_x6m: parity / floor tests, then C4 / C5 A/B (base = HEAD, nowide = leaves
# only, new = this tree) and a C5 kernel table
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v15
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_floor.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in base nowide new; do
  DH_LIB_PATH=ab/$v.so timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 > $O/ab_${v}.json 2> $O/ab_${v}.err || exit 1
done
python tools/ab_table.py $O/ab_base.json $O/ab_nowide.json $O/ab_new.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o run -- python3 bench.py --nspins 20 0 --flux 57 --steps 2 --warmup 1 --burn-in 0 --no-cpu-baseline --no-components --extra-configs= > $O/bench_c5.json || exit 1
python3 tools/prof_summary.py $(find $O/trace_c5 -name "*kernel_stats.csv") "r06_v15 c5" > $O/kernel_stats_c5.md
head -22 $O/kernel_stats_c5.md
