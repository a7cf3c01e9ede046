#!/bin/bash
# round 6 v17: layer 1 of the local energy at N = 10, 20 in one launch (layer1_ch_kernel):
# o~ route / parity / floor tests, then the C2 / C4 / C5 A/B (base = HEAD, new = this tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v17
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ofeat.py tests/test_gpu_parity.py tests/test_gpu_floor.py > $O/tests.log 2>&1
rc=$?; grep -E "N=|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
for v in base new; do
  DH_LIB_PATH=ab/$v.so timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 > $O/ab_${v}.json 2> $O/ab_${v}.err || exit 1
done
python tools/ab_table.py $O/ab_base.json $O/ab_new.json
