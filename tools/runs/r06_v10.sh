#!/bin/bash
# round 6 v10: layer 1's attention prologue spread over the whole workgroup: parity tests, chain
# stamps, A/B (c1 = previous commit, new = this tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v10
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_floor.py tests/test_gpu_ofeat.py tests/test_gpu_generic.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
DH_LIB_PATH=ab/chain_stamp.so timeout -k 10 200 python tools/chain_stamp.py 6 4096 > $O/chain_stamps.txt 2>&1 || exit 1
head -18 $O/chain_stamps.txt
for i in 1 2; do
  for v in c1 new; do
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --extra-configs= > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || exit 1
  done
done
python tools/ab_table.py $O/ab_c1_*.json $O/ab_new_*.json
