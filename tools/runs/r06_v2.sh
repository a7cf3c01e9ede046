#!/bin/bash
# round 6 v2: the o~ cross-route test (quantiles), then the same-box A/B of the bench
# (old = round-5 final library, new = this tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ofeat.py \
  > $O/tests.log 2>&1
rc=$?; grep "N=" $O/tests.log; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in old new; do
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || exit 1
    echo "$v $i done"
  done
done
python tools/ab_table.py $O/ab_old_*.json $O/ab_new_*.json
