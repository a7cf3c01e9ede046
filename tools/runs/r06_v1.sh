#!/bin/bash
# round 6 v1: layer 1's attention output in feature space (o~, K = 32 for the first map) +
# every getenv knob removed: GPU suite, smoke, then a same-box A/B of the bench (old = round-5
# final library, new = this tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v1
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ \
  > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
for i in 1 2; do
  for v in old new; do
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || exit 1
    echo "$v $i done"
  done
done
python tools/ab_table.py $O/ab_old_*.json $O/ab_new_*.json 2>/dev/null | tail -30
