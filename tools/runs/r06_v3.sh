#!/bin/bash
# round 6 v3: layer 1 whole in one launch (gemm_lnch MODE 2, coefficient space): GPU suite,
# smoke, then a same-box A/B (old = round-5 final, v1 = o~ only, new = this tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v3
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --maxfail=8 --timeout 300 --timeout-method thread -m gpu tests/ \
  > $O/tests.log 2>&1
rc=$?; tail -12 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
for i in 1 2; do
  for v in old v1 new; do
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || exit 1
    echo "$v $i done"
  done
done
python tools/ab_table.py $O/ab_old_*.json $O/ab_v1_*.json $O/ab_new_*.json
