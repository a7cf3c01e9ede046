#!/bin/bash
# round 6 v7: the log-psi chain's layer 1 in coefficient space: GPU suite, then A/B
# (v1 = o~ only, m2 = + gemm_lnch MODE 2, new = + chain layer 1 coefficient form)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v7
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --maxfail=8 --timeout 300 --timeout-method thread -m gpu tests/ \
  > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in v1 m2 new; do
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || exit 1
  done
done
python tools/ab_table.py $O/ab_v1_*.json $O/ab_m2_*.json $O/ab_new_*.json
