#!/bin/bash
# round 5 v30: energy assembly with the determinant weights p_k formed once (ab/det_pk.so) vs the
# in-tree build: E_L and observables bitwise at N = 6, 3, 10; full GPU suite through the variant;
# same-box bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
for n in 6 3 10; do
  timeout -k 10 200 python tools/lp_dump.py gpurun_out/r05/v30_el_old_$n.npy $n 4096 el || exit 1
  DH_LIB_PATH=ab/det_pk.so timeout -k 10 200 python tools/lp_dump.py gpurun_out/r05/v30_el_new_$n.npy $n 4096 el || exit 1
  python -c "import numpy as np; a=np.load('gpurun_out/r05/v30_el_old_$n.npy'); b=np.load('gpurun_out/r05/v30_el_new_$n.npy'); print('N=$n E_L + observables bitwise equal:', np.array_equal(a, b, equal_nan=True))"
done
DH_LIB_PATH=ab/det_pk.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v30_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v30_tests.log; [ $rc -eq 0 ] || exit $rc
B2="python bench.py --no-cpu-baseline --steps 20 --mcmc-calls 3 --extra-configs="
for i in 1 2 3; do
  timeout -k 10 300 $B2 > gpurun_out/r05/v30_ab_head_$i.json 2>/dev/null || exit 1
  DH_LIB_PATH=ab/det_pk.so timeout -k 10 300 $B2 > gpurun_out/r05/v30_ab_pk_$i.json 2>/dev/null || exit 1
  echo "round $i done"
done
