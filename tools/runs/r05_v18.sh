#!/bin/bash
# round 5 v18: det_value_kernel<MGV> (N = 10, 20) with the next row's F loads in flight while a row
# is contracted.  GPU suite; log psi bitwise against HEAD's det.hip (ab/det_head.so) at N = 20, 10;
# C5 det stamps; same-box C4 / C5 bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v18_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v18_tests.log; [ $rc -eq 0 ] || exit $rc
for n in 20 10; do
  DH_LIB_PATH=ab/det_head.so timeout -k 10 200 python tools/lp_dump.py gpurun_out/r05/v18_lp_old_$n.npy $n 4096 || exit 1
  timeout -k 10 200 python tools/lp_dump.py gpurun_out/r05/v18_lp_new_$n.npy $n 4096 || exit 1
  python -c "import numpy as np; a=np.load('gpurun_out/r05/v18_lp_old_$n.npy'); b=np.load('gpurun_out/r05/v18_lp_new_$n.npy'); print('N=$n bitwise equal:', np.array_equal(a, b, equal_nan=True))"
done
DH_LIB_PATH=ab/det_stamp.so timeout -k 10 200 python tools/det_stamp.py 20 4096 > gpurun_out/r05/v18_det_stamps_c5.txt 2>&1 || exit 1
echo det-stamps-done
B="python bench.py --no-cpu-baseline --steps 3 --mcmc-calls 2 --extra-configs=C4,C5 --extra-steps 3"
for i in 1 2; do
  DH_LIB_PATH=ab/det_head.so timeout -k 10 400 $B > gpurun_out/r05/v18_ab_head_$i.json 2>/dev/null || exit 1
  timeout -k 10 400 $B > gpurun_out/r05/v18_ab_new_$i.json 2>/dev/null || exit 1
  echo "round $i done"
done
