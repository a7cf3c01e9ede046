#!/bin/bash
# round 5 v15: GPU suite with det_value's register LU (DET_LU_REG=1); same-box A/B against
# ab/nolureg.so (LDS eliminate) on mcmc_step, and det_value phase stamps (ab/det_stamp.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v15_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v15_tests.log; [ $rc -eq 0 ] || exit $rc
for n in 6 3; do
  DH_LIB_PATH=ab/nolureg.so timeout -k 10 200 python tools/lp_dump.py gpurun_out/r05/v15_lp_old_$n.npy $n 4096 || exit 1
  timeout -k 10 200 python tools/lp_dump.py gpurun_out/r05/v15_lp_new_$n.npy $n 4096 || exit 1
  python -c "import numpy as np; a=np.load('gpurun_out/r05/v15_lp_old_$n.npy'); b=np.load('gpurun_out/r05/v15_lp_new_$n.npy'); print('N=$n bitwise equal:', np.array_equal(a, b, equal_nan=True), 'max diff', np.nanmax(np.abs(a-b)[np.isfinite(a-b)]))"
done
DH_LIB_PATH=ab/det_stamp.so timeout -k 10 200 python tools/det_stamp.py 6 4096 > gpurun_out/r05/v15_det_stamps.txt 2>&1 || exit 1
echo det-stamps-done
B2="python bench.py --no-cpu-baseline --steps 20 --mcmc-calls 20 --extra-configs="
for i in 1 2 3; do
  DH_LIB_PATH=ab/nolureg.so timeout -k 10 300 $B2 > gpurun_out/r05/v15_ab_nolureg_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B2 > gpurun_out/r05/v15_ab_lureg_$i.json 2>/dev/null || exit 1
  echo "round $i done"
done
