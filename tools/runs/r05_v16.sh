#!/bin/bash
# round 5 v16: GPU suite with det_value's register LU on v_readlane broadcasts and both of a
# half-wave's entries loaded together, det_energy_wave_kernel's channel rows two channels
# ahead; lp bitwise against HEAD's det.hip (ab/det_head.so), det stamps, same-box bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v16_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v16_tests.log; [ $rc -eq 0 ] || exit $rc
for n in 6 3; do
  DH_LIB_PATH=ab/det_head.so timeout -k 10 200 python tools/lp_dump.py gpurun_out/r05/v16_lp_old_$n.npy $n 4096 || exit 1
  timeout -k 10 200 python tools/lp_dump.py gpurun_out/r05/v16_lp_new_$n.npy $n 4096 || exit 1
  python -c "import numpy as np; a=np.load('gpurun_out/r05/v16_lp_old_$n.npy'); b=np.load('gpurun_out/r05/v16_lp_new_$n.npy'); print('N=$n bitwise equal:', np.array_equal(a, b, equal_nan=True))"
done
DH_LIB_PATH=ab/det_stamp.so timeout -k 10 200 python tools/det_stamp.py 6 4096 > gpurun_out/r05/v16_det_stamps.txt 2>&1 || exit 1
echo det-stamps-done
B2="python bench.py --no-cpu-baseline --steps 20 --mcmc-calls 20 --extra-configs="
for i in 1 2 3; do
  DH_LIB_PATH=ab/det_head.so timeout -k 10 300 $B2 > gpurun_out/r05/v16_ab_head_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B2 > gpurun_out/r05/v16_ab_new_$i.json 2>/dev/null || exit 1
  echo "round $i done"
done
