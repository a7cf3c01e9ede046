#!/bin/bash
# round 5 v28: det_energy_wave_kernel's envelope leaves with integer powers by squaring
# (ab/det_sq.so, DET_WAVE_SQ=1) vs powf (in-tree): full GPU suite through the variant (floor
# gates), det stamps of both, same-box bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
DH_LIB_PATH=ab/det_sq.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v28_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v28_tests.log; [ $rc -eq 0 ] || exit $rc
DH_LIB_PATH=ab/det_stamp_sq.so timeout -k 10 200 python tools/det_stamp.py 6 4096 > gpurun_out/r05/v28_det_stamps_sq.txt 2>&1 || exit 1
DH_LIB_PATH=ab/det_stamp_powf.so timeout -k 10 200 python tools/det_stamp.py 6 4096 > gpurun_out/r05/v28_det_stamps_powf.txt 2>&1 || exit 1
echo stamps-done
B2="python bench.py --no-cpu-baseline --steps 20 --mcmc-calls 3 --extra-configs="
for i in 1 2 3; do
  timeout -k 10 300 $B2 > gpurun_out/r05/v28_ab_powf_$i.json 2>/dev/null || exit 1
  DH_LIB_PATH=ab/det_sq.so timeout -k 10 300 $B2 > gpurun_out/r05/v28_ab_sq_$i.json 2>/dev/null || exit 1
  echo "round $i done"
done
