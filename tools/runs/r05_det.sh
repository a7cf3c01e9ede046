#!/bin/bash
# round 5: det_energy_wave_kernel parity (floor + parity suites) and a same-box A/B
# (DH_DET_V2=0: det_energy_kernel, 1: the wave form), C2 bench without C4/C5 extras.
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_floor.py tests/test_gpu_parity.py -m gpu > gpurun_out/r05/det_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05/det_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    DH_DET_V2=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --extra-configs "" \
      > gpurun_out/r05/det_ab_v${v}_$i.json 2> gpurun_out/r05/det_ab_v${v}_$i.err || exit 1
    echo "v$v $i done"
  done
done
