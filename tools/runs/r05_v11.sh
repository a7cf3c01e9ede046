#!/bin/bash
# round 5 v11: det_energy_wave_kernel occupancy A/B on the C2 line: the compiler's choice
# (216 VGPRs, 2 waves / SIMD) vs amdgpu_waves_per_eu 3 (168 VGPRs, 96 B scratch) and 4 (128
# VGPRs, 256 B scratch): ab/detw3.so, ab/detw4.so
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
B="python bench.py --no-cpu-baseline --steps 20 --mcmc-calls 3 --extra-configs="
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/r05/v11_ab_w2_$i.json 2>/dev/null || exit 1
  DH_LIB_PATH=ab/detw3.so timeout -k 10 300 $B > gpurun_out/r05/v11_ab_w3_$i.json 2>/dev/null || exit 1
  DH_LIB_PATH=ab/detw4.so timeout -k 10 300 $B > gpurun_out/r05/v11_ab_w4_$i.json 2>/dev/null || exit 1
  echo "ab round $i done"
done
