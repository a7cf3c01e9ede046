#!/bin/bash
# round 5 v12: GPU suite with LDS-only barriers in the chain kernel (CHAIN_LBAR) and gemm_lnch
# (LNCH_LBAR); same-box A/Bs: ab/nolbar.so (chain __syncthreads), ab/nolbarln.so (gemm_lnch
# __syncthreads) on the C2 line, det_energy_wave_kernel's occupancy (ab/detw3.so, ab/detw4.so);
# chain stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v12_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v12_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --steps 20 --mcmc-calls 20 --extra-configs="
for i in 1 2 3; do
  DH_LIB_PATH=ab/nolbar.so timeout -k 10 300 $B > gpurun_out/r05/v12_ab_nolbar_$i.json 2>/dev/null || exit 1
  DH_LIB_PATH=ab/nolbarln.so timeout -k 10 300 $B > gpurun_out/r05/v12_ab_nolbarln_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B > gpurun_out/r05/v12_ab_lbar_$i.json 2>/dev/null || exit 1
  echo "ab round $i done"
done
for i in 1 2; do
  DH_LIB_PATH=ab/detw3.so timeout -k 10 300 $B > gpurun_out/r05/v12_ab_detw3_$i.json 2>/dev/null || exit 1
  DH_LIB_PATH=ab/detw4.so timeout -k 10 300 $B > gpurun_out/r05/v12_ab_detw4_$i.json 2>/dev/null || exit 1
  echo "det round $i done"
done
DH_LIB_PATH=ab/chain_stamp.so timeout -k 10 200 python tools/chain_stamp.py 6 4096 > gpurun_out/r05/v12_chain_stamps.txt 2>&1 || exit 1
echo stamps-done
