#!/bin/bash
# round 5 v13: GPU suite with LDS-only barriers in det_energy_wave_kernel's channel loop
# and env_stream_kernel (DET_WAVE_LBAR) and attention_mfma_kernel (ATTN_MFMA_LBAR); same-box
# A/Bs: ab/nolbardet.so on the C2 and C5 lines, ab/nolbarat.so on the C4 / C5 lines, and the
# chain prologue's geometry staged in LDS (ab/noprogeo.so: the previous gemm_x6.hip) on mcmc_step,
# gemm_lnch's 3-buffer residual chunks (ab/nor3.so: LNCH_R3=0) on the local energy
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v13_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v13_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --steps 20 --mcmc-calls 3 --extra-configs=C5 --extra-steps 3"
for i in 1 2; do
  DH_LIB_PATH=ab/nolbardet.so timeout -k 10 300 $B > gpurun_out/r05/v13_ab_nolbardet_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B > gpurun_out/r05/v13_ab_lbardet_$i.json 2>/dev/null || exit 1
  echo "det round $i done"
done
B2="python bench.py --no-cpu-baseline --steps 20 --mcmc-calls 20 --extra-configs="
for i in 1 2 3; do
  DH_LIB_PATH=ab/noprogeo.so timeout -k 10 300 $B2 > gpurun_out/r05/v13_ab_noprogeo_$i.json 2>/dev/null || exit 1
  DH_LIB_PATH=ab/nor3.so timeout -k 10 300 $B2 > gpurun_out/r05/v13_ab_nor3_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B2 > gpurun_out/r05/v13_ab_progeo_$i.json 2>/dev/null || exit 1
  echo "prologue round $i done"
done
B="python bench.py --no-cpu-baseline --steps 3 --mcmc-calls 2 --extra-configs=C4,C5 --extra-steps 3"
for i in 1 2; do
  DH_LIB_PATH=ab/nolbarat.so timeout -k 10 300 $B > gpurun_out/r05/v13_ab_nolbarat_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B > gpurun_out/r05/v13_ab_lbarat_$i.json 2>/dev/null || exit 1
  echo "attn round $i done"
done
