#!/bin/bash
# round 5 v1: the full GPU suite on the new kernels (wave-per-walker det_energy, feature-space
# layer-1 attention), then a same-box A/B: ab/r04.so (round-4 HEAD) against this tree with
# each new form switched off in turn (DH_DET_V2=0, DH_ATTN_FEAT=0) and all on.  C2 only.
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05/v1_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --steps 20 --extra-configs="
for i in 1 2; do
  DH_LIB_PATH=ab/r04.so timeout -k 10 300 $B > gpurun_out/r05/v1_ab_r04_$i.json 2>/dev/null || exit 1
  DH_DET_V2=0 timeout -k 10 300 $B > gpurun_out/r05/v1_ab_nodet_$i.json 2>/dev/null || exit 1
  DH_ATTN_FEAT=0 timeout -k 10 300 $B > gpurun_out/r05/v1_ab_nofeat_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B > gpurun_out/r05/v1_ab_new_$i.json 2>/dev/null || exit 1
  echo "round $i done"
done
