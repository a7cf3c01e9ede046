#!/bin/bash
# round 5 v26: gemm_lnch.hip compiled without the SLP vectorizer (ab/lnch_noslp.so: the layer-1
# residual form no longer spills, 44 -> 0 B per lane) vs the production build, same box: channel
# tail tests through the variant, then bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
DH_LIB_PATH=ab/lnch_noslp.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lnch.py tests/test_gpu_floor.py \
  > gpurun_out/r05/v26_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v26_tests.log; [ $rc -eq 0 ] || exit $rc
B2="python bench.py --no-cpu-baseline --steps 20 --mcmc-calls 3 --extra-configs="
for i in 1 2 3; do
  DH_LIB_PATH=ab/lnch_noslp.so timeout -k 10 300 $B2 > gpurun_out/r05/v26_ab_noslp_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B2 > gpurun_out/r05/v26_ab_prod_$i.json 2>/dev/null || exit 1
  echo "round $i done"
done
