#!/bin/bash
# round 5 v23: dh_energy_stats: shared histograms + batched sum loads (in-tree, 1024 threads) and the 512-thread form (ab/stats_512.so) vs HEAD (ab/stats_radix.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
(for B in 1 7 1000 4096 32768; do
  for pen in 0 1; do
    timeout -k 10 120 python tools/stats_bench.py $B 200 gpurun_out/r05/v23_new_${B}_$pen.npy $pen || exit 1
    DH_LIB_PATH=ab/stats_radix.so timeout -k 10 120 python tools/stats_bench.py $B 200 gpurun_out/r05/v23_old_${B}_$pen.npy $pen || exit 1
    DH_LIB_PATH=ab/stats_512.so timeout -k 10 120 python tools/stats_bench.py $B 200 gpurun_out/r05/v23_n512_${B}_$pen.npy $pen || exit 1
    python -c "import numpy as np; a=np.load('gpurun_out/r05/v23_old_${B}_$pen.npy'); b=np.load('gpurun_out/r05/v23_new_${B}_$pen.npy'); c=np.load('gpurun_out/r05/v23_n512_${B}_$pen.npy'); print('B=$B pen=$pen bitwise equal:', np.array_equal(a, b, equal_nan=True), np.array_equal(a, c, equal_nan=True))"
  done
done) 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05/v23_stats.txt || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "stats" tests/test_gpu_grad.py \
  > gpurun_out/r05/v23_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v23_tests.log; exit $rc
