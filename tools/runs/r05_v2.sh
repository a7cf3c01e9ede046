#!/bin/bash
# round 5 v2: GPU suite on the chain changes (one-round LayerNorm, no dead h store), same-box
# A/B against ab/noln1p.so (CHAIN_LN1P=0), chain phase stamps, then the round profile
# (rocprofv3 kernel stats + GEMM traffic PMC + the full bench line with C4 / C5 and the CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r05/v2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/v2_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --steps 20 --extra-configs="
for i in 1 2; do
  DH_LIB_PATH=ab/noln1p.so timeout -k 10 300 $B > gpurun_out/r05/v2_ab_noln1p_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 $B > gpurun_out/r05/v2_ab_new_$i.json 2>/dev/null || exit 1
  echo "ab round $i done"
done
DH_LIB_PATH=ab/chain_stamp.so timeout -k 10 200 python tools/chain_stamp.py 6 4096 > gpurun_out/r05/v2_chain_stamps.txt 2>&1 || exit 1
echo stamps-done
TAG=r05/v2 bash tools/profile_round.sh
