#!/bin/bash
# round 5 v9: the round profile of the current code (rocprofv3 kernel stats, GEMM PMC traffic,
# the full bench line with C4 / C5 and the CPU baseline) and the chain kernel's phase stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
DH_LIB_PATH=ab/chain_stamp.so timeout -k 10 200 python tools/chain_stamp.py 6 4096 > gpurun_out/r05/v9_chain_stamps.txt 2>&1 || exit 1
echo stamps-done
TAG=r05/v9 bash tools/profile_round.sh
