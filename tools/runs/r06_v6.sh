#!/bin/bash
# round 6 v6: gemm_lnch MODE 2 phase stamps (C2, B = 4096)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_v6
DH_LIB_PATH=ab/stamp2.so timeout -k 10 200 python tools/lnch_mode2_stamp.py 4096 > gpurun_out/r06_v6/stamps.txt 2>&1; rc=$?
cat gpurun_out/r06_v6/stamps.txt; exit $rc
