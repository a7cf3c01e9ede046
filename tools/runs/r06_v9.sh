#!/bin/bash
# round 6 v9: log-psi chain phase stamps (C2, B = 4096) after the coefficient-space layer 1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_v9
DH_LIB_PATH=ab/chain_stamp.so timeout -k 10 200 python tools/chain_stamp.py 6 4096 > gpurun_out/r06_v9/chain_stamps.txt 2>&1; rc=$?
cat gpurun_out/r06_v9/chain_stamps.txt; exit $rc
