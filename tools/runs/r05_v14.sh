#!/bin/bash
# round 5 v14: phase stamps of det_value / det_energy_wave (ab/det_stamp.so) and of the chain
# kernel (ab/chain_stamp.so) on the current code
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
DH_LIB_PATH=ab/det_stamp.so timeout -k 10 200 python tools/det_stamp.py 6 4096 > gpurun_out/r05/v14_det_stamps.txt 2>&1 || exit 1
echo det-stamps-done
DH_LIB_PATH=ab/chain_stamp.so timeout -k 10 200 python tools/chain_stamp.py 6 4096 > gpurun_out/r05/v14_chain_stamps.txt 2>&1 || exit 1
echo chain-stamps-done
