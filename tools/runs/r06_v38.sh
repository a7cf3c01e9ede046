#!/bin/bash
# round 6 v38: det_value / det_energy_wave phase stamps at C2 and C5 (DET_STAMP build)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v38
mkdir -p $O
DH_LIB_PATH=ab/det_stamp.so timeout -k 10 300 python tools/det_stamp.py 6 4096 > $O/stamps_c2.txt 2>&1 || exit 1
DH_LIB_PATH=ab/det_stamp.so timeout -k 10 300 python tools/det_stamp.py 20 4096 > $O/stamps_c5.txt 2>&1 || exit 1
cat $O/stamps_c2.txt $O/stamps_c5.txt | grep -v amdgpu.ids
