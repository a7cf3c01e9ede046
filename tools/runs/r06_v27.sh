#!/bin/bash
# round 6 v27: layer1_ch (fused) against the two-kernel layer 1 (x6all_unfused) at C4 / C5
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_v27
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lnch.py -k "C4 or C5" > $O/tests.log 2>&1
rc=$?; grep -E "C4|C5|passed|failed|Error" $O/tests.log | tail -30; exit $rc
