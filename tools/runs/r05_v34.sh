#!/bin/bash
# round 5 v34: round profile of the final tree (kernel stats, GEMM PMC traffic, full default bench line)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05_v34 bash tools/profile_round.sh
