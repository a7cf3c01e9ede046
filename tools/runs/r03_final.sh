# round-3 GPU check on one box: every -m gpu test, then the profile round (rocprofv3 stats,
# PMC traffic of the GEMM kernels, a full bench line)
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03_final_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r03_final_tests.log
[ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r03_v3} bash tools/profile_round.sh > gpurun_out/profile_round.log 2>&1
rc=$?; tail -2 gpurun_out/profile_round.log
[ $rc -eq 0 ] || exit $rc
head -c 400 gpurun_out/${TAG:-r03_v3}/bench.json
