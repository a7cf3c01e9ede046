# round-4 closing run: the GPU suite, smoke(), then tools/profile_round.sh (kernel stats, GEMM
# traffic by PMC, the full bench line with the CPU baseline and the C4 / C5 lines)
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04_final_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_final_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r04_final_smoke.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r04_v4} bash tools/profile_round.sh
