# round-3 closing check on one box: every -m gpu test (tightened f32-floor gate), then the
# default bench line
cd $GRAFT_REPO_ROOT
timeout -k 10 780 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03_confirm_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_confirm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03_confirm_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r03_confirm_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r03_confirm_bench.json 2> gpurun_out/r03_confirm_bench.err
rc=$?; head -c 600 gpurun_out/r03_confirm_bench.json; exit $rc
