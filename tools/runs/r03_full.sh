# full GPU check: every -m gpu test, then the default bench line (one box acquisition)
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03_full_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r03_full_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err
rc=$?
tail -c 3000 gpurun_out/r03_bench.json
exit $rc
