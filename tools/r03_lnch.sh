# fused channel GEMM + LayerNorm: its own test, the f32-floor / parity suites, then the bench
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lnch.py -s > gpurun_out/lnch_test.log 2>&1
rc=$?; grep -E "max|passed|failed|Error" gpurun_out/lnch_test.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_floor.py tests/test_gpu_parity.py > gpurun_out/lnch_parity.log 2>&1
rc=$?; tail -3 gpurun_out/lnch_parity.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/lnch_bench.json 2> gpurun_out/lnch_bench.err
rc=$?; head -c 700 gpurun_out/lnch_bench.json; echo; python3 -c "
import json;d=json.load(open('gpurun_out/lnch_bench.json'));print(json.dumps(d['kernels']))"
exit $rc
