# fused channel GEMM + LayerNorm: its own test, the f32-floor / parity suites, then the bench
# (fused, and DH_LNCH=0 for the two-kernel form on the same box)
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lnch.py -s > gpurun_out/lnch_test.log 2>&1
rc=$?; grep -E "max|passed|failed|Error" gpurun_out/lnch_test.log | grep -v "^N1\|^N2\|potential" | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_floor.py tests/test_gpu_parity.py > gpurun_out/lnch_parity.log 2>&1
rc=$?; tail -3 gpurun_out/lnch_parity.log
[ $rc -eq 0 ] || exit $rc
for v in 1 0; do
DH_LNCH=$v timeout -k 10 600 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/lnch_bench_$v.json 2> gpurun_out/lnch_bench_$v.err
rc=$?; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json;d=json.load(open('gpurun_out/lnch_bench_$v.json'));print('DH_LNCH=$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us']);print({k:round(v['ms_per_step'],3) for k,v in d['kernels'].items()})"
done
