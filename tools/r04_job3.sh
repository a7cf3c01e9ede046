# the cos-theta gauge (det.hip env_gauge) through the f32-floor survey and the parity suite;
# the fixed KFAC tests; the two-tiles-per-CU fused tail (DH_LNCH=2, gemm_lnch2.hip) through its
# tests and timing at N = 6, 10, 20; bench lines with both forms
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lnch.py -k slot > gpurun_out/r04_slot_test.log 2>&1
rc=$?; tail -3 gpurun_out/r04_slot_test.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1; do
  DH_LNCH=2 timeout -k 10 60 python tools/lnch_one.py 6 4096 $m 20 2>&1 | grep -v amdgpu.ids || exit 1
  DH_LNCH=1 timeout -k 10 60 python tools/lnch_one.py 6 4096 $m 20 2>&1 | grep -v amdgpu.ids || exit 1
  DH_LNCH=2 timeout -k 10 60 python tools/lnch_one.py 10 4096 $m 10 2>&1 | grep -v amdgpu.ids || exit 1
  DH_LNCH=2 timeout -k 10 60 python tools/lnch_one.py 20 4096 $m 5 2>&1 | grep -v amdgpu.ids || exit 1
done
DH_LNCH=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lnch.py > gpurun_out/r04_lnch2_test.log 2>&1
rc=$?; tail -3 gpurun_out/r04_lnch2_test.log; [ $rc -eq 0 ] || exit $rc
for f in 2 1; do
  DH_LNCH=$f timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench_lnch$f.json 2> gpurun_out/r04_bench_lnch$f.err || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/r04_bench_lnch$f.json'));print('DH_LNCH=$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], {k:(v['value'],v['ms_per_step']) for k,v in d.get('configs_1gpu',{}).items()})"
done
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_0_multirank.py -k kfac tests/test_gpu_kfac.py > gpurun_out/r04_kfac2.log 2>&1
tail -15 gpurun_out/r04_kfac2.log | grep -E "PASS|FAIL|Error|passed|failed"
bash tools/r04_floor_survey.sh > gpurun_out/r04_survey.log 2>&1; tail -12 gpurun_out/r04_survey.log
