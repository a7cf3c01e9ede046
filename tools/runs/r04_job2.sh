# stamps of the fused channel tail (base vs LDS-DMA residual), the KFAC suite (sparse, C2
# step, chunked statistics, two ranks), then the f32-floor margin survey
cd $GRAFT_REPO_ROOT
for v in lnch_stamp0 lnch_stamp; do for m in 0 1; do
  DH_LIB_PATH=ab/$v.so timeout -k 10 60 python tools/lnch_one.py 6 4096 $m 5 2>&1 | grep -v amdgpu.ids | sed "s/^/$v: /" || exit 1
done; done
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_0_multirank.py -k kfac tests/test_gpu_kfac.py > gpurun_out/r04_kfac.log 2>&1
tail -15 gpurun_out/r04_kfac.log | grep -E "PASS|FAIL|Error|passed|failed"
bash tools/r04_floor_survey.sh > gpurun_out/r04_survey.log 2>&1; tail -12 gpurun_out/r04_survey.log
