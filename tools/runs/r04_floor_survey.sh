# round-4 margin survey of the f32-floor gate: every gate evaluation's
# HIP / float32-run ratios over the floor and parity suites with the enlarged fixtures, in the
# default split-bf16 mode and with DH_GEMM=f32 (exact-f32 MFMA GEMMs everywhere), and the
# per-walker diagnosis of the C2 / C5 fixtures in each mode.
cd $GRAFT_REPO_ROOT
for mode in x6all f32 x6all_unfused; do
  rm -f gpurun_out/r04_survey_$mode.jsonl
  DH_GEMM=$mode DH_FLOOR_LOG=$GRAFT_REPO_ROOT/gpurun_out/r04_survey_$mode.jsonl timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_floor.py tests/test_gpu_parity.py > gpurun_out/r04_survey_$mode.log 2>&1
  tail -3 gpurun_out/r04_survey_$mode.log
  for t in C2 C5 C2_pole MIX_pole; do
    DH_GEMM=$mode timeout -k 10 200 python -u tools/diag_floor.py $t > gpurun_out/r04_diag_${mode}_$t.txt 2>&1 || exit 1
  done
done
echo survey-done
