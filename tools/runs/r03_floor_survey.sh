# margins of the f32-floor gate: every evaluation's HIP / float32-run error ratios (median,
# p90, max) over the floor and parity suites, written to gpurun_out/floor_survey.jsonl
cd $GRAFT_REPO_ROOT
rm -f gpurun_out/floor_survey.jsonl
DH_FLOOR_LOG=$GRAFT_REPO_ROOT/gpurun_out/floor_survey.jsonl timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_floor.py tests/test_gpu_parity.py tests/test_gpu_lnch.py > gpurun_out/floor_survey_tests.log 2>&1
rc=$?; tail -2 gpurun_out/floor_survey_tests.log
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/floor_survey.jsonl')]
print(len(rows),'gate evaluations')
for k in ('med','p90','max'):
    rr=sorted(rows,key=lambda r:-r[k])[:5]
    print(k,[ (round(r[k],2), r['test'].split('::')[-1][:60], r['emax']<=r['floor_abs']) for r in rr])
PY
exit $rc
