cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_floor.py tests/test_gpu_parity.py tests/test_gpu_laughlin.py > gpurun_out/r03_det_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03_det_tests.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1; do
  DH_DET_WAVE=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03_det_$m.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r03_det_$m.json').read().strip().splitlines()[-1]);k=d['kernels'];print('wave=$m',d['value'],d['ms_per_step'],round(k['det_energy']['ms_per_step'],3))"
done
for m in 0 1; do
  DH_DET_WAVE=$m timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --nspins 20 0 --flux 57 --no-cpu-baseline > gpurun_out/r03_det_c5_$m.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r03_det_c5_$m.json').read().strip().splitlines()[-1]);k=d['kernels'];print('C5 wave=$m',d['value'],d['ms_per_step'],round(k['det_energy']['ms_per_step'],3))"
done
