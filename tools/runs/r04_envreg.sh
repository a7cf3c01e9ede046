# env_contract segment form: tangent-row envelope factors held in registers (in-tree) vs read from LDS per row (ab/noreg.so)
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_floor.py -k C5 tests/test_gpu_parity.py -k "C5 or repeatable" > gpurun_out/r04_envring_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04_envring_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 500 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_floor.py > gpurun_out/r04_envring_floor.log 2>&1
rc=$?; tail -1 gpurun_out/r04_envring_floor.log; [ $rc -eq 0 ] || exit $rc
for v in old new old new; do
  if [ $v = old ]; then L=ab/noreg.so; else L=""; fi
  DH_LIB_PATH=$L timeout -k 10 300 python -u bench.py --nspins 20 0 --flux 57 --steps 3 --warmup 2 --no-cpu-baseline --extra-configs= > gpurun_out/ab_c5_$v.json 2>/dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/ab_c5_$v.json'));k=d.get('kernels',{})
print('$v', d['value'], d['ms_per_step'], k.get('det_energy',{}).get('ms_per_step'))"
done
