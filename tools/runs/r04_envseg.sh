# env_contract_kernel with segment DMA (SEG, default where usable) vs the one-dword pieces
# (DH_ENV_SEG0=1): floor / parity suites (C5 fixtures run the precontracted path), then C5 A/B
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_floor.py tests/test_gpu_parity.py > gpurun_out/r04_envseg_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04_envseg_tests.log; [ $rc -eq 0 ] || exit $rc
for v in old new old new; do
  if [ $v = old ]; then E="DH_ENV_SEG0=1"; else E="DH_X=0"; fi
  env $E timeout -k 10 300 python -u bench.py --nspins 20 0 --flux 57 --steps 3 --warmup 2 --no-cpu-baseline --extra-configs= > gpurun_out/ab_c5_$v.json 2>/dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/ab_c5_$v.json'));k=d.get('kernels',{})
print('$v', d['value'], d['ms_per_step'], {n:round(v['ms_per_step'],2) for n,v in k.items() if isinstance(v,dict) and 'ms_per_step' in v})"
done
