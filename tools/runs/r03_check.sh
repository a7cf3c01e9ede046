# parity subset + bench twice (C2)
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_floor.py tests/test_gpu_parity.py tests/test_gpu_chain_attn.py ${EXTRA_TESTS} > gpurun_out/r03_check_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03_check_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03_check_$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r03_check_$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print(d['value'],d['ms_per_step'],{n:round(v['ms_per_step'],3) for n,v in k.items()})"
done
