# chain kernel: LN scale / shift and the P2 bias staged in LDS (in-tree) vs read from global
# memory inside the epilogues (ab/noprm.so); chain / chain-attention / parity tests first
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k chain tests/test_gpu_chain_attn.py > gpurun_out/r04_prm_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04_prm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r04_prm_tests2.log 2>&1
rc=$?; tail -1 gpurun_out/r04_prm_tests2.log; [ $rc -eq 0 ] || exit $rc
for v in old new old new; do
  if [ $v = old ]; then L=ab/noprm.so; else L=""; fi
  DH_LIB_PATH=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --extra-configs= --steps 5 --warmup 2 > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/ab_$v.json'));c=d.get('components',{});k=d.get('kernels',{})
print('$v', d['value'], d['ms_per_step'], c.get('mcmc_step_ms'), c.get('local_energy_ms'), k.get('gemm',{}).get('avg_us'))"
done
