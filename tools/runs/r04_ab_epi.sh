# epilogue load placement A/B on one box: ab/old.so (bias / LayerNorm-parameter loads between
# the stores in gemm_x6m, chain_x6s P3 and gemm_lnch) vs the in-tree build (loads hoisted)
cd $GRAFT_REPO_ROOT
for v in old new old new; do
  if [ $v = old ]; then L=ab/old.so; else L=""; fi
  DH_LIB_PATH=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --extra-configs '' --steps 5 --warmup 2 > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/ab_$v.json'));c=d.get('components',{});k=d.get('kernels',{})
print('$v', d['value'], d['ms_per_step'], c.get('mcmc_step_ms'), c.get('local_energy_ms'), {n:round(v['avg_us'],1) for n,v in k.items() if isinstance(v,dict) and 'avg_us' in v})"
done
