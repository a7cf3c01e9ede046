# layer-1 attention in the chain prologue: 2 (default) vs 4 walkers per attn_val_core call
# (ant4), and the first weight fragments requested after the attention (ant4apf)
cd $GRAFT_REPO_ROOT
DH_LIB_PATH=ab/ant4.so timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread -m gpu tests/test_gpu_chain_attn.py > gpurun_out/r04_ant4_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04_ant4_tests.log; [ $rc -eq 0 ] || exit $rc
for v in base_stamp ant4_stamp; do echo "== $v"; DH_LIB_PATH=ab/$v.so timeout -k 10 120 python tools/chain_stamp.py 6 4096 2>&1 | grep -v amdgpu.ids | grep -E "== layer 1|prologue" || exit 1; done
for v in new ant4 ant4apf new ant4 ant4apf; do
  if [ $v = new ]; then L=""; else L=ab/$v.so; fi
  DH_LIB_PATH=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --extra-configs '' --steps 5 --warmup 2 > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/ab_$v.json'));c=d.get('components',{})
print('$v', d['value'], d['ms_per_step'], c.get('mcmc_step_ms'), c.get('local_energy_ms'))"
done
