cd $GRAFT_REPO_ROOT
for v in chain_stamp chain_stamp_exp; do echo "== $v"; DH_LIB_PATH=ab/$v.so timeout -k 10 120 python tools/chain_stamp.py 6 4096 2>&1 | grep -v amdgpu.ids | grep -E "==|LayerNorm|tanh|planes" || exit 1; done
for v in "" ab/tanh_exp.so "" ab/tanh_exp.so; do
  DH_LIB_PATH=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --extra-configs '' > gpurun_out/ab.json 2>/dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/ab.json'));c=d.get('components',{});print('lib=$v', d['value'], d['ms_per_step'], c.get('mcmc_step_ms'))"
done
