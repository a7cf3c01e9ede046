# chain kernel A/B (ab/ builds of gemm_x6.hip): P3 bias loads between the stores (base) vs
# hoisted (p3b), and the exp-form tanh (p3bexp); phase stamps of base and p3b
cd $GRAFT_REPO_ROOT
for v in base_stamp p3b_stamp; do echo "== $v"; DH_LIB_PATH=ab/$v.so timeout -k 10 120 python tools/chain_stamp.py 6 4096 2>&1 | grep -v amdgpu.ids | grep -E "==|P3|LayerNorm" || exit 1; done
for v in base p3b p3bexp base p3b p3bexp; do
  DH_LIB_PATH=ab/$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --extra-configs '' --steps 5 --warmup 2 > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/ab_$v.json'));c=d.get('components',{});print('$v', d['value'], d['ms_per_step'], c.get('mcmc_step_ms'))"
done
