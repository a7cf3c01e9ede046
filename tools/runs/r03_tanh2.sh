# gemm_lnch with the branch-free tanh + epilogue indices from mbcnt (ab/new2.so = the in-tree
# build) against the round-3 HEAD build (ab/old.so): isolated launches, the fused-kernel and
# parity tests, then a same-box bench A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for v in old new2 old new2; do
  for m in 0 1; do
    DH_LIB_PATH=ab/$v.so timeout -k 10 120 python tools/lnch_one.py 6 4096 $m 100 > gpurun_out/ab/lnch_${v}_$m.txt 2>&1 || exit 1
    echo "$v $(cat gpurun_out/ab/lnch_${v}_$m.txt | tail -1)"
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lnch.py tests/test_gpu_floor.py tests/test_gpu_parity.py tests/test_gpu_kernels.py > gpurun_out/r03_tanh2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03_tanh2_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab/*.json
mv ab/new2.so ab/new.so
ROUNDS=3 bash tools/ab_bench.sh || exit 1
mv ab/new.so ab/new2.so
for f in gpurun_out/ab/*.json; do
  python3 -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);k=d['kernels'];print('$f',d['value'],d['ms_per_step'],{n:round(v['ms_per_step'],3) for n,v in k.items() if n in ('gemm_ch','gemm','attention_ch')})"
done
