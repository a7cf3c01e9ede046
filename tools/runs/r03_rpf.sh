# MODE 0 residual-line touch (ab/rpf.so) against the current build (ab/new2.so): isolated
# launches, the fused-kernel + parity tests on rpf, a same-box bench A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for v in new2 rpf new2 rpf; do
  DH_LIB_PATH=ab/$v.so timeout -k 10 120 python tools/lnch_one.py 6 4096 0 100 > gpurun_out/ab/rpf_${v}.txt 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/ab/rpf_${v}.txt)"
done
DH_LIB_PATH=ab/rpf.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lnch.py tests/test_gpu_floor.py tests/test_gpu_parity.py > gpurun_out/r03_rpf_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03_rpf_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab/*.json
cp ab/new2.so ab/old.so; cp ab/rpf.so ab/new.so
ROUNDS=2 bash tools/ab_bench.sh || exit 1
for f in gpurun_out/ab/*.json; do
  python3 -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);k=d['kernels'];print('$f',d['value'],d['ms_per_step'],{n:round(v['ms_per_step'],3) for n,v in k.items() if n in ('gemm_ch','gemm','attention_ch')})"
done
