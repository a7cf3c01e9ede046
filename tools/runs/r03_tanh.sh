# tanh_ocml exhaustive check, every -m gpu test on the new build, then a same-box A/B
# (ab/old.so = before the branch-free tanh, ab/new.so = after)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/tanh_exact > gpurun_out/r03_tanh_exact.txt 2>&1
rc=$?; cat gpurun_out/r03_tanh_exact.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 780 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03_tanh_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_tanh_tests.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=2 bash tools/ab_bench.sh || exit 1
for f in gpurun_out/ab/*.json; do
  python3 -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);k=d['kernels'];print('$f',d['value'],d['ms_per_step'],{n:round(v['ms_per_step'],3) for n,v in k.items()})"
done
