# gemm_lnch statistics reduction: LDS-only (default) vs permlane32/16 swaps (LNCH_PERMLANE=1):
# per-tile stamps and isolated launch time, both modes, alternating
cd $GRAFT_REPO_ROOT
for r in 1 2; do for v in lnst perm_st; do for m in 0 1; do
  echo "== $v mode $m"; DH_LIB_PATH=ab/$v.so timeout -k 10 60 python tools/lnch_one.py 6 4096 $m 20 2>&1 | grep -E "gemm_lnch|reduce|LN \+" || exit 1
done; done; done
DH_LIB_PATH=ab/perm.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lnch.py > gpurun_out/r04_perm_lnch.log 2>&1
rc=$?; tail -1 gpurun_out/r04_perm_lnch.log; [ $rc -le 1 ] || exit $rc
