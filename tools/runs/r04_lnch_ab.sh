# gemm_lnch A/B on one box: isolated launch timing of each ab/lnch_*.so variant (both modes,
# interleaved rounds), the fused-kernel test on the in-tree library, then PMC of the in-tree build.
cd $GRAFT_REPO_ROOT
V=${VARIANTS:-"lnch_base lnch_rdma lnch_rdma0"}
for r in 1 2; do
  for v in $V; do
    for m in 0 1; do
      DH_LIB_PATH=ab/$v.so timeout -k 10 60 python tools/lnch_one.py 6 4096 $m 20 | sed "s/^/$v r$r: /" || exit 1
    done
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lnch.py > gpurun_out/r04_lnch_test.log 2>&1
rc=$?; tail -3 gpurun_out/r04_lnch_test.log; [ $rc -eq 0 ] || exit $rc
echo ab-done
