# round-4 checkpoint: the whole GPU suite, then the round-3 permlane-reduction variant of
# gemm_lnch through the per-slot and full-chip determinism tests
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
DH_LIB_PATH=ab/perm.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lnch.py -k "slot or deterministic" > gpurun_out/r04_perm_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_perm_tests.log; [ $rc -le 1 ] || exit $rc
