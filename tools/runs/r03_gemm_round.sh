# Round-3 GEMM iteration on the GPU box: variant tests, bench, PMC (one box acquisition)
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "x6_variants" > gpurun_out/r03_x6m_test.log 2>&1
timeout -k 10 300 python -u tools/gemm_bench.py ${BENCH_VARIANTS:-256 280 284 281 285} > gpurun_out/r03_x6m_bench.log 2>&1
VARIANTS="${PMC_VARIANTS:-256 280 284}" SHAPE="417792 768 256" TAG=el_qkv timeout -k 10 400 bash tools/pmc_gemm.sh > gpurun_out/r03_pmc.log 2>&1
