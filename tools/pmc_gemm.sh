# PMC counters of GEMM variants on the channel-mode D x D shape (run on the GPU box).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcg
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmcg/counters.txt 2>&1 || true
for v in ${VARIANTS:-9 106}; do
  R="--kernel-include-regex gemm --output-format csv"
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS $R -d gpurun_out/pmcg/v$v -o a -- python tools/gemm_one.py $v 417792 256 256 3 > /dev/null
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE $R -d gpurun_out/pmcg/v$v -o b -- python tools/gemm_one.py $v 417792 256 256 3 > /dev/null || \
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE $R -d gpurun_out/pmcg/v$v -o b -- python tools/gemm_one.py $v 417792 256 256 3 > /dev/null
done
echo pmc-done
