# PMC counters of GEMM variants on one hot-path shape (run on the GPU box).
# VARIANTS="106 200" SHAPE="417792 256 256" TAG=el_d bash tools/pmc_gemm.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SHAPE=${SHAPE:-"417792 256 256"}
TAG=${TAG:-el_d}
for v in ${VARIANTS:-9 106}; do
  D=gpurun_out/pmcg/$TAG/v$v
  mkdir -p $D
  R="--kernel-include-regex gemm --output-format csv"
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS $R -d $D -o a -- python tools/gemm_one.py $v $SHAPE 3 > /dev/null
  timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE $R -d $D -o b -- python tools/gemm_one.py $v $SHAPE 3 > /dev/null
done
echo pmc-done
