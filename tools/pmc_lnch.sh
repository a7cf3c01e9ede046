# timing + PMC counters of the fused channel GEMM + LayerNorm kernel (C2 shape), on the GPU box
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${TAG:-lnch}
D=gpurun_out/pmcl/$TAG
mkdir -p $D
timeout -k 10 60 python tools/lnch_one.py 6 4096 0 10
timeout -k 10 60 python tools/lnch_one.py 6 4096 1 10
R="--kernel-include-regex gemm_lnch --output-format csv"
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS $R -d $D -o a -- python tools/lnch_one.py 6 4096 0 2 > /dev/null
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE $R -d $D -o b -- python tools/lnch_one.py 6 4096 0 2 > /dev/null
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE $R -d $D -o f -- python tools/lnch_one.py 6 4096 0 2 > /dev/null
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE $R -d $D -o w -- python tools/lnch_one.py 6 4096 0 2 > /dev/null
python3 tools/pmc_table.py $(find $D -name "*counter_collection.csv") 2>/dev/null || true
echo pmc-done
