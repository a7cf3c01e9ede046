# PMC of the fused channel GEMM + LayerNorm kernel, BOTH modes (C2 shape, B = 4096), plus
# isolated launch timing.  Usage: TAG=r04_base bash tools/r04_lnch_pmc.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${TAG:-lnch}
D=gpurun_out/pmcl/$TAG
mkdir -p $D
N=${LNCH_N:-6}
for m in 0 1; do
  timeout -k 10 60 python tools/lnch_one.py $N 4096 $m 20
done
R="--kernel-include-regex gemm_lnch --output-format csv"
for m in 0 1; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS $R -d $D/m$m -o a -- python tools/lnch_one.py $N 4096 $m 2 > /dev/null
  timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE $R -d $D/m$m -o b -- python tools/lnch_one.py $N 4096 $m 2 > /dev/null
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE $R -d $D/m$m -o f -- python tools/lnch_one.py $N 4096 $m 2 > /dev/null
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE $R -d $D/m$m -o w -- python tools/lnch_one.py $N 4096 $m 2 > /dev/null
  echo "== mode $m"
  python3 tools/pmc_table.py $(find $D/m$m -name "*counter_collection.csv")
done
echo pmc-done
