set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
R="--kernel-include-regex ${KREGEX:-attention_wave|det_energy} --output-format csv"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS $R -d gpurun_out/pmc/p1 -o p1 -- python tools/run_el.py 4096 1 > /dev/null
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS $R -d gpurun_out/pmc/p2 -o p2 -- python tools/run_el.py 4096 1 > /dev/null
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE $R -d gpurun_out/pmc/p3 -o p3 -- python tools/run_el.py 4096 1 > /dev/null
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE $R -d gpurun_out/pmc/p4 -o p4 -- python tools/run_el.py 4096 1 > /dev/null
echo pmc-done
