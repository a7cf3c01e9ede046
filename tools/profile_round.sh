# Round profile on the GPU box: rocprofv3 kernel stats of the bench, HBM traffic of the
# GEMM kernels (separate FETCH_SIZE / WRITE_SIZE passes, MI355X_MICROARCH.md HBM section)
# and a full bench line.  Usage: TAG=r01_v9 bash tools/profile_round.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${TAG:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="bench.py --steps 5 --warmup 1 --burn-in 0 --no-cpu-baseline --no-components --extra-configs="
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/bench_under_rocprof.json
R="--kernel-include-regex (gemm|chain) --output-format csv"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE $R -d $OUT/fetch -o f -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-components --no-kernel-events --extra-configs= > /dev/null
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE $R -d $OUT/write -o w -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-components --no-kernel-events --extra-configs= > /dev/null
python3 tools/pmc_traffic.py $(find $OUT/fetch -name "*counter_collection.csv") $(find $OUT/write -name "*counter_collection.csv") > $OUT/gemm_traffic.json
R2="--kernel-include-regex (gemm|chain) --output-format csv"
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE $R2 -d $OUT/mfma -o m -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-components --no-kernel-events --extra-configs= > /dev/null
python3 tools/pmc_mfma.py $TAG $(find $OUT/mfma -name "*counter_collection.csv") > $OUT/mfma_pmc.json
timeout -k 10 400 python3 bench.py > $OUT/bench.json
python3 tools/prof_summary.py $(find $OUT/trace -name "*kernel_stats.csv") "$TAG: rocprofv3 --kernel-trace --stats -- python bench.py --steps 5 --warmup 1 --burn-in 0 (C2, B=4096; every dispatch belongs to a full VMC step, the same mix as the bench instrumented region)" > $OUT/kernel_stats.md
echo profile-done
