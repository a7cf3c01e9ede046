# rocprofv3 kernel stats of one bench config: TAG=... ARGS="--nspins 20 0 --flux 57" bash tools/r03_prof_cfg.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${TAG:-cfg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps ${STEPS:-3} --warmup 1 --burn-in 0 --no-cpu-baseline --no-components $ARGS > $OUT/bench_under_rocprof.json || exit 1
python3 tools/prof_summary.py $(find $OUT/trace -name "*kernel_stats.csv") "$TAG: rocprofv3 --kernel-trace --stats -- python bench.py --steps ${STEPS:-3} --warmup 1 --burn-in 0 $ARGS" > $OUT/kernel_stats.md
head -30 $OUT/kernel_stats.md
