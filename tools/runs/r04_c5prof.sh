# C5 kernel stats (one-GPU, 4096 walkers): which kernels the 96 ms step is made of
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_c5prof -o run -- python3 bench.py --nspins 20 0 --flux 57 --steps 2 --warmup 1 --burn-in 0 --no-cpu-baseline --no-components --extra-configs= > gpurun_out/r04_c5prof/bench.json 2>/dev/null || exit 1
python3 tools/prof_summary.py $(find gpurun_out/r04_c5prof -name "*kernel_stats.csv" | head -1) "r04 C5: rocprofv3 --kernel-trace --stats -- python bench.py --nspins 20 0 --flux 57 --steps 2 --warmup 1 --burn-in 0 (3 VMC iterations incl. warmup + the bench's instrumented pass)" > gpurun_out/r04_c5prof/kernel_stats.md
head -24 gpurun_out/r04_c5prof/kernel_stats.md
