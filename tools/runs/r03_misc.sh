cd $GRAFT_REPO_ROOT
for v in base co; do L=$PWD/var_$v/lib.so; [ $v = base ] && L=$PWD/deephall_amd/_lib/libdeephall_amd.so; echo VAR $v; for m in 0 1; do DH_LIB_PATH=$L timeout -k 10 60 python tools/lnch_one.py 6 4096 $m 10 || exit 1; done; done
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --nspins 10 0 --flux 23 --no-cpu-baseline > gpurun_out/r03_c4.json 2>/dev/null || exit 1
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --nspins 20 0 --flux 57 --no-cpu-baseline > gpurun_out/r03_c5.json 2>/dev/null || exit 1
for f in c4 c5; do python3 -c "import json;d=json.loads(open('gpurun_out/r03_$f.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],d['walker_steps_per_sec'],d['roofline']['frac'],{n:round(v['ms_per_step'],2) for n,v in d['kernels'].items()})"; done
