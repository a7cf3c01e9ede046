# same-box A/B: x6m off / on (C2), then C5 with the det_energy LDS fix
cd $GRAFT_REPO_ROOT
for m in 0 1 0 1; do
  DH_X6M=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03_ab_$m.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r03_ab_$m.json').read().strip().splitlines()[-1]);k=d['kernels'];print('x6m=$m',d['value'],d['ms_per_step'],round(k['gemm_ch']['ms_per_step'],3),round(k['gemm_ch']['avg_us'],1))"
done
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --nspins 20 0 --flux 57 --no-cpu-baseline > gpurun_out/r03_c5.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/r03_c5.json').read().strip().splitlines()[-1]);k=d['kernels'];print('C5',d['value'],d['ms_per_step'],{n:round(v['ms_per_step'],2) for n,v in k.items()})"
