# fp16mx: parity tests, then interleaved A/B of the k_mx.hip blocks 2-7 (SPEF_OPT_MX_KERNELS 1) vs the x2 slab form (0)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_mx.py -x -v -s --timeout 150 --timeout-method thread \
  > gpurun_out/r5_pt3.log 2>&1 || { tail -60 gpurun_out/r5_pt3.log; exit 1; }
grep -E "passed|failed|sharp head|block output|max \|d|B=64" gpurun_out/r5_pt3.log | tail -12
for pass in 1 2; do
  for v in 1 0; do
    timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-keypoint --no-int8 --no-peaks --no-x2 --no-fp16 \
      --no-cpu-baseline --set-option 8=$v > gpurun_out/r5_ab_$v$pass.json 2> gpurun_out/r5_ab_$v$pass.err || { tail -30 gpurun_out/r5_ab_$v$pass.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/r5_ab_$v$pass.json')); print('mx_kernels=$v', d['value'], d['ms_per_step'])
ks=d['kernels']; print('  ', {k.split('<')[0][:6]+'<'+k.split('<')[1]: round(v['ms_per_step']*1e3,1) for k,v in ks.items() if 'irb' in k and ('s2' in k or ',24,' in k or ',32,s1' in k) or 'front' in k})"
  done
done
