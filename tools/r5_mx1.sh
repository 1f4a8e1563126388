# round 5: fp16mx first GPU pass -- new/changed x2 kernels' parity tests, then a short headline bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_x2.py tests/test_gpu_pipeline.py -x -v -s \
  --timeout 150 --timeout-method thread > gpurun_out/r5_pt1.log 2>&1 || { tail -60 gpurun_out/r5_pt1.log; exit 1; }
grep -E "passed|failed|sharp head|block output|max \|d|B=64" gpurun_out/r5_pt1.log | tail -30
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-keypoint --no-int8 --no-peaks > gpurun_out/r5_b1.json \
  2> gpurun_out/r5_b1.err || { tail -30 gpurun_out/r5_b1.err; exit 1; }
python - <<'PY'
import json
d = json.load(open('gpurun_out/r5_b1.json'))
print('headline', d['dtype'], d['value'], d['ms_per_step'], d.get('sclk_timed_region', {}).get('sclk_mhz'))
print('pose', d.get('pose_err_vs_fp32'), 'sharp', d.get('pose_err_vs_fp32_sharp_head'))
for k in ('fp16', 'fp16x2'):
    if k in d: print(k, d[k]['value'], d[k]['ms_per_step'])
for k, v in d['kernels'].items(): print(f"{v['ms_per_step']*1e3:8.1f} us  {k}")
if 'fp16x2' in d:
    for k, v in d['fp16x2']['kernels'].items(): print(f"x2 {v['ms_per_step']*1e3:8.1f} us  {k}")
PY
