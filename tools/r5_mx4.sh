R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_mx.py "tests/test_gpu_keypoints.py::test_keypoint_mode_b64_pipeline_vs_oracle" -x -v -s --timeout 200 --timeout-method thread \
  > gpurun_out/r5_pt4.log 2>&1 || { tail -60 gpurun_out/r5_pt4.log; exit 1; }
grep -E "passed|failed|sharp head|block output|B=64" gpurun_out/r5_pt4.log | tail -12
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-keypoint --no-int8 --no-peaks --no-x2 --no-fp16 --no-cpu-baseline > gpurun_out/r5_b4.json 2> gpurun_out/r5_b4.err || { tail -30 gpurun_out/r5_b4.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r5_b4.json')); print('headline', d['value'], d['ms_per_step'])
print({k.split('<')[0][:6]+'<'+k.split('<')[1]: round(x['ms_per_step']*1e3,1) for k,x in d['kernels'].items()})"
