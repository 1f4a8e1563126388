R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-keypoint --no-int8 --no-peaks --no-x2 --no-fp16 --no-cpu-baseline \
  > gpurun_out/r5_b2.json 2> gpurun_out/r5_b2.err || { tail -30 gpurun_out/r5_b2.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r5_b2.json')); print('headline', d['dtype'], d['value'], d['ms_per_step'])
for k, v in d['kernels'].items(): print(f\"{v['ms_per_step']*1e3:8.1f} us  {k}\")"
DT=fp16mx timeout -k 10 600 bash tools/r5_pmc.sh mx
