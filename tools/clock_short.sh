R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for a in "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 100 --warmup 10" "--steps 20 --warmup 5 --no-peaks"; do
  timeout -k 10 300 python $R/bench.py $a --no-cpu-baseline --no-int8 --no-keypoint > $R/gpurun_out/s.json 2> $R/gpurun_out/s.err || { tail -5 $R/gpurun_out/s.err; exit 1; }
  python -c "
import json; d=json.load(open('$R/gpurun_out/s.json')); print('$a', d['value'], d['ms_per_step'], d['sclk_timed_region']['sclk_mhz'], d['sclk_timed_region']['spread_mhz'])"
done
