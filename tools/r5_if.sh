R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for n in 2 3 4 6 3; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 5 --no-keypoint --no-int8 --no-peaks --no-x2 --no-fp16 --no-cpu-baseline --sharp-frames 0 --inflight $n > gpurun_out/if_$n.json 2> gpurun_out/if_$n.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/if_$n.json')); print('inflight $n', d['value'], d['ms_per_step'], d['sclk_timed_region']['sclk_mhz'])"
done
