#!/bin/bash
# In-flight batch count sweep of the bench pipeline (GPU box, repo root), interleaved twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for pass in 1 2; do
  for n in ${INFLIGHT:-2 3 4 5}; do
    timeout -k 10 300 python $R/bench.py --inflight $n --steps 200 --no-cpu-baseline --no-int8 --no-keypoint --no-peaks > $R/gpurun_out/s.json 2> $R/gpurun_out/s.err || { tail -5 $R/gpurun_out/s.err; exit 1; }
    python -c "
import json; d=json.load(open('$R/gpurun_out/s.json')); print('inflight $n', d['value'], d['ms_per_step'], d['sclk_timed_region']['sclk_mhz'])"
  done
done
