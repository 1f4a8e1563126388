#!/bin/bash
# GPU check of a kernel change: the GPU tests, then an interleaved A/B against abbase/base.so, then a quick bench.
# usage (on the box): bash tools/gpu_ab.sh [pytest -k expr] [ab rounds]
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
K=${1:-}
N=${2:-2}
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} \
  > $R/gpurun_out/pt.log 2>&1 || { tail -40 $R/gpurun_out/pt.log; exit 1; }
tail -2 $R/gpurun_out/pt.log
timeout -k 10 400 python -u $R/tools/ab.py $R/${BASE:-abbase/base.so} $N > $R/gpurun_out/ab.log 2>&1 || { tail -20 $R/gpurun_out/ab.log; exit 1; }
head -30 $R/gpurun_out/ab.log
timeout -k 10 300 python $R/bench.py --no-cpu-baseline > $R/gpurun_out/bq.json 2> $R/gpurun_out/bq.err || { tail -20 $R/gpurun_out/bq.err; exit 1; }
python -c "
import json; d=json.load(open('$R/gpurun_out/bq.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'sclk', d.get('sclk_timed_region',{}).get('sclk_mhz'), 'err', d.get('pose_err_vs_fp32'))"
