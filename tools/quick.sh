#!/bin/bash
# Quick GPU check: parity tests + short bench (no CPU baseline). Usage: bash tools/quick.sh [pytest -k expr]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -m pytest $R/tests -m gpu -q -x -k "$K" > $R/gpurun_out/pt.log 2>&1 || { tail -30 $R/gpurun_out/pt.log; exit 1; }
else
  timeout -k 10 600 python -m pytest $R/tests -m gpu -q -x > $R/gpurun_out/pt.log 2>&1 || { tail -30 $R/gpurun_out/pt.log; exit 1; }
fi
tail -1 $R/gpurun_out/pt.log
timeout -k 10 300 python $R/bench.py --no-cpu-baseline > $R/gpurun_out/bq.json 2> $R/gpurun_out/bq.err
python - <<'PY'
import json, os
d = json.load(open(os.path.join(os.environ.get('GRAFT_REPO_ROOT', '.'), 'gpurun_out', 'bq.json')))
print('value', d['value'], 'ms', d['ms_per_step'])
for k, v in list(d['kernels'].items())[:16]:
    print(f"{v['ms_per_step']*1000:8.1f} us  x{v['launches_per_step']:.0f}  {k}")
PY
