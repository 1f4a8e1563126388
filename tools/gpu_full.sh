R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/pt.log 2>&1 || { tail -40 $R/gpurun_out/pt.log; exit 1; }
tail -1 $R/gpurun_out/pt.log
timeout -k 10 600 python $R/bench.py > $R/gpurun_out/bfull.json 2> $R/gpurun_out/bfull.err || { tail -20 $R/gpurun_out/bfull.err; exit 1; }
python -c "
import json; d=json.load(open('$R/gpurun_out/bfull.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'sclk', d['sclk_timed_region']['sclk_mhz'], 'err', d['pose_err_vs_fp32'], 'c5', d['c5']['value'], d['roofline'])"
