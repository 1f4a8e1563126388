# final-tree check on the GPU box: the GPU suite, smoke(), one default bench line
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/verify_tests.log 2>&1 || { tail -40 gpurun_out/verify_tests.log; exit 1; }
tail -2 gpurun_out/verify_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/verify_bench.json 2> gpurun_out/verify_bench.err || { tail -20 gpurun_out/verify_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/verify_bench.json')); print('bench', d['value'], d['ms_per_step'], d['sclk_timed_region']['sclk_mhz'], d['roofline']['traffic'])"
