# GPU box, final tree: the GPU suite, smoke(), then the driver's default bench command (every sub-record and the CPU
# baseline) -> gpurun_out/final_bench.json (+ gpurun_out/bench_detail.json)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { tail -40 gpurun_out/final_tests.log; exit 1; }
tail -2 gpurun_out/final_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 400 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -20 gpurun_out/final_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/final_bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic_over_algorithmic'], d['cpu_baseline']['value'], d['sub_records']['keypoint_mode'], d['sub_records']['epnp'])"
