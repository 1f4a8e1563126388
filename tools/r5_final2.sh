# round-5 end-of-work pass (final tree): the full GPU suite, smoke(), bench + profiles
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R

timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { tail -40 gpurun_out/final_tests.log; exit 1; }
tail -2 gpurun_out/final_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
bash tools/r5_profile.sh r05f full || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/bench_r05f.json')); print('bench', d['value'], d['ms_per_step'], d['sclk_timed_region']['sclk_mhz'], d['pose_err_vs_fp32_sharp_head']['fp16mx'], d['keypoint_mode']['epnp']['value'], d['keypoint_mode']['epnp']['latency_b64_us'])"
