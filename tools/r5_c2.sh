# in-tree build: full GPU suite, EPnP timing, interleaved bench against the alias + deinterleave variant
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 100 python tools/epnp_time.py || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c2_tests.log 2>&1 || { tail -40 gpurun_out/c2_tests.log; exit 1; }
tail -3 gpurun_out/c2_tests.log
bash tools/r5_var.sh "cur al1 pk1d0" 2
