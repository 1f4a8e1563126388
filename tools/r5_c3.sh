R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_mx.py tests/test_gpu_x2.py > gpurun_out/c3_tests.log 2>&1 || { tail -40 gpurun_out/c3_tests.log; exit 1; }
tail -2 gpurun_out/c3_tests.log
bash tools/r5_var.sh "cur al2" 2
