# fp16x2 tests on the in-tree library, then interleaved A/B of abx2/ builds
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_x2.py tests/test_gpu_keypoints.py -m gpu -x -q --timeout 90 --timeout-method thread > gpurun_out/x2t.log 2>&1; rc=$?
tail -n 3 gpurun_out/x2t.log
[ $rc -eq 0 ] || exit $rc
bash tools/x2_ab.sh "$@"
