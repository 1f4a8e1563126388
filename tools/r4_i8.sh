# int8 role-split late blocks: bit-exact tests on the in-tree library, then int8 A/B of abx2/ builds
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_int8.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/i8t.log 2>&1; rc=$?
tail -n 5 gpurun_out/i8t.log
[ $rc -eq 0 ] || exit $rc
bash tools/i8_ab.sh "$@"
