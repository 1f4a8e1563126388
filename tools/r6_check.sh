# GPU box: the GPU suite, then the driver's bench command (compact line -> gpurun_out/r6_bench.out, full record in
# gpurun_out/bench_detail.json). Usage: bash tools/r6_check.sh [tag]
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-chk}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --detail-out gpurun_out/${T}_detail.json > gpurun_out/${T}_bench.out 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -c 1500 gpurun_out/${T}_bench.out
