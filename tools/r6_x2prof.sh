# GPU box: round-6 profiles of the fp16x2 (parity variant) workload: rocprofv3 --kernel-trace --stats of the bench
# leg, then separate FETCH_SIZE / WRITE_SIZE passes of the fp16x2 forward. Then (here):
#   python tools/rocprof_summary.py --tag r06_x2 --stats gpurun_out/prof_x2 --fetch gpurun_out/pmc_fetch_x2 \
#       --write gpurun_out/pmc_write_x2 --leg 10 --per-step x2_front_kernel
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_x2 -o run --output-format csv \
  -- python3 $R/bench.py --dtype fp16x2 --steps 10 --no-cpu-baseline --no-int8 --no-keypoint --no-x2 --no-fp16 --sharp-frames 0 --no-peaks) \
  > $O/prof_x2.log 2>&1
echo "stats ok"
(cd /tmp && DT=fp16x2 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_x2 -o run --output-format csv \
  -- python3 $R/tools/fwd_only.py 2) > $O/pmc_fetch_x2.log 2>&1
echo "fetch ok"
(cd /tmp && DT=fp16x2 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_x2 -o run --output-format csv \
  -- python3 $R/tools/fwd_only.py 2) > $O/pmc_write_x2.log 2>&1
echo "write ok"
