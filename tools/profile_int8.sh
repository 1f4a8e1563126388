#!/bin/bash
# INT8 (C5) measurement pass on the GPU box, from the repo root: rocprofv3 --stats of a short int8 bench, separate
# FETCH_SIZE / WRITE_SIZE passes over tools/fwd_only.py (DT=int8), their summary (profiles/<tag>_*), then the int8
# bench line (cpu baseline + roofline traffic from that summary). Everything judged is copied to gpurun_out/<tag>/.
set -e
TAG=${1:-r01_int8}
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/$TAG
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv \
  -- python3 $R/bench.py --dtype int8 --steps 10 --no-cpu-baseline --no-keypoint --no-peaks) > $O/prof_$TAG.log 2>&1
echo "stats ok"
(cd /tmp && DT=int8 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$TAG -o run --output-format csv \
  -- python3 $R/tools/fwd_only.py 2) > $O/pmc_fetch_$TAG.log 2>&1
echo "fetch ok"
(cd /tmp && DT=int8 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$TAG -o run --output-format csv \
  -- python3 $R/tools/fwd_only.py 2) > $O/pmc_write_$TAG.log 2>&1
echo "write ok"
python3 $R/tools/rocprof_summary.py --tag $TAG --stats $O/prof_$TAG --fetch $O/pmc_fetch_$TAG \
  --write $O/pmc_write_$TAG --leg 10 --per-step q_stem
timeout -k 10 300 python3 $R/bench.py --dtype int8 > $O/$TAG/${TAG}_bench.json 2> $O/bench_$TAG.err
cp $R/profiles/${TAG}_* $O/$TAG/
echo "bench ok"
