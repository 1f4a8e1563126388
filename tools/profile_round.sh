#!/bin/bash
# One GPU-box pass producing the round's measurement artefacts (run from the repo root on the box):
#   gpurun_out/bench_<tag>.json    bench.py line (N=1, with cpu_baseline and pose error)
#   gpurun_out/prof_<tag>/         rocprofv3 --kernel-trace --stats of a short bench run
#   gpurun_out/pmc_fetch_<tag>/, pmc_write_<tag>/   separate FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md)
# then: python tools/rocprof_summary.py --tag <tag> --stats gpurun_out/prof_<tag> \
#         --fetch gpurun_out/pmc_fetch_<tag> --write gpurun_out/pmc_write_<tag> --leg 10 --per-step front_vp_kernel
# (the traced run is the fp16 C3 workload alone -- no int8 / fp16x2 / sharp-head / keypoint legs, whose smaller front kernels would land in
# the last dispatches -- with bench.py's own settle phase, so the traced leg runs at the clock the bench line sees;
# the leg = the last 10 steps' dispatches of every kernel, counted against the once-per-step front kernel)
set -e
TAG=${1:-r01}
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python3 $R/bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err
echo "bench ok"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv \
  -- python3 $R/bench.py --steps 10 --no-cpu-baseline --no-int8 --no-keypoint --no-x2 --sharp-frames 0 --no-peaks) \
  > $O/prof_$TAG.log 2>&1
echo "stats ok"
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$TAG -o run --output-format csv \
  -- python3 $R/tools/fwd_only.py 2) > $O/pmc_fetch_$TAG.log 2>&1
echo "fetch ok"
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$TAG -o run --output-format csv \
  -- python3 $R/tools/fwd_only.py 2) > $O/pmc_write_$TAG.log 2>&1
echo "write ok"
