#!/bin/bash
# rocprofv3 kernel statistics of the precision variants (GPU box, repo root): the keypoint leg (fp32, fp16x2, fp16 at
# 240x384, B=64: forward + sigmoid + EPnP) and the fp16x2 URSONet forward at 512^2, B=64 (tools/variant_time.py), plus
# separate FETCH_SIZE / WRITE_SIZE passes over the fp16x2 forward (tools/fwd_only.py). Summaries:
#   python tools/rocprof_summary.py --tag r04_<name> --stats gpurun_out/prof_r04_<name> [--fetch .. --write ..]
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for spec in "fp32 keypoints kp_fp32" "fp16x2 keypoints kp_x2" "fp16 keypoints kp_fp16" "fp16x2 ursonet x2"; do
  set -- $spec
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_r04_$3 -o run --output-format csv \
    -- python3 $R/tools/variant_time.py $1 $2 64) > $O/prof_r04_$3.log 2>&1
  echo "stats $3 ok"
done
(cd /tmp && DT=fp16x2 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_r04_x2 -o run --output-format csv \
  -- python3 $R/tools/fwd_only.py 2) > $O/pmc_fetch_r04_x2.log 2>&1
echo "fetch ok"
(cd /tmp && DT=fp16x2 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_r04_x2 -o run --output-format csv \
  -- python3 $R/tools/fwd_only.py 2) > $O/pmc_write_r04_x2.log 2>&1
echo "write ok"
