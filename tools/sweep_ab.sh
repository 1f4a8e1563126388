#!/bin/bash
# Tile-variant sweep (SPEF_OPT_IRB_VARIANT 0,1,2) of two library builds, interleaved (GPU box, repo root):
#   bash tools/sweep_ab.sh abbase/other.so [kernel-name-regex]
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
F=${2:-irb_kernel}
for i in 1 2; do
  for lib in "" "$1"; do
    echo "### lib=${lib:-in-tree} pass $i"
    SPEF_LIB=$lib SWEEP=0,1,2 timeout -k 10 200 python $R/tools/explore.py > $R/gpurun_out/sw.log 2>&1 || { tail -20 $R/gpurun_out/sw.log; exit 1; }
    grep -E "^==|$F" $R/gpurun_out/sw.log
  done
done
