#!/bin/bash
# Runs the ablation binaries of tools/kbench/ablate.sh on the GPU box, interleaved (two passes, order reversed).
# usage: tools/kbench/abl_run.sh "<blk_trace args>" name...
set -e
cd "$(dirname "$0")/abl"
ARGS=$1; shift
for pass in 1 2; do
  if [ $pass = 1 ]; then L="$*"; else L=$(echo "$@" | tr ' ' '\n' | tac | tr '\n' ' '); fi
  for v in $L; do
    printf "%-12s " $v; timeout -k 5 60 ./blk_$v $ARGS
  done
done
