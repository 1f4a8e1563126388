#!/bin/bash
# One kbench binary, several kernel variants of one geometry, interleaved (two passes, order reversed).
# usage: tools/kbench/var_run.sh <binary> "<kind CIN HID COUT S RES H W B>" variant...
set -e
BIN=$1; ARGS=$2; shift 2
for pass in 1 2; do
  if [ $pass = 1 ]; then L="$*"; else L=$(echo "$@" | tr ' ' '\n' | tac | tr '\n' ' '); fi
  for v in $L; do
    printf "variant %-3s " $v; timeout -k 5 60 $BIN $ARGS $v 200
  done
done
