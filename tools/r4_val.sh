# Round-4 validation on the GPU box: fp16x2 tests + timings, C2 table, irp weight-load ablation (kbrun/ binaries)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/x2run.sh || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_c2_precision.py -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/c2.log 2>&1; rc=$?
grep -E "^C2|passed|failed" gpurun_out/c2.log
[ $rc -eq 0 ] || exit $rc
if false; then
  for pass in 1 2; do
    for v in base no_wload; do
      for g in "irp 160 960 160 1 1 16 16" "irp 96 576 160 2 0 32 32" "irp 160 960 320 1 0 16 16"; do
        printf "%-9s %-28s " $v "$g"; timeout -k 5 60 ./kbrun/blk_$v $g || exit $?
      done
    done
  done
fi
bash tools/r4_abl.sh && \
bash tools/x2_ab.sh A B C D
