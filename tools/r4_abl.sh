# Memory-phase ablations of the fused kernels (kbrun/ = tools/kbench/ablate.sh binaries; timing only, wrong results)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for pass in 1 2; do
  for g in "front 3 32 16 2 0 512 512" "irb 16 96 24 2 0 256 256" "irw 64 384 64 1 1 32 32" "irw 96 576 96 1 1 32 32" \
           "irp 160 960 160 1 1 16 16" "irp 160 960 320 1 0 16 16"; do
    for v in base no_xload no_ystore no_mem no_wload; do
      if [ $pass = 2 ]; then case $v in base) v=no_wload;; no_wload) v=base;; esac; fi
      printf "%-10s %-28s " $v "$g"; timeout -k 5 60 ./kbrun/blk_$v $g || exit $?
    done
  done
done
