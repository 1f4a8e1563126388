# irp weight-streaming ablations (kbrun/ binaries from tools/kbench/ablate.sh base no_wload no_eload no_pload fixed_wload)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for pass in 1 2; do
  for g in "irp 96 576 160 2 0 32 32" "irp 160 960 160 1 1 16 16" "irp 160 960 320 1 0 16 16"; do
    L="base no_wload no_eload no_pload fixed_wload"; [ $pass = 2 ] && L="fixed_wload no_pload no_eload no_wload base"
    for v in $L; do
      printf "%-12s %-28s " $v "$g"; timeout -k 5 60 ./kbrun/blk_$v $g || exit $?
    done
  done
done
