# Interleaved per-kernel timings of fp16x2 library builds (abx2/*.so) with tools/variant_time.py (GPU box)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for pass in 1 2; do
  L="$*"; [ $pass = 2 ] && L=$(echo "$@" | tr ' ' '\n' | tac | tr '\n' ' ')
  for v in $L; do
    echo "### $v pass $pass"
    SPEF_LIB=$R/abx2/$v.so timeout -k 10 120 python tools/variant_time.py fp16x2 ursonet 64 > gpurun_out/x2ab_$v$pass.log 2>&1 || exit $?
    grep -E "^==|x2_irw|x2_irb_kernel<96|x2_irb_kernel<64" gpurun_out/x2ab_$v$pass.log
    SPEF_LIB=$R/abx2/$v.so timeout -k 10 120 python tools/variant_time.py fp16x2 keypoints 64 > gpurun_out/x2abk_$v$pass.log 2>&1 || exit $?
    grep -E "^==|x2_irw|x2_irb_kernel<96|x2_irb_kernel<64" gpurun_out/x2abk_$v$pass.log
  done
done
