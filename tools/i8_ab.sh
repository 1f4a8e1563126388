# Interleaved per-kernel timings of int8 library builds (abx2/*.so) with tools/variant_time.py (GPU box)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for pass in 1 2; do
  L="$*"; [ $pass = 2 ] && L=$(echo "$@" | tr ' ' '\n' | tac | tr '\n' ' ')
  for v in $L; do
    echo "### $v pass $pass"
    SPEF_LIB=$R/abx2/$v.so timeout -k 10 120 python tools/variant_time.py int8 ursonet 64 > gpurun_out/i8ab_$v$pass.log 2>&1 || { tail -5 gpurun_out/i8ab_$v$pass.log; exit 1; }
    grep -E "^==|q_irb_kernel<(64|96|160)" gpurun_out/i8ab_$v$pass.log
  done
done
