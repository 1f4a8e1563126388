# Interleaved keypoint-mode fp16x2 timings of abx2/*.so builds (tools/variant_time.py, single stream)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for pass in 1 2; do
  L="$*"; [ $pass = 2 ] && L=$(echo "$@" | tr ' ' '\n' | tac | tr '\n' ' ')
  for v in $L; do
    SPEF_LIB=$R/abx2/$v.so timeout -k 10 120 python tools/variant_time.py fp16x2 keypoints 64 > gpurun_out/x2k_$v$pass.log 2>&1 || exit 1
    echo "$v: $(grep -E '^==' gpurun_out/x2k_$v$pass.log)"; grep -E "kernel<160" gpurun_out/x2k_$v$pass.log
  done
done
