# Interleaved fp16x2 per-kernel timings of abx2/*.so builds, URSONet 512^2 and keypoint mode (GPU box)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for pass in 1 2; do
  L="$*"; [ $pass = 2 ] && L=$(echo "$@" | tr ' ' '\n' | tac | tr '\n' ' ')
  for v in $L; do
    for h in ursonet keypoints; do
      SPEF_LIB=$R/abx2/$v.so timeout -k 10 120 python tools/variant_time.py fp16x2 $h 64 > gpurun_out/x2v_$v$h$pass.log 2>&1 || exit 1
      echo "$v $(grep -E '^==' gpurun_out/x2v_$v$h$pass.log)"; grep -E "x2_pw" gpurun_out/x2v_$v$h$pass.log
    done
  done
done
