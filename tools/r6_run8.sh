# GPU box: EPnP A/B fin vs osj (one-sided Jacobi on M) and the EPnP tests on osj; static wave priority A/B
# (s_setprio 1): pv = three-stage VALU waves, pm = three-stage MFMA waves, we = role-split expand waves; against fin
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r6_ep.sh "fin osj" || exit 1
SPEF_LIB=$R/abx2/osj.so timeout -k 10 300 python -u -m pytest tests/test_gpu_keypoints.py -k "epnp" -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/osj_tests.log 2>&1; tail -3 gpurun_out/osj_tests.log
bash tools/r6_ab.sh "fin pv pm we" 2
