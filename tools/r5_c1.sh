# EPnP variant timing + staging bit-identity + the in-tree build's parity tests + interleaved bench variants
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
for v in ep3 fd fr fr_r32t26; do echo $v; SPEF_LIB=abx2/$v.so timeout -k 10 100 python tools/epnp_time.py || exit 1; done
for v in g0 g1; do SPEF_LIB=abx2/$v.so timeout -k 10 200 python tools/lib_cmp.py fp16mx gpurun_out/cmp_$v.npz > /dev/null 2>&1 || { echo "lib_cmp $v failed"; exit 1; }; done
python tools/lib_cmp.py --cmp gpurun_out/cmp_g0.npz gpurun_out/cmp_g1.npz
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_keypoints.py tests/test_gpu_mx.py tests/test_gpu_x2.py \
  > gpurun_out/c1_tests.log 2>&1 || { tail -40 gpurun_out/c1_tests.log; exit 1; }
tail -3 gpurun_out/c1_tests.log
bash tools/r5_var.sh "pk0 pk1d0 g0 g1 fw1 hl1 al1" 2
