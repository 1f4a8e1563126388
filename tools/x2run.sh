# fp16x2 tests + per-kernel timings of the precision variants (GPU box)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_x2.py $R/tests/test_gpu_measure.py -m gpu -x -v -s --timeout 90 --timeout-method thread > $R/gpurun_out/x2t.log 2>&1; rc=$?
tail -25 $R/gpurun_out/x2t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 python -c "
import sys; sys.path[:0]=['$R','$R/spacecraft-pose-estimation-framework_amd']
from spef_amd.measure import measure_peaks; print(measure_peaks(0, 2))" &&
timeout -k 10 120 python $R/tools/variant_time.py fp16x2 ursonet 64 > $R/gpurun_out/x2u.log 2>&1 && cat $R/gpurun_out/x2u.log &&
timeout -k 10 120 python $R/tools/variant_time.py fp16x2 keypoints 64 > $R/gpurun_out/x2k.log 2>&1 && cat $R/gpurun_out/x2k.log
