# GPU box: EPnP timing of abx2/<name>.so builds (tools/epnp_time.py) + bit-identity of their outputs against the first:
# bash tools/r6_ep.sh "a b"
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
first=""
for v in $1; do
  echo "== $v"
  EPNP_DUMP=gpurun_out/ep_$v SPEF_LIB=$R/abx2/$v.so timeout -k 10 120 python tools/epnp_time.py 2> gpurun_out/ep_$v.err || { tail -5 gpurun_out/ep_$v.err; exit 1; }
  if [ -n "$first" ]; then
    python -c "
import numpy as np
for P in (64, 512, 1800):
    a, b = np.load('gpurun_out/ep_${first}_%d.npz' % P), np.load('gpurun_out/ep_${v}_%d.npz' % P)
    print(P, 'bit-identical' if all(np.array_equal(a[k], b[k]) for k in a) else 'DIFF %.2e' % max(np.abs(a[k] - b[k]).max() for k in a))"
  else first=$v; fi
done
