# GPU box: FETCH_SIZE / WRITE_SIZE passes (separate runs) of the fp16mx forward for abx2/<name>.so builds:
# bash tools/r6_traffic.sh "a b"  -> gpurun_out/tr_<name>_{fetch,write}/ + a per-kernel MB table
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
set -e
for v in $1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf $R/gpurun_out/tr_${v}_$c
    (cd /tmp && SPEF_LIB=$R/abx2/$v.so DT=fp16mx timeout -s KILL 150 rocprofv3 --pmc $c -d $R/gpurun_out/tr_${v}_$c -o run \
      --output-format csv -- python3 $R/tools/fwd_only.py 2) > $R/gpurun_out/tr_${v}_$c.log 2>&1
  done
  echo "== $v (HBM MB per launch = (2 FETCH + WRITE) KB x 1024)"
  python3 - $R/gpurun_out/tr_${v}_FETCH_SIZE $R/gpurun_out/tr_${v}_WRITE_SIZE <<'PY'
import csv, glob, sys, os
sys.path.insert(0, os.path.join(os.environ.get('GRAFT_REPO_ROOT', '.'), 'tools'))
from rocprof_summary import short_name
from collections import defaultdict
v = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            v[short_name(r['Kernel_Name'])][r['Counter_Name']].append(float(r['Counter_Value']))
for k, c in sorted(v.items()):
    fe = sum(c['FETCH_SIZE']) / max(1, len(c['FETCH_SIZE'])); wr = sum(c['WRITE_SIZE']) / max(1, len(c['WRITE_SIZE']))
    print(f'{k:45s} {(2 * fe + wr) * 1024 / 1e6:8.1f} MB  (fetch {fe * 1024 / 1e6:.1f}, write {wr * 1024 / 1e6:.1f})')
PY
done
