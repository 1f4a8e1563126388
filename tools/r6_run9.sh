# GPU box: fp16mx A/B fin vs swz2 (stride-2 slab swizzle with per-lane tap-column bases precomputed), bit-identity,
# LDS bank-conflict counters of both
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r6_ab.sh "fin swz2" 3 || exit 1
for v in fin swz2; do
  (cd /tmp && SPEF_LIB=$R/abx2/$v.so DT=fp16mx timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VALU \
    -d $R/gpurun_out/lds_$v -o run --output-format csv -- python3 $R/tools/fwd_only.py 2) > $R/gpurun_out/lds_$v.log 2>&1 || exit 1
  python3 - $R/gpurun_out/lds_$v <<'PY'
import csv, glob, sys, os
sys.path.insert(0, os.path.join(os.environ.get('GRAFT_REPO_ROOT', '.'), 'tools'))
from rocprof_summary import short_name
from collections import defaultdict
v = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        v[short_name(r['Kernel_Name'])][r['Counter_Name']].append(float(r['Counter_Value']))
print('==', sys.argv[1])
for k, c in sorted(v.items()):
    if 'mx_' in k:
        m = lambda n: sum(c[n]) / max(1, len(c[n]))
        print(f"{k:45s} conflict/active {m('SQ_LDS_BANK_CONFLICT') / max(1, m('SQ_LDS_IDX_ACTIVE')):.3f}  valu/wave {m('SQ_INSTS_VALU') / max(1, m('SQ_WAVES')):.0f}")
PY
done
