# GPU box: EPnP A/B (ep0 default, eprot = fp32 rotation + one fp64 Newton step), fp16mx A/B cur vs mj1 / mj2 (the
# MFMA waves issue 1 / 2 rounds of the expand-stage LDS-DMA pieces in the PT three-stage kernels) and swz (stride-2
# slab swizzle), timelines of mj2, LDS bank-conflict counters of cur and swz
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r6_ep.sh "ep0 eprot" || exit 1
bash tools/r6_ab.sh "cur mj1 mj2 swz k6mj2 perm permswz allmx" 2 || exit 1
SPEF_LIB=$R/abx2/stampmj2.so timeout -k 10 120 python tools/kstamp_irp.py 12:18 11:12 || exit 1
for v in cur permswz; do
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
    if 'mx_' in k or 'front' in k:
        m = lambda n: sum(c[n]) / max(1, len(c[n]))
        print(f"{k:45s} conflict/active {m('SQ_LDS_BANK_CONFLICT') / max(1, m('SQ_LDS_IDX_ACTIVE')):.3f}  valu/wave {m('SQ_INSTS_VALU') / max(1, m('SQ_WAVES')):.0f}")
PY
done
