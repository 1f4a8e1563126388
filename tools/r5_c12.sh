R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
SPEF_LIB=abx2/stamp.so timeout -k 10 200 python tools/kstamp.py > gpurun_out/kstamp3.log 2>&1 || { tail -5 gpurun_out/kstamp3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/kstamp3.log
bash tools/r5_var.sh "p1 g0" 2 > /dev/null
python3 -c "
import json
rows={}
for f in ['p11','g01','p12','g02']:
    d=json.load(open('gpurun_out/var_'+f+'.json'))
    print(f, d['value'], d['ms_per_step'])
    for k,x in d['kernels'].items():
        if 'x2_irb' in k: rows.setdefault(k,{})[f]=round(x['ms_per_step']*1e3,1)
for k,v in rows.items(): print(k, v)
"
