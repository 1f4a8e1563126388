R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in p0 p1; do SPEF_LIB=abx2/$v.so timeout -k 10 200 python tools/lib_cmp.py fp16mx gpurun_out/cmp_$v.npz > gpurun_out/cmp_$v.log 2>&1 || { echo "lib_cmp $v failed"; tail -5 gpurun_out/cmp_$v.log; exit 1; }; done
python tools/lib_cmp.py --cmp gpurun_out/cmp_p0.npz gpurun_out/cmp_p1.npz
bash tools/r5_var.sh "p0 p1" 2 > /dev/null
python3 -c "
import json
rows={}
for f in ['p01','p11','p02','p12']:
    d=json.load(open('gpurun_out/var_'+f+'.json'))
    print(f, d['value'], d['ms_per_step'])
    for k,x in d['kernels'].items():
        if 'x2_irb' in k: rows.setdefault(k,{})[f]=round(x['ms_per_step']*1e3,1)
for k,v in rows.items(): print(k, v)
"
