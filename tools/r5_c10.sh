R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in xc0 xc3; do SPEF_LIB=abx2/$v.so timeout -k 10 200 python tools/lib_cmp.py fp16mx gpurun_out/cmp_$v.npz > gpurun_out/cmp_$v.log 2>&1 || { echo "lib_cmp $v failed"; tail -5 gpurun_out/cmp_$v.log; exit 1; }; done
python tools/lib_cmp.py --cmp gpurun_out/cmp_xc0.npz gpurun_out/cmp_xc3.npz
bash tools/r5_var.sh "xc0 xc3" 2 > /dev/null
python3 -c "
import json
rows={}
for f in ['xc01','xc31','xc02','xc32']:
    d=json.load(open('gpurun_out/var_'+f+'.json'))
    print(f, d['value'], d['ms_per_step'])
    for k,x in d['kernels'].items():
        if 'x2_irb' in k: rows.setdefault(k,{})[f]=round(x['ms_per_step']*1e3,1)
for k,v in rows.items(): print(k, v)
"
