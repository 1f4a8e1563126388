R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in cur2 m8; do SPEF_LIB=abx2/$v.so timeout -k 10 200 python tools/lib_cmp.py fp16mx gpurun_out/cmp_$v.npz > /dev/null 2>&1 || { echo "lib_cmp $v failed"; exit 1; }; done
python tools/lib_cmp.py --cmp gpurun_out/cmp_cur2.npz gpurun_out/cmp_m8.npz
bash tools/r5_var.sh "cur2 m8" 2
python3 -c "
import json
rows={}
for f in ['var_cur21','var_m81','var_cur22','var_m82']:
    d=json.load(open('gpurun_out/'+f+'.json'))
    for k,x in d['kernels'].items():
        if 'x2_irb' in k: rows.setdefault(k,{})[f[4:]]=round(x['ms_per_step']*1e3,1)
for k,v in rows.items(): print(k, v)
"
