R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r5_var.sh "cur5 s1t16 s2t4" 2 > /dev/null
python3 -c "
import json
rows={}
for f in ['cur51','s1t161','s2t41','cur52','s1t162','s2t42']:
    d=json.load(open('gpurun_out/var_'+f+'.json'))
    print(f, d['value'], d['ms_per_step'])
    for k,x in d['kernels'].items():
        if 'mx' in k: rows.setdefault(k,{})[f]=round(x['ms_per_step']*1e3,1)
for k,v in rows.items(): print(k, v)
"
