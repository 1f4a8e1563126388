R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r5_var.sh "g0 cur3" 2 > /dev/null
python3 -c "
import json
rows={}
for f in ['var_g01','var_cur31','var_g02','var_cur32']:
    d=json.load(open('gpurun_out/'+f+'.json'))
    print(f, d['value'])
    for k,x in d['kernels'].items():
        if 'x2_irb' in k: rows.setdefault(k,{})[f[4:]]=round(x['ms_per_step']*1e3,1)
for k,v in rows.items(): print(k, v)
"
