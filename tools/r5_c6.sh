R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r5_var.sh "cur4 ex0 lh1" 2 > /dev/null
python3 -c "
import json
rows={}
for f in ['cur41','ex01','lh11','cur42','ex02','lh12']:
    d=json.load(open('gpurun_out/var_'+f+'.json'))
    print(f, d['value'], d['ms_per_step'])
    for k,x in d['kernels'].items():
        if ('32,192' in k) or ('mx' in k): rows.setdefault(k,{})[f]=round(x['ms_per_step']*1e3,1)
for k,v in rows.items(): print(k, v)
"
