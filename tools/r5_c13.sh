R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
V="${1:-p1 w2 d1 d2}"
for v in $V; do SPEF_LIB=abx2/$v.so timeout -k 10 200 python tools/lib_cmp.py fp16mx gpurun_out/cmp_$v.npz > gpurun_out/cmp_$v.log 2>&1 || { echo "lib_cmp $v failed"; tail -5 gpurun_out/cmp_$v.log; exit 1; }; done
F=$(echo $V | cut -d' ' -f1)
for v in $V; do echo "$F vs $v"; python tools/lib_cmp.py --cmp gpurun_out/cmp_$F.npz gpurun_out/cmp_$v.npz; done
bash tools/r5_var.sh "$V" 2 > /dev/null
python3 -c "
import json,sys
V=sys.argv[1].split()
rows={}
for r in (1,2):
  for v in V:
    f=v+str(r)
    d=json.load(open('gpurun_out/var_'+f+'.json'))
    print(f, d['value'], d['ms_per_step'])
    for k,x in d['kernels'].items():
        if 'x2_irb' in k or 'x2_pw' in k: rows.setdefault(k,{})[f]=round(x['ms_per_step']*1e3,1)
for k,v in rows.items(): print(k, v)
" "$V"
