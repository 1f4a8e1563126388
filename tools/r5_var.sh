# interleaved pipelined-bench A/B of abx2/<name>.so builds (fp16mx headline): bash tools/r5_var.sh "a b c" [passes]
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
LIBS=$1; N=${2:-2}; shift 2; EXTRA="$*"
for r in $(seq $N); do
  L=$LIBS; [ $((r % 2)) = 0 ] && L=$(echo $LIBS | tr ' ' '\n' | tac | tr '\n' ' ')
  for v in $L; do
    SPEF_LIB=$R/abx2/$v.so timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-keypoint --no-int8 --no-peaks \
      --no-x2 --no-fp16 --no-cpu-baseline $EXTRA > gpurun_out/var_$v$r.json 2> gpurun_out/var_$v$r.err || { tail -20 gpurun_out/var_$v$r.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/var_$v$r.json')); print('$v', d['value'], d['ms_per_step'], d['sclk_timed_region']['sclk_mhz'])
print('   ', {k.split('<')[0][:6]+'<'+k.split('<')[1]: round(x['ms_per_step']*1e3,1) for k,x in d['kernels'].items() if 'mx_' in k or 'front' in k})"
  done
done
