# GPU box: bit-identity of abx2/<name>.so builds against the first (fp16mx URSONet + keypoint outputs, tools/lib_cmp.py),
# then interleaved pipelined-bench A/B (fp16mx headline, 50 steps): bash tools/r6_ab.sh "a b c" [passes] [bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
LIBS=$1; N=${2:-2}; shift 2; EXTRA="$*"
first=""
for v in $LIBS; do
  SPEF_LIB=$R/abx2/$v.so timeout -k 10 120 python tools/lib_cmp.py ${CMP_DT:-fp16mx} gpurun_out/cmp_$v.npz > /dev/null 2> gpurun_out/cmp_$v.err || { tail -5 gpurun_out/cmp_$v.err; exit 1; }
  if [ -n "$first" ]; then echo "== $v vs $first"; python tools/lib_cmp.py --cmp gpurun_out/cmp_$first.npz gpurun_out/cmp_$v.npz; else first=$v; fi
done
for r in $(seq $N); do
  L=$LIBS; [ $((r % 2)) = 0 ] && L=$(echo $LIBS | tr ' ' '\n' | tac | tr '\n' ' ')
  for v in $L; do
    SPEF_LIB=$R/abx2/$v.so timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-keypoint --no-int8 --no-peaks \
      --no-x2 --no-fp16 --no-cpu-baseline --sharp-frames 0 --detail-out gpurun_out/ab_$v$r.json $EXTRA > /dev/null 2> gpurun_out/ab_$v$r.err || { tail -20 gpurun_out/ab_$v$r.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/ab_$v$r.json')); print('$v', d['value'], d['ms_per_step'], d['sclk_timed_region']['sclk_mhz'], 'leg', d['roofline']['sclk_mhz'])
print('   ', {k.split('_kernel')[0][:4]+'<'+k.split('<')[-1]: round(x['ms_per_step']*1e3,1) for k,x in d['kernels'].items()})"
  done
done
