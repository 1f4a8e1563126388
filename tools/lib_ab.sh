# Pipelined bench A/B of library builds (abx2/<name>.so): bash tools/lib_ab.sh int8 "L0 L1 L2" [rounds] [extra bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
DT=$1; LIBS=$2; N=${3:-2}; shift 3; EXTRA="$*"
for r in $(seq $N); do
  L=$LIBS; [ $((r % 2)) = 0 ] && L=$(echo $LIBS | tr ' ' '\n' | tac | tr '\n' ' ')
  for v in $L; do
    SPEF_LIB=$R/abx2/$v.so timeout -k 10 120 python bench.py --dtype $DT --steps 200 --no-cpu-baseline --no-int8 \
      --no-keypoint --no-x2 --no-peaks --sharp-frames 0 $EXTRA > gpurun_out/lab_$DT$v$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/lab_$DT$v$r.json'));print('$DT $v', d['value'], d['ms_per_step'], d['sclk_timed_region']['sclk_mhz'])"
  done
done
