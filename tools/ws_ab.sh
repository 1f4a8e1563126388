# Pipelined bench A/B of the late-block schedule (--wavespec) for one dtype: bash tools/ws_ab.sh int8 "0 2" [rounds]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
DT=$1; MODES=$2; N=${3:-3}
for r in $(seq $N); do
  L=$MODES; [ $((r % 2)) = 0 ] && L=$(echo $MODES | tr ' ' '\n' | tac | tr '\n' ' ')
  for m in $L; do
    timeout -k 10 120 python bench.py --dtype $DT --wavespec $m --steps 200 --no-cpu-baseline --no-int8 --no-keypoint \
      --no-x2 --no-peaks --sharp-frames 0 > gpurun_out/ws_$DT$m$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ws_$DT$m$r.json'));print('$DT wavespec $m', d['value'], d['ms_per_step'], d['sclk_timed_region']['sclk_mhz'])"
  done
done
