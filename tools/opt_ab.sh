# Pipelined bench A/B of schedule options: bash tools/opt_ab.sh fp16 "base|--wavespec 1|--set-option 4=1" [rounds]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
DT=$1; IFS='|' read -ra VARS <<< "$2"; N=${3:-2}
for r in $(seq $N); do
  for ((j = 0; j < ${#VARS[@]}; j++)); do
    k=$j; [ $((r % 2)) = 0 ] && k=$((${#VARS[@]} - 1 - j))
    v=${VARS[$k]}; a=$v; [ "$v" = base ] && a=""
    timeout -k 10 120 python bench.py --dtype $DT $a --steps 200 --no-cpu-baseline --no-int8 --no-keypoint --no-x2 \
      --no-peaks --sharp-frames 0 > gpurun_out/oab.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/oab.json'));print('$DT [$v]', d['value'], d['ms_per_step'], d['sclk_timed_region']['sclk_mhz'])"
  done
done
