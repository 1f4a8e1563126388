# GPU box: per-kernel forward times of abx2/<name>.so builds, interleaved: bash tools/ktime.sh "a b c" [passes]
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
LIBS=$1; N=${2:-2}
for r in $(seq $N); do
  L=$LIBS; [ $((r % 2)) = 0 ] && L=$(echo $LIBS | tr ' ' '\n' | tac | tr '\n' ' ')
  for v in $L; do
    echo -n "$v " >> gpurun_out/kt.txt
    SPEF_LIB=$R/abx2/$v.so timeout -k 10 120 python tools/ktime.py >> gpurun_out/kt.txt 2> gpurun_out/kt_$v.err || { tail -5 gpurun_out/kt_$v.err; exit 1; }
  done
done
python tools/kt_table.py gpurun_out/kt.txt
