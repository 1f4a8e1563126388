# GPU box: pipeline depth / graphs A/B on this tree (50-step fp16mx headline legs, interleaved), then the round-6
# measurement artefacts of this tree (tools/r6_profile.sh r06 full: bench line with every sub-record, rocprofv3 stats,
# FETCH / WRITE passes, SQ counters)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for r in 1 2; do
  for a in "--inflight 3" "--inflight 2" "--inflight 4" "--graphs"; do
    timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-keypoint --no-int8 --no-peaks --no-x2 --no-fp16 \
      --no-cpu-baseline --sharp-frames 0 --detail-out gpurun_out/pl.json $a > /dev/null 2> gpurun_out/pl.err || { tail -20 gpurun_out/pl.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/pl.json')); print('$a', d['value'], d['ms_per_step'], d['sclk_timed_region']['sclk_mhz'])"
  done
done
bash tools/r6_profile.sh r06 full
bash tools/r6_ab.sh "fin dmal fastin" 2
