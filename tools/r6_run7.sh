# GPU box: the verify suite of this tree (GPU tests, smoke, bench), then the static wave-priority A/B (tools/r6_run8.sh)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r5_verify.sh || exit 1
bash tools/r6_run8.sh
