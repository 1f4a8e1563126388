# GPU box: the verify suite (GPU tests, smoke, bench), the EPnP A/B of abx2/ep{0,1,2}.so, the mx A/B of abx2/mx{0,1}.so
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r5_verify.sh || exit 1
bash tools/r6_ep.sh "ep0 ep1 ep2" || exit 1
bash tools/r6_ab.sh "mx0 mx1" 2
