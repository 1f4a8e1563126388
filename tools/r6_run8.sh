# GPU box: static wave priority A/B (s_setprio 1): pv = three-stage VALU waves, pm = three-stage MFMA waves,
# we = role-split expand waves; against fin (this tree's default)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r6_ab.sh "fin pv pm we" 2
