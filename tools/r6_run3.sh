# GPU box: EPnP A/B (ep0 default, ep1 = look-ahead rounds on a rotation wave), fp16mx A/B cur vs nt (nontemporal
# x2_irp output stores), FETCH/WRITE traffic of both
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r6_ep.sh "ep0 ep1" || exit 1
bash tools/r6_ab.sh "cur nt" 2 || exit 1
bash tools/r6_traffic.sh "cur nt"
