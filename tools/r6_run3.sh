# GPU box: EPnP A/B (ep0 default, ep1 = look-ahead rounds on a rotation wave, ept20 / ept16 = Jacobi stop at
# off^2 <= 1e-20 / 1e-16 diag^2), fp16mx A/B cur vs nt (nontemporal x2_irp output stores), FETCH/WRITE traffic of both,
# then per-chunk timelines of the three-stage kernels (abx2/stamp3.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r6_ep.sh "ep0 ep1 ept20 ept16" || exit 1
bash tools/r6_ab.sh "cur nt" 2 || exit 1
bash tools/r6_traffic.sh "cur nt" || exit 1
SPEF_LIB=$R/abx2/stamp3.so timeout -k 10 120 python tools/kstamp_irp.py 12:36 11:24 15:30 17:30
