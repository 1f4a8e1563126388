# GPU box: EPnP A/B (abx2/ep0 = current default, ep1 = look-ahead Jacobi rounds), then the fp16mx A/B of mx0 (previous
# tree), cur (this tree's default) and b3w2 (block 3 at two waves per SIMD with row-batched depthwise reads)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r6_ep.sh "ep0 ep1" || exit 1
bash tools/r6_ab.sh "mx0 cur b3w2" 2
