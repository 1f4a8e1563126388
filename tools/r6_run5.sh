# GPU box: the verify suite of this tree (GPU tests, smoke, bench), then A/B + bit-identity of abx2/fin.so (this tree)
# against abx2/cur.so (the tree before the hidden-channel permutation / stride-1 row reads)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r5_verify.sh || exit 1
bash tools/r6_ab.sh "cur fin" 2
