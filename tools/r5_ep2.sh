R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in eab0 eab1 eab2 eab3 eab4; do echo $v; SPEF_LIB=abx2/$v.so timeout -k 10 100 python tools/epnp_time.py 2>&1 | grep "P=64\|P=1800" || exit 1; done
