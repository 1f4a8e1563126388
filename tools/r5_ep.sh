R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in ew0 ew2 ew3 ew0; do echo $v; SPEF_LIB=abx2/$v.so timeout -k 10 100 python tools/epnp_time.py || exit 1; done
