# A/B of the spec var encode's shape: chunks in flight per lane (U) x LDS
# window bytes, each against the library default, one process per U.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-encab}
mkdir -p $O
for u in ${US:-4 8}; do
  U=$u NOSTAMP=1 IMAGES="${IMAGES:-4096 8192 12288 16384}" timeout -k 10 300 python -u tools/tune/enc_stamps.py run ${SCH:-recvar rpc vecrec} > $O/u$u.log 2>&1 || { tail -5 $O/u$u.log; exit 1; }
  grep -v "^/opt" $O/u$u.log | sed "s/^/U=$u /"
done
