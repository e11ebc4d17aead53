# A/B of the var encode's window pipelining on one box, one process per
# variant (tools/tune/enc_stamps.py, NOSTAMP): each variant's code object
# (built here beforehand: TAG=<v> NOSTAMP=1 [CFLAGS=...] enc_stamps.py build)
# timed against the library, interleaved, bytes checked against it.
#   gpurun -- 'VARIANTS="base p1" bash tools/gpu/enc_pair_ab.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${OUT_TAG:-encpair}
mkdir -p "$O"
for v in ${VARIANTS:-base p1}; do
  TAG=$v NOSTAMP=1 IMAGES="${IMAGES:-4096}" timeout -k 10 300 python3 -u tools/tune/enc_stamps.py run ${SCH:-recvar rpc} > "$O/$v.log" 2>&1 || { tail -5 "$O/$v.log"; exit 1; }
  grep -v "^/opt" "$O/$v.log" | sed "s/^/$v /"
done
