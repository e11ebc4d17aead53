# A/B of encode code-object variants built by tools/tune/enc_stamps.py
# (NOSTAMP=1 TAG=<t> CFLAGS=... build), each against the library in one
# process, interleaved; then optionally the profile round.
#   gpurun -- 'TAGS="pipe0 pipe1" bash tools/gpu/enc_tags.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${OUT_TAG:-enctags}
mkdir -p "$O"
for t in ${TAGS:-pipe0 pipe1}; do
  NOSTAMP=1 TAG=$t IMAGES="${IMAGES:--1}" timeout -k 10 300 python3 -u tools/tune/enc_stamps.py run ${SCH:-recvar rpc vecrec} > "$O/$t.log" 2>&1 || { tail -5 "$O/$t.log"; exit 1; }
  grep -v "^/opt" "$O/$t.log" | sed "s/^/$t /"
done
