# Stamped phase timings of the spec encode for several U (chunks in flight
# per lane) x LDS window sizes: tools/tune/enc_stamps.py run per U.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${OUT_TAG:-stampsweep}
mkdir -p "$O"
for u in ${US:-2 4}; do
  U=$u TAG=${TAG:-st} IMAGES="${IMAGES:-2048 4096}" timeout -k 10 300 python3 -u tools/tune/enc_stamps.py run ${SCH:-recvar rpc} > "$O/u$u.log" 2>&1 || { tail -5 "$O/u$u.log"; exit 1; }
  grep -v "^/opt" "$O/u$u.log" | sed "s/^/U=$u /"
done
