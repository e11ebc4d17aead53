# Decode option A/B for a packed plan (tools/tune/dec_ab.py, VALS as there),
# then the same under rocprofv3 --pmc WRITE_SIZE (21 decode dispatches per
# option set, in VALS order).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-stage}; mkdir -p $O
timeout -k 10 240 python3 -u tools/tune/dec_ab.py ${SCHEMA:-vecrec} > $O/ab.log 2>&1 \
  && grep -v amdgpu.ids $O/ab.log | tail -20 \
  && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/w" -o run --output-format csv -- python3 tools/tune/dec_ab.py ${SCHEMA:-vecrec} > "$O/w.log" 2>&1
