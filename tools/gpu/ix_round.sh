# Record index: GPU tests, 1M bench (fast vs list ranking), rocprof stats.
#   gpurun -- 'TAG=ix4 bash tools/gpu/ix_round.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ix}
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_record_index.py -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
timeout -k 10 200 python3 -u tools/gpu/ix_bench.py > "$O/ix.log" 2>&1 || exit $?
cat "$O/ix.log"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof" -o k --output-format csv -- python3 tools/gpu/ix_bench.py ${SCHEMAS:-recvar,rpc} > "$O/prof.log" 2>&1
