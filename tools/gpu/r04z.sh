# round 4: same-process rocprof of the encode phase, two-pass record kernel vs walk-first,
# kernel stats + FETCH_SIZE / WRITE_SIZE passes (separate runs)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04z}
mkdir -p $O
export VARIANTS="two_pass walk_first" REPS=10
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/stats -o k --output-format csv -- python3 tools/tune/stream_ab.py recvar rpc > $O/stats.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o k --output-format csv -- python3 tools/tune/stream_ab.py recvar rpc > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/write -o k --output-format csv -- python3 tools/tune/stream_ab.py recvar rpc > $O/write.log 2>&1 || exit 1
