# round 4: line-buffered frame-walk encode: parity + rp_list bench + PMC
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04ag
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 90 --timeout-method thread -m gpu tests/test_deep.py tests/test_containers.py tests/test_gpu_parity.py tests/test_gpu_messages.py -k "rp_list or deep or recursive or container or spec" > $O/pytest.log 2>&1 || exit 1
B="bench.py --no-cpu-baseline --no-large --no-cold --no-host-inclusive --no-plain --steps 10 --warmup 3 --schema rp_list"
timeout -k 10 300 python3 $B > $O/bench_rp_list.json 2> $O/bench_rp_list.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/stats_rp_list -o k --output-format csv -- python3 $B > $O/stats_rp_list.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_rp_list -o k --output-format csv -- python3 $B > $O/fetch_rp_list.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/write_rp_list -o k --output-format csv -- python3 $B > $O/write_rp_list.log 2>&1 || exit 1
