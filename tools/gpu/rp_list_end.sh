# rp_list end set after the list decode: GPU tests, smoke, the rp_list bench line,
# rocprof kernel stats and FETCH/WRITE passes (gpurun_out/r06fin2).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06fin2
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -20 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > "$O/smoke.log" 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --schema rp_list > "$O/bench_rp_list.log" 2>&1 || exit 1
B="bench.py --no-cpu-baseline --no-large --no-cold --no-host-inclusive --no-plain --no-shard --steps 10 --warmup 3"
s=rp_list
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/stats_$s" -o k --output-format csv -- python3 $B --schema "$s" > "$O/stats_$s.log" 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch_$s" -o k --output-format csv -- python3 $B --schema "$s" > "$O/fetch_$s.log" 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/write_$s" -o k --output-format csv -- python3 $B --schema "$s" > "$O/write_$s.log" 2>&1 || exit 1
echo done
