# The size walk's chain pass: the recursive-plan GPU tests, then the rp_list bench line.
export TMPDIR=/tmp
O=gpurun_out/r06ch; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_deep.py tests/test_graph_capture.py tests/test_record_index.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 -u bench.py --schema rp_list --no-cpu-baseline > $O/bench_rp.log 2>&1 || { tail -20 $O/bench_rp.log; exit 1; }
tail -c 1500 $O/bench_rp.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/stats -o k --output-format csv -- python3 bench.py --no-cpu-baseline --no-large --no-cold --no-host-inclusive --no-plain --steps 10 --warmup 3 --schema rp_list > $O/stats.log 2>&1
