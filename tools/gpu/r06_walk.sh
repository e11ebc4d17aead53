# Record/message index walk with several segments per workgroup: index tests, kernel times, bench lines.
export TMPDIR=/tmp
O=gpurun_out/r06wk; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_record_index.py tests/test_gpu_messages.py tests/test_long_messages.py tests/test_deep.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof -o k --output-format csv -- python3 tools/gpu/ix_bench.py vecrec,containertest,rpc,recvar > $O/prof.log 2>&1 && python3 tools/gpu/ix_trace.py $O/prof vecrec,containertest,rpc,recvar
for sc in containertest vecrec rpc; do timeout -k 10 300 python3 -u bench.py --schema $sc --no-cpu-baseline > $O/bench_$sc.log 2>&1 || exit 1; done
echo benches done
