export TMPDIR=/tmp
O=gpurun_out/r06ix2; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_record_index.py tests/test_deep.py tests/test_graph_capture.py tests/test_gpu_messages.py tests/test_long_messages.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python3 -u tools/gpu/rx_whole_diag.py rp_list > $O/diag_rp.log 2>&1 && tail -2 $O/diag_rp.log
timeout -k 10 120 python3 -u tools/gpu/rx_whole_diag.py bigrec > $O/diag_big.log 2>&1 && tail -2 $O/diag_big.log
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof -o k --output-format csv -- python3 tools/gpu/ix_bench.py vecrec,containertest,rpc > $O/prof.log 2>&1 && python3 tools/gpu/ix_trace.py $O/prof vecrec,containertest,rpc
WHOLE=1 timeout -k 10 200 python3 -u tools/tune/ix_stamps.py run containertest vecrec > $O/stamps.log 2>&1; cat $O/stamps.log
timeout -k 10 300 python3 -u bench.py --schema containertest --no-cpu-baseline > $O/bench_ct.log 2>&1
timeout -k 10 300 python3 -u bench.py --schema rp_list --no-cpu-baseline > $O/bench_rp.log 2>&1
timeout -k 10 300 python3 -u bench.py --schema vecrec --no-cpu-baseline > $O/bench_vec.log 2>&1
