# round 4: one-pass encode v4 + rp_list (parity, bench) + frame-walk modules
mkdir -p gpurun_out/r04r
true
true
timeout -k 10 300 python -u bench.py --schema rp_list --steps 10 --warmup 3 > gpurun_out/r04r/bench_rp_list.json 2> gpurun_out/r04r/bench_rp_list.err || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_stream_encode.py > gpurun_out/r04r/pytest_stream.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/tune/stream_stamps.py run recvar rpc > gpurun_out/r04r/stamps.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/tune/stream_ab.py recvar rpc > gpurun_out/r04r/ab.log 2>&1 || exit 1
