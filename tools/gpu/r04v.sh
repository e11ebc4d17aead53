# round 4: packed element-subroutine areas (containertest) parity + bench; encode halves A/B
mkdir -p gpurun_out/r04v
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_containers.py tests/test_gpu_parity.py tests/test_gpu_messages.py tests/test_deep.py tests/test_record_index.py > gpurun_out/r04v/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --schema containertest --steps 10 --warmup 3 > gpurun_out/r04v/bench_containertest.json 2> gpurun_out/r04v/bench_containertest.err || exit 1
timeout -k 10 200 python -u tools/tune/stream_ab.py recvar rpc > gpurun_out/r04v/ab.log 2>&1 || exit 1
