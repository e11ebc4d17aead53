# round 4: walk-first encode (look-back) tests, stamps, A/B
mkdir -p gpurun_out/r04s
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_stream_encode.py > gpurun_out/r04s/pytest_stream.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/tune/stream_ab.py recvar rpc > gpurun_out/r04s/ab.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/tune/stream_stamps.py run recvar rpc > gpurun_out/r04s/stamps.log 2>&1 || exit 1
