# round 4: walk-first record kernel without the native tile (records loaded into registers)
mkdir -p gpurun_out/r04ac
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_stream_encode.py > gpurun_out/r04ac/pytest_stream.log 2>&1 || exit 1
VARIANTS="two_pass walk_first lb sized" REPS=20 timeout -k 10 300 python -u tools/tune/stream_ab.py recvar rpc > gpurun_out/r04ac/ab.log 2>&1 || exit 1
