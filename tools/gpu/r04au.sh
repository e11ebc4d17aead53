# round 4: odd bounds (maxlen, ragged stream ends) through the clamped staged parse
mkdir -p gpurun_out/r04au
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_record_index.py tests/test_long_messages.py tests/test_gpu_messages.py > gpurun_out/r04au/pytest.log 2>&1 || exit 1
