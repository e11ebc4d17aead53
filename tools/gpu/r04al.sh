# round 4: register-walk encode without the native tile (vecrec, containertest): parity + timings
mkdir -p gpurun_out/r04al
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_containers.py tests/test_gpu_parity.py tests/test_gpu_messages.py tests/test_codegen.py tests/test_direct_mode.py > gpurun_out/r04al/pytest.log 2>&1 || exit 1
NOSTAMP=1 timeout -k 10 300 python -u tools/tune/enc_stamps.py run containertest vecrec > gpurun_out/r04al/times.log 2>&1 || exit 1
