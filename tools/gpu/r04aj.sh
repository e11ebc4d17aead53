# round 4: containertest/vecrec decode, share walk stopping early (new) vs full (old); parity
mkdir -p gpurun_out/r04aj
timeout -k 10 400 python -u -m pytest -x -q --timeout 90 --timeout-method thread -m gpu tests/test_containers.py tests/test_gpu_parity.py tests/test_gpu_messages.py -k "container or vecrec" > gpurun_out/r04aj/pytest.log 2>&1 || exit 1
for t in _old _new _old _new; do
  NOSTAMP=1 TAG=$t timeout -k 10 300 python -u tools/tune/enc_stamps.py run containertest vecrec >> gpurun_out/r04aj/ab$t.log 2>&1 || exit 1
done
