# round 4: sticky-failure staged parse (rlen_st) of the speculative index walk
mkdir -p gpurun_out/r04av
timeout -k 10 300 python -u tools/tune/ix_stamps.py run containertest rpc recvar > gpurun_out/r04av/ix_stamps.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_record_index.py tests/test_long_messages.py tests/test_gpu_messages.py > gpurun_out/r04av/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --schema rpc --steps 10 --warmup 3 --no-cpu-baseline --no-large --no-cold --no-host-inclusive > gpurun_out/r04av/bench_rpc.json 2> gpurun_out/r04av/bench.err || exit 1
timeout -k 10 300 python -u bench.py --schema containertest --steps 10 --warmup 3 --no-cpu-baseline --no-large --no-cold --no-host-inclusive > gpurun_out/r04av/bench_containertest.json 2>> gpurun_out/r04av/bench.err || exit 1
