# round 4: index walk without the prefix test (r04bg A/B: it cost more than it saved)
mkdir -p gpurun_out/r04bh
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_record_index.py tests/test_long_messages.py tests/test_gpu_messages.py tests/test_codegen.py > gpurun_out/r04bh/pytest.log 2>&1 || exit 1
REPS=30 timeout -k 10 300 python -u tools/tune/ix_time.py rpc recvar containertest > gpurun_out/r04bh/ix.log 2>&1 || exit 1
for s in rpc containertest; do timeout -k 10 300 python -u bench.py --schema $s --steps 10 --warmup 3 --no-cpu-baseline --no-large --no-cold --no-host-inclusive > gpurun_out/r04bh/bench_$s.json 2>> gpurun_out/r04bh/bench.err || exit 1; done
