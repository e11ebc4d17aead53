# round 4: generated size walk by default for linear plans; full GPU suite, recvar/rpc bench lines
mkdir -p gpurun_out/r04bd
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04bd/pytest.log 2>&1 || exit 1
for s in recvar rpc; do timeout -k 10 300 python -u bench.py --schema $s --steps 20 --warmup 5 --no-cpu-baseline --no-large --no-cold --no-host-inclusive > gpurun_out/r04bd/bench_$s.json 2>> gpurun_out/r04bd/bench.err || exit 1; done
