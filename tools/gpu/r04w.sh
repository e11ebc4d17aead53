# round 4: full GPU suite + var bench lines with the walk-first record kernel default
mkdir -p gpurun_out/r04w
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04w/pytest.log 2>&1 || exit 1
for s in recvar rpc; do
  timeout -k 10 300 python -u bench.py --schema $s --steps 20 --warmup 5 > gpurun_out/r04w/bench_$s.json 2> gpurun_out/r04w/bench_$s.err || exit 1
done
