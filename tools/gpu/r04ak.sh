# round 4: containertest decode stamps + bench line
mkdir -p gpurun_out/r04ak
timeout -k 10 300 python -u tools/tune/enc_stamps.py run containertest > gpurun_out/r04ak/stamps.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --schema containertest --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04ak/bench_containertest.json 2> gpurun_out/r04ak/bench.err || exit 1
