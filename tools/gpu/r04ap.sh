# round 4: index-walk phase stamps after the second-word filter; rpc bench index ratio
mkdir -p gpurun_out/r04ap
timeout -k 10 300 python -u tools/tune/ix_stamps.py run containertest rpc recvar > gpurun_out/r04ap/ix_stamps.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --schema rpc --steps 10 --warmup 3 --no-cpu-baseline --no-large --no-cold --no-host-inclusive > gpurun_out/r04ap/bench_rpc.json 2> gpurun_out/r04ap/bench.err || exit 1
