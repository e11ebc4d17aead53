# round 4: same-box A/B of the encode phase + rocprof kernel stats of the rpc/recvar benches
mkdir -p gpurun_out/r04x
timeout -k 10 200 python -u tools/tune/stream_ab.py recvar rpc > gpurun_out/r04x/ab.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for s in recvar rpc; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04x/prof_$s -o run -- python3 bench.py --schema $s --steps 20 --warmup 5 --no-plain --no-cpu-baseline > gpurun_out/r04x/bench_$s.json 2> gpurun_out/r04x/bench_$s.err || exit 1
done
