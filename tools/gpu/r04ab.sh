# round 4: bench lines, walk-first record kernel (default) vs the per-window walk (enc_stream=0), one box
mkdir -p gpurun_out/r04ab
B="--steps 20 --warmup 5 --no-plain --no-cpu-baseline --no-large --no-cold --no-host-inclusive"
for s in recvar rpc; do
  timeout -k 10 300 python -u bench.py --schema $s $B > gpurun_out/r04ab/bench_${s}_default.json 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --schema $s $B --plan-opt enc_stream=0 > gpurun_out/r04ab/bench_${s}_enc0.json 2>&1 || exit 1
done
