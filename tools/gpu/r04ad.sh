# round 4: waves-per-SIMD bound of the walk-first record kernel (4/5/6), sized half timed alone
mkdir -p gpurun_out/r04ad
for w in 4 5 6 4 5 6; do
  NOSTAMP=1 TAG=_w$w timeout -k 10 200 python -u tools/tune/stream_stamps.py run recvar rpc >> gpurun_out/r04ad/w$w.log 2>&1 || exit 1
done
