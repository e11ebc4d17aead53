# round 4: look-back window per poll (4/16/32 blocks per lane), stamps + A/B
mkdir -p gpurun_out/r04t
for per in 4 16 32; do
  TAG=_p$per timeout -k 10 200 python -u tools/tune/stream_stamps.py run recvar rpc > gpurun_out/r04t/stamps_p$per.log 2>&1 || exit 1
done
timeout -k 10 200 python -u tools/tune/stream_ab.py recvar rpc > gpurun_out/r04t/ab.log 2>&1 || exit 1
