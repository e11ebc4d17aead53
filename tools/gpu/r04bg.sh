# round 4: rpc / containertest index walk with and without the prefix test, same box (stamped builds)
mkdir -p gpurun_out/r04bg
for i in 1 2; do
  timeout -k 10 300 python -u tools/tune/ix_stamps.py run rpc containertest >> gpurun_out/r04bg/with_prefix.log 2>&1 || exit 1
  STAMPS_DIR=_stamps_ix_nopx timeout -k 10 300 python -u tools/tune/ix_stamps.py run rpc containertest >> gpurun_out/r04bg/no_prefix.log 2>&1 || exit 1
done
