# round 4: record index, host-gated walk (1) vs asynchronous walk (2), same box
mkdir -p gpurun_out/r04be
for f in 1 2 1 2; do FAST=$f REPS=30 timeout -k 10 300 python -u tools/tune/ix_time.py rpc recvar containertest >> gpurun_out/r04be/ix_fast$f.log 2>&1 || exit 1; done
