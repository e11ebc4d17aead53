# round 4: record-index walk phase stamps (containertest, rpc, recvar)
mkdir -p gpurun_out/r04am
timeout -k 10 300 python -u tools/tune/ix_stamps.py run containertest rpc recvar > gpurun_out/r04am/ix_stamps.log 2>&1 || exit 1
