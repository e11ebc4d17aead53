# round 4: per-lane guess-phase stamps of the speculative index walk
mkdir -p gpurun_out/r04ar
timeout -k 10 300 python -u tools/tune/ix_stamps.py run containertest rpc recvar > gpurun_out/r04ar/ix_stamps.log 2>&1 || exit 1
