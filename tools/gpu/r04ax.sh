# round 4: walk-first encode window sizes, same box
mkdir -p gpurun_out/r04ax
VARIANTS="walk_first wf2k wf3k wf6k wf8k two_pass" REPS=30 timeout -k 10 300 python -u tools/tune/stream_ab.py recvar rpc > gpurun_out/r04ax/ab.log 2>&1 || exit 1
