# round 4: window size of the walk-first record kernel
mkdir -p gpurun_out/r04aa
VARIANTS="two_pass walk_first wf2k wf3k wf6k wf8k" REPS=20 timeout -k 10 300 python -u tools/tune/stream_ab.py recvar rpc > gpurun_out/r04aa/ab.log 2>&1 || exit 1
