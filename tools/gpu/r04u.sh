# round 4: two-pass vs size pass + walk-first record kernel (halves), A/B + rocprof
mkdir -p gpurun_out/r04u
timeout -k 10 200 python -u tools/tune/stream_ab.py recvar rpc > gpurun_out/r04u/ab.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
VARIANTS="two_pass halves" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04u/prof -o run -- python3 tools/tune/stream_ab.py recvar rpc > gpurun_out/r04u/prof.log 2>&1 || exit 1
