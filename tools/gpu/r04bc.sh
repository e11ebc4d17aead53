# round 4: recvar size pass, linear kernel vs the generated register-load walk
mkdir -p gpurun_out/r04bc
VARIANTS="walk_first wf_nolin two_pass two_pass_nolin" REPS=40 timeout -k 10 300 python -u tools/tune/stream_ab.py recvar > gpurun_out/r04bc/ab.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VARIANTS="walk_first wf_nolin" REPS=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04bc/prof -o ab -- python3 -u tools/tune/stream_ab.py recvar > gpurun_out/r04bc/ab_prof.log 2>&1 || exit 1
