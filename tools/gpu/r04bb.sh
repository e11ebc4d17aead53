# round 4: size pass with each record loaded into registers (generated plans)
mkdir -p gpurun_out/r04bb
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_stream_encode.py tests/test_codegen.py tests/test_containers.py > gpurun_out/r04bb/pytest.log 2>&1 || exit 1
VARIANTS="walk_first two_pass lb" REPS=30 timeout -k 10 300 python -u tools/tune/stream_ab.py recvar rpc > gpurun_out/r04bb/ab.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04bb/prof -o ab -- python3 -u tools/tune/stream_ab.py recvar rpc > gpurun_out/r04bb/ab_prof.log 2>&1 || exit 1
