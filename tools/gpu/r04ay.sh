# round 4: record index kernels of rpc / containertest under rocprofv3
mkdir -p gpurun_out/r04ay
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04ay/prof -o ix -- python3 -u tools/tune/ix_time.py rpc containertest > gpurun_out/r04ay/ix.log 2>&1 || exit 1
