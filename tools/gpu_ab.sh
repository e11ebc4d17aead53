# A/B of var kernels (bit-exact cross-check inside) + per-kernel rocprof stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/tune/ab_var.py recvar rpc && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab -o run --output-format csv -- python3 tools/tune/ab_var.py recvar rpc > gpurun_out/prof_ab.log 2>&1 && \
find gpurun_out/prof_ab -name "*kernel_stats.csv" -exec cp {} gpurun_out/ab_kernel_stats.csv \;
