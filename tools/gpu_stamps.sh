#!/bin/bash
# Phase stamps + per-kernel rocprof stats for the var-length kernels.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/tune/stamps_var.py recvar rpc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_var -o run -- python3 tools/tune/ab_var.py recvar rpc > gpurun_out/prof_var.log 2>&1
find gpurun_out/prof_var -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/var_kernel_stats.csv
